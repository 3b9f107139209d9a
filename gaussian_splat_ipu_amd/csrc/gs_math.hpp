// gs_math.hpp -- fp32 device math shared by the frame kernels (gs_kernels.hip)
// and the lattice emulator (gs_lattice.hip).  Internal to libgsplat.so; every
// function performs exactly the IEEE operations written (-ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsk {
namespace {

// --------------------------------------------------------------- math
// Shared expf specification (oracle/gs_oracle.cpp: or_expf): Cody-Waite
// reduction + degree-6 polynomial; fmaf is one fused op on both sides.
__device__ __forceinline__ float gs_expf(float x) {
  // branch-free: clamp into the finite range, evaluate, then select the
  // NaN / overflow / underflow results (same selects in the oracle)
  float xc = (x != x) ? 0.0f : x;
  xc = (xc < -104.0f) ? -104.0f : xc;
  xc = (xc > 89.0f) ? 89.0f : xc;
  const float k = __builtin_rintf(xc * 1.44269502162933349609f);
  float r = __builtin_fmaf(k, -0.693145751953125f, xc);
  r = __builtin_fmaf(k, -1.428606765330187045e-06f, r);
  float p = 1.9875691500e-4f;
  p = __builtin_fmaf(p, r, 1.3981999507e-3f);
  p = __builtin_fmaf(p, r, 8.3334519073e-3f);
  p = __builtin_fmaf(p, r, 4.1665795894e-2f);
  p = __builtin_fmaf(p, r, 1.6666665459e-1f);
  p = __builtin_fmaf(p, r, 5.0000001201e-1f);
  const float r2 = r * r;
  p = __builtin_fmaf(p, r2, r);
  p = p + 1.0f;
  int ki = (int)k;
  const bool lo = ki < -125;
  p = lo ? p * 5.42101086242752217004e-20f : p;  // 2^-64
  ki = lo ? ki + 64 : ki;
  const bool hi = ki > 127;
  p = hi ? p * 2.0f : p;
  ki = hi ? ki - 1 : ki;
  float res = p * __uint_as_float((uint32_t)(ki + 127) << 23);
  res = (x < -103.972084045410f) ? 0.0f : res;
  res = (x > 88.72283935546875f) ? __builtin_huge_valf() : res;
  return (x != x) ? x : res;
}

// Wave ballot of a bool.  HIP's __ballot(int) turns the bool into 0 / 1 in a
// VGPR and compares it again; the builtin takes the lane mask as is.
__device__ __forceinline__ unsigned long long ballot64(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ float smax(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float smin(float a, float b) { return a < b ? a : b; }

struct M3 {
  float m[3][3];  // glm column-major: m[c][r]
};

// glm mat3 * mat3: (A[0][r]*B[c][0] + A[1][r]*B[c][1]) + A[2][r]*B[c][2]
__device__ __forceinline__ M3 m3_mul(const M3& A, const M3& B) {
  M3 R;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      float s = A.m[0][r] * B.m[c][0];
      s = s + A.m[1][r] * B.m[c][1];
      s = s + A.m[2][r] * B.m[c][2];
      R.m[c][r] = s;
    }
  return R;
}

__device__ __forceinline__ M3 m3_t(const M3& A) {
  M3 R;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) R.m[c][r] = A.m[r][c];
  return R;
}

// glm mat4 * vec4 row r: (m0*x + m1*y) + (m2*z + m3*w)
__device__ __forceinline__ float mv_row(const float* m, int r, float x, float y, float z, float w) {
  const float a = m[0 * 4 + r] * x + m[1 * 4 + r] * y;
  const float b = m[2 * 4 + r] * z + m[3 * 4 + r] * w;
  return a + b;
}

// Gaussian3D::ComputeCov3D (ipu_geometry.hpp:315-323) with scale already
// divided by fxy[1] (codelets.cpp:463).
__device__ __forceinline__ M3 cov3d(float4 q4, float sx, float sy, float sz) {
  const float qw = q4.x, qx = q4.y, qy = q4.z, qz = q4.w;  // glm::quat(w, x, y, z)
  const float dot = (qw * qw + qx * qx) + (qy * qy + qz * qz);
  const float len = __builtin_sqrtf(dot);
  float w, x, y, z;
  if (len <= 0.0f) {
    w = 1.0f; x = 0.0f; y = 0.0f; z = 0.0f;
  } else {
    const float inv = 1.0f / len;
    w = qw * inv; x = qx * inv; y = qy * inv; z = qz * inv;
  }
  const float qxx = x * x, qyy = y * y, qzz = z * z;
  const float qxz = x * z, qxy = x * y, qyz = y * z;
  const float qwx = w * x, qwy = w * y, qwz = w * z;
  M3 R;
  R.m[0][0] = 1.0f - 2.0f * (qyy + qzz);
  R.m[0][1] = 2.0f * (qxy + qwz);
  R.m[0][2] = 2.0f * (qxz - qwy);
  R.m[1][0] = 2.0f * (qxy - qwz);
  R.m[1][1] = 1.0f - 2.0f * (qxx + qzz);
  R.m[1][2] = 2.0f * (qyz + qwx);
  R.m[2][0] = 2.0f * (qxz + qwy);
  R.m[2][1] = 2.0f * (qyz - qwx);
  R.m[2][2] = 1.0f - 2.0f * (qxx + qyy);
  M3 S;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) S.m[c][r] = 0.0f;
  S.m[0][0] = gs_expf(sx);
  S.m[1][1] = gs_expf(sy);
  S.m[2][2] = gs_expf(sz);
  return m3_mul(m3_mul(m3_mul(R, S), m3_t(S)), m3_t(R));
}


// ------------------------------------------------------ streaming access
// Non-temporal loads / stores (the `nt` bit) for bytes a frame touches once:
// the projection's scene reads and the blend's RGBA f32 pixels.  They leave
// the L2s and the Infinity Cache to what the frames in flight re-read (the
// records, lists and pairs).  Interleaved on one box against the plain
// loads/stores: config 3 8 624 -> 8 833 frames/s (the projection alone 22.6
// -> 25 us, slower by itself), config 5 1 535 -> 1 556 (its HBM-bound
// projection 150 -> 135 us), 8 bands of config 4 unchanged (35.8 / 35.3 us;
// their scene reads stay plain).  Not the BGR8 bytes: streaming
// byte stores lose the L2's write combining (blend 74 -> 92 us).  Nor the
// intermediates' last reads (the count's and emit's rectangles, the sort's
// pairs): config 3 +0.7 %, config 5 -1 %.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 load_stream(const float4* p) {
  const f32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float load_stream(const float* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void store_stream(float4* p, float4 v) {
  const f32x4_t w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<f32x4_t*>(p));
}

// ------------------------------------------------------------- BGR8 pack
__device__ __forceinline__ uint8_t to_u8(float v) {
  // cv::min(v * 255, 255) -> convertTo(CV_8U): round half to even, saturate
  float x = v * 255.0f;
  x = (255.0f < x) ? 255.0f : x;
  if (x != x) return 0;
  const float r = __builtin_rintf(x);
  if (r < 0.0f) return 0;
  if (r > 255.0f) return 255;
  return (uint8_t)r;
}

}  // namespace
}  // namespace gsk
