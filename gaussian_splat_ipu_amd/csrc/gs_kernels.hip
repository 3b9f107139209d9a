// gs_kernels.hip -- the frame path as hand-written HIP for gfx950 (MI355X).
//
//   project  one thread per Gaussian: MVP transform, clip-space EWA covariance,
//            eigenvalue radius, guard band + z cull, conic, alpha footprint
//            (pcut + integer pixel box), tile rectangle and its alpha-box cut;
//            V per 256-Gaussian block (no single-address atomics)
//            reference: codelets.cpp:437-499, ipu_geometry.hpp:247-383
//   bin      chunked LDS binning: count (one 1024-thread workgroup per chunk of
//            Gaussians keeps the chunk's per-tile histogram in LDS; runs of
//            equal rectangles add once), colscan (per tile, exclusive scan over
//            the chunks), scan_multi (tile starts, sort queues, frame counters
//            straight into mapped host memory), emit (LDS cursors per tile)
//            -- the converged lattice of codelets.cpp:194-293, 507-602 in one
//            frame; global-atomic fallback kernels for huge tile grids
//   sort     one launch for all lists, longest first: register bitonic
//            networks (DPP / permlane) for <= 256 keys, register runs + LDS
//            merge path for <= 2048, and a sample sort over many workgroups
//            (lazy: only each big list's nearest keys before the blend)
//            reference: codelets.cpp:295-356 (per-tile quicksort by clip z)
//   blend    one wave per 8x8 pixel block of a tile: batches of 64 records
//            staged in LDS, one 64-bit record mask per pixel from column / row
//            ballots, a per-lane walk of the mask (one record per step) with
//            the reference's early exit; RGBA f32 + BGR8 stores fused
//            reference: codelets.cpp:358-421, ipu_rasteriser.cpp:131-144
//
// Arithmetic: fp32 everywhere, compiled with -ffp-contract=off and the default
// correctly rounded divide / sqrt, so every expression below performs exactly
// the IEEE operations written (and matches the CPU oracle bit for bit).
#include <algorithm>
#include <vector>

#include "gs_kernels.hpp"
#include "gs_math.hpp"

// blend: 1 = one record mask per pixel (blend 82 -> 78 us), 0 = per 2x2 quad
// blend: waves per workgroup (the waves are independent)
#ifndef GS_BLEND_WPG
#define GS_BLEND_WPG 4
#endif
// sort: register bitonic networks with E <= this many keys per lane fully
// unrolled (compile-time stages: sort 42.8 -> 29.6 us against rolled loops)
#ifndef GS_SORT_UNROLL_E
#define GS_SORT_UNROLL_E 4
#endif
// two-pixel blend: waves per workgroup (2 = one tile, 4 = two tiles)
#ifndef GS_PX2_WPG
#define GS_PX2_WPG 4
#endif
// the one-pixel blend kernels' fewest waves per SIMD (8: at most 64 VGPRs)
#ifndef GS_BLEND_WPE
#define GS_BLEND_WPE 8
#endif

namespace gsk {
namespace {

__device__ __forceinline__ uint32_t depth_key_of(float z) {
  // order-preserving: ascending float z <-> ascending key (z < 0 here)
  const uint32_t b = __float_as_uint(z);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

constexpr uint2 kEmptyRect = {1u, 1u};  // tx0 = 1 > tx1 = 0

// the alpha box of record g (the z, w of the second float4 of its 32-B record)
__device__ __forceinline__ uint2 rec_box(const FrameParams& fp, const Buffers& b, uint32_t g) {
  return reinterpret_cast<const uint2*>(b.rec)[(2ull * g + 1ull) * 2ull + 1ull];
}

// FrameParams::rect8: a rectangle's four tile bounds, 8 bits each
__device__ __forceinline__ uint32_t rect8_pack(uint2 r) {
  return (r.x & 0xFFu) | ((r.x >> 16) & 0xFFu) << 8 | (r.y & 0xFFu) << 16 | (r.y >> 16) << 24;
}
__device__ __forceinline__ uint2 rect8_unpack(uint32_t v) {
  return make_uint2((v & 0xFFu) | ((v >> 8) & 0xFFu) << 16, ((v >> 16) & 0xFFu) | (v >> 24) << 16);
}
// the rectangles of Gaussian i as the projection stored them
__device__ __forceinline__ void store_rects(const FrameParams& fp, const Buffers& b, int i, uint2 rect, uint2 crect) {
  if (fp.rect8) {
    reinterpret_cast<uint32_t*>(b.rect)[i] = rect8_pack(rect);
    reinterpret_cast<uint32_t*>(b.crect)[i] = rect8_pack(crect);
  } else {
    b.rect[i] = rect;
    if (fp.pair_cull) b.crect[i] = crect;
  }
}
constexpr uint32_t kEmptyBox = 0x80007FFFu;  // lo = +32767 > hi = -32768
constexpr uint32_t kFullBox = 0x7FFF8000u;   // lo = -32768, hi = +32767

__device__ __forceinline__ uint32_t pack_i16x2(float lo, float hi) {
  lo = fmaxf(-32768.0f, fminf(32767.0f, lo));
  hi = fmaxf(-32768.0f, fminf(32767.0f, hi));
  return ((uint32_t)(int)lo & 0xFFFFu) | ((uint32_t)(int)hi << 16);
}

// Conservative alpha footprint of one 2D Gaussian, used to skip work that
// cannot change a pixel ("blend culling"):
//   pcut: a lane with power < pcut has op * expf(power) < 1/255, i.e. the
//         reference would `continue` (codelets.cpp:401-403);
//   box:  integer pixel box (x0,x1 | y0,y1) outside of which every pixel has
//         power < pcut (the bounding box of the ellipse { d^T Q d <= -2 pcut }
//         of the conic Q, widened to cover its own fp32 rounding; pixel
//         centres are the integer coordinates the blend evaluates).
// Both only ever remove evaluations whose outcome is "skip", so the blended
// result is bit-identical to evaluating every list entry.  fp32 throughout,
// each rounding covered by an explicit margin (the bounds are in DESIGN.md).
__device__ __forceinline__ void alpha_footprint(float mx, float my, float k0, float k1, float k2,
                                                float op, const FrameParams& fp, float& pcut,
                                                uint32_t& box_x, uint32_t& box_y) {
  pcut = -__builtin_huge_valf();  // no per-lane cut
  box_x = kFullBox;
  box_y = kFullBox;
  const bool nice = __builtin_fabsf(k0) < 1e30f && __builtin_fabsf(k1) < 1e30f &&
                    __builtin_fabsf(k2) < 1e30f && __builtin_fabsf(mx) < 1e30f &&
                    __builtin_fabsf(my) < 1e30f && fp.width <= 32767 && fp.height <= 32767;
  if (!nice || op != op) return;  // NaN opacity: alpha = min(0.99, NaN) = 0.99, never skipped
  if (op < 1.0f / 255.0f) {       // alpha <= op < 1/255 for every pixel: always skipped
    pcut = __builtin_huge_valf();
    box_x = kEmptyBox;
    box_y = kEmptyBox;
    return;
  }
  // pc = ln(1 / (255 op)) - 0.05 (power below it: alpha < 0.96 / 255), pushed
  // down by far more than the error of v_log_f32 and the product 255 * op
  const float ln = __builtin_amdgcn_logf(255.0f * op) * 0.693147182f;  // >= 0
  if (!(ln < 1e30f)) return;                                          // op = +inf
  const float pc = -ln - 0.05f;
  pcut = pc - (ln * 1e-5f + 1e-5f);
  const float a = k0, b = k1, c = k2;
  const float det = __builtin_fmaf(a, c, -(b * b));  // relative error < 6e-5 when kept
  // Well-conditioned conics only (1 - rho^2 > 1e-3): then the fp32 rounding of
  // the reference's power expression is < 7.2e-4 relative.  A pixel outside
  // the box has |d| > 1.00096 x the ellipse's extent (1.001 minus the < 4e-5
  // error of ex), so d^T Q d > 1.0019 R and its fp32 power < 1.0011 pcut < pcut.
  if (a > 0.0f && c > 0.0f && det > 1e-3f * a * c) {
    const float R = -2.0f * pcut;
    const float ex = __builtin_sqrtf(R * c / det) * 1.001f;
    const float ey = __builtin_sqrtf(R * a / det) * 1.001f;
    // slack for the rounding of m -/+ e (< 2^-24 of their magnitude)
    const float sx = (__builtin_fabsf(mx) + ex) * 4.8e-7f + 1e-6f;
    const float sy = (__builtin_fabsf(my) + ey) * 4.8e-7f + 1e-6f;
    box_x = pack_i16x2(__builtin_ceilf(mx - ex - sx), __builtin_floorf(mx + ex + sx));
    box_y = pack_i16x2(__builtin_ceilf(my - ey - sy), __builtin_floorf(my + ey + sy));
  }
}

// ------------------------------------------------------------------ project
// x / d.  P2: d is a power of two (FrameParams::pow2), so x * (1 / d) is the
// same correctly rounded value (scaling by 2^k is exact; both round the same
// real number), and a non-negative int divided by 2^k is a shift.
template <bool P2>
__device__ __forceinline__ float div_p2(float x, float d, float inv_d) {
  return P2 ? x * inv_d : x / d;
}
template <bool P2>
__device__ __forceinline__ int idiv_p2(int x, int d, int sh) {  // x >= 0
  return P2 ? x >> sh : x / d;
}
// The band rows [yb0, yb1] (band-local) among absolute tile rows [fy0, fy1]
// (clamped to the frame); empty when yb0 > yb1.
template <bool P2>
__device__ __forceinline__ void band_rows_of(const FrameParams& fp, float fy0, float fy1, int& yb0,
                                             int& yb1) {
  const float gy1 = (float)(fp.tiles_y - 1);
  if (fy0 < 0.0f) fy0 = 0.0f;
  if (fy1 > gy1) fy1 = gy1;
  yb0 = 0;
  yb1 = -1;
  if (fy0 <= fy1) {
    const int a0 = (int)fy0 - fp.band_ty0, a1 = (int)fy1 - fp.band_ty0, S = fp.band_stride;
    // P2: S = 2^sh_stride, and both numerators are >= 0 here
    yb0 = a0 <= 0 ? 0 : (P2 ? (a0 + S - 1) >> fp.sh_stride : (a0 + S - 1) / S);
    yb1 = a1 < 0 ? -1 : min(P2 ? a1 >> fp.sh_stride : a1 / S, fp.band_nrows - 1);
  }
}

// GS_FLAG_BAND_CULL: true when a Gaussian provably has no tile row in this
// band, from an upper bound on its eigen radius that needs only the mean, the
// scales and T (the clip-space Jacobian product of ComputeCov2D, computed by
// the same code as the full projection).  With C the 3D covariance and
// a = cov00 + 0.3, c = cov11 + 0.3, b = cov01 (b^2 <= (a - .3)(c - .3) < ac,
// the 2x2 block of a PSD matrix), mid^2 - det = (a - c)^2 / 4 + b^2 < mid^2, so
//   radius = ceil(3 sqrt(l1)),  l1 = mid + sqrt(max(0.1, mid^2 - det))
//                                  <= a + c + 0.32 = cov00 + cov11 + 0.92,
//   cov00 + cov11 <= trace(T^T C T) <= lambda_max(C) ||T||_F^2,
//   lambda_max(C) = max_i exp(s_i / fxy[1])^2   (R orthonormal).
// (Rounds 2-5 carried a further factor 2 on lambda_max ||T||_F^2: the same
// test, looser.)
// The bound is inflated by 5 % + 2 px against fp32 rounding, and the tile-row
// range is computed with the rectangle's own (monotone) formulas from the same
// vy, so it contains the true rows.  Non-finite values never cull.
template <bool P2>
__device__ __forceinline__ bool band_culled(const FrameParams& fp, float vy, const M3& T, float4 sg,
                                            float extra = 0.0f) {
  float t2 = 0.0f;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) t2 += T.m[c][r] * T.m[c][r];
  const float smax = div_p2<P2>(fmaxf(fmaxf(sg.x, sg.y), sg.z), fp.scale_div, fp.inv_sd);
  const float lc = __expf(2.0f * smax) * 1.01f;
  const float r = 3.0f * __builtin_sqrtf(1.05f * (lc * t2) + 1.0f) + 2.0f + extra;
  if (!(__builtin_fabsf(vy) < 1e30f) || !(r < 1e30f)) return false;
  const float fy0 = __builtin_floorf(div_p2<P2>(__builtin_floorf(vy - r), fp.th, fp.inv_th));
  const float fy1 = __builtin_floorf(div_p2<P2>(__builtin_ceilf(vy + r), fp.th, fp.inv_th));
  int yb0, yb1;
  band_rows_of<P2>(fp, fy0, fy1, yb0, yb1);
  return yb0 > yb1;
}

// The band cull's first, cheap pass: the same bound as band_culled, from vy
// and T computed with v_rcp instead of correctly rounded divisions (each
// quotient within ~1 ulp; the bound's 5 % inflation covers T, and vy gets
// 1e-5 |vy| + 0.05 px more).  Only a Gaussian this pass proves outside the
// band is skipped; the exact test in project_one still runs for the rest.
// From the band cull's 16-B record (gs_renderer.hip: the mean with w = 1 and
// the largest log-scale; NaN for an empty slot, +inf for a mean with w != 1,
// neither of which is culled): the same test as band_culled with the mean and
// the scales, bit for bit.
template <bool P2>
__device__ __forceinline__ bool band_culled_fast(const FrameParams& fp, float4 cr) {
  const float* m = fp.mvp;
  const float4 mean = make_float4(cr.x, cr.y, cr.z, 1.0f);
  const float4 sg = make_float4(cr.w, cr.w, cr.w, 1.0f);
  const float cy = mv_row(m, 1, mean.x, mean.y, mean.z, mean.w);
  const float cw = mv_row(m, 3, mean.x, mean.y, mean.z, mean.w);
  const float vy = (cy * (0.5f * __builtin_amdgcn_rcpf(cw)) + 0.5f) * fp.H;
  const float tx = mv_row(m, 0, mean.x, mean.y, mean.z, 1.0f);
  const float ty = mv_row(m, 1, mean.x, mean.y, mean.z, 1.0f);
  const float tz = mv_row(m, 2, mean.x, mean.y, mean.z, 1.0f);
  const float itz = __builtin_amdgcn_rcpf(tz);
  const float lim = 1.3f * fp.tanfov;
  const float ctx = fminf(lim, fmaxf(-lim, tx * itz)) * tz;
  const float cty = fminf(lim, fmaxf(-lim, ty * itz)) * tz;
  M3 J;
  J.m[0][0] = fp.focal_x * itz;
  J.m[0][1] = 0.0f;
  J.m[0][2] = -(fp.focal_x * ctx) * (itz * itz);
  J.m[1][0] = 0.0f;
  J.m[1][1] = fp.focal_y * itz;
  J.m[1][2] = -(fp.focal_y * cty) * (itz * itz);
  J.m[2][0] = 0.0f;
  J.m[2][1] = 0.0f;
  J.m[2][2] = 0.0f;
  M3 W;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) W.m[c][r] = m[c * 4 + r];
  return band_culled<P2>(fp, vy, m3_mul(W, J), sg, 1e-5f * __builtin_fabsf(vy) + 0.05f);
}

// gs_set_sh (opt-in, not in the reference: its loader reads
// f_dc only, file_io.cpp:66-68): the view-dependent colour of the 3DGS
// convention (degree <= 3) for the direction from the camera to the mean.
// The scene's frame has z negated against the PLY's (splat.cpp:93-100), so
// the direction's z is negated back before the basis is evaluated.  Every
// operation is written out in the order oracle/gs_oracle.cpp
// (or_sh_colours) restates; degree 0 is the scene preparation's own colour,
// max(0.28209479 f_dc + 0.5, 0) (splat.cpp:136-147, gs_scene.cpp), bit for bit.
__device__ __forceinline__ float sh_coef(const Buffers& b, int n, int k, int c, int i) {
  return b.sh[((size_t)(k * 3 + c)) * (size_t)n + (size_t)i];
}

__device__ __forceinline__ void sh_colour(const FrameParams& fp, const Buffers& b, int i, float4 mean, float4& col) {
  const float ddx = mean.x - fp.campos[0], ddy = mean.y - fp.campos[1], ddz = mean.z - fp.campos[2];
  const float len = __builtin_sqrtf((ddx * ddx + ddy * ddy) + ddz * ddz);
  const float x = ddx / len, y = ddy / len, z = -ddz / len;
  const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
  float out[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float r = 0.28209479177387814f * sh_coef(b, fp.n, 0, c, i);
    if (fp.sh_degree > 0) {
      r = r - (0.4886025119029199f * y) * sh_coef(b, fp.n, 1, c, i);
      r = r + (0.4886025119029199f * z) * sh_coef(b, fp.n, 2, c, i);
      r = r - (0.4886025119029199f * x) * sh_coef(b, fp.n, 3, c, i);
      if (fp.sh_degree > 1) {
        r = r + (1.0925484305920792f * xy) * sh_coef(b, fp.n, 4, c, i);
        r = r + (-1.0925484305920792f * yz) * sh_coef(b, fp.n, 5, c, i);
        r = r + (0.31539156525252005f * ((2.0f * zz - xx) - yy)) * sh_coef(b, fp.n, 6, c, i);
        r = r + (-1.0925484305920792f * xz) * sh_coef(b, fp.n, 7, c, i);
        r = r + (0.5462742152960396f * (xx - yy)) * sh_coef(b, fp.n, 8, c, i);
        if (fp.sh_degree > 2) {
          r = r + ((-0.5900435899266435f * y) * (3.0f * xx - yy)) * sh_coef(b, fp.n, 9, c, i);
          r = r + ((2.890611442640554f * xy) * z) * sh_coef(b, fp.n, 10, c, i);
          r = r + ((-0.4570457994644658f * y) * ((4.0f * zz - xx) - yy)) * sh_coef(b, fp.n, 11, c, i);
          r = r + ((0.3731763325901154f * z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy)) * sh_coef(b, fp.n, 12, c, i);
          r = r + ((-0.4570457994644658f * x) * ((4.0f * zz - xx) - yy)) * sh_coef(b, fp.n, 13, c, i);
          r = r + ((1.445305721320277f * z) * (xx - yy)) * sh_coef(b, fp.n, 14, c, i);
          r = r + ((-0.5900435899266435f * x) * (xx - 3.0f * yy)) * sh_coef(b, fp.n, 15, c, i);
        }
      }
    }
    r = r + 0.5f;
    out[c] = (r < 0.0f) ? 0.0f : r;  // glm::max(colour, vec3(0)) as the scene preparation
  }
  col.x = out[0];
  col.y = out[1];
  col.z = out[2];
}

template <bool P2>
__device__ __forceinline__ bool project_one(const FrameParams& fp, const Buffers& b, int i, uint2& rect_out,
                                            uint2& crect_out, float4* stage = nullptr, uint32_t* dkey_out = nullptr) {
  bool rendered = false;
  // mean_w1: the mean's w is 1 and the colour's rgb is not needed (the blend
  // reads it from the scene): one 16-B load of xyz + opacity instead of 32 B
  float4 mean, col = make_float4(0.f, 0.f, 0.f, 0.f), rot = col;
  if (fp.mean_w1) {
    // (streamed on whole frames; a row band's frame moves so few other bytes
    // that the scene stays in the Infinity Cache between frames: 8 bands of
    // config 4 35.7 -> 36.5 us per frame with streaming loads)
    const float4 mo = fp.band_cull ? b.mean_op[i] : load_stream(b.mean_op + i);
    mean = make_float4(mo.x, mo.y, mo.z, 1.0f);
    col.w = mo.w;
  } else {
    mean = b.mean[i];
  }
  // FrameParams::cov_cache: the 3D covariance (and the gid) from the scene's
  // cache instead of the rotation and the scales (the band cull still reads
  // the scales, for its bound)
  const size_t nn = (size_t)fp.n;
  float4 sg;
  float c3[9];
  if (fp.cov_cache && !fp.band_cull) {
    sg = make_float4(0.f, 0.f, 0.f, 1.0f);  // (liveness: the sign of Sigma[2][2], below)
  } else {
    sg = b.scale_gid[i];
  }
  // without the band cull every live Gaussian needs its colour and rotation
  // (or covariance): load them with the mean (one memory round trip)
  if (!fp.band_cull) {
    if (!fp.mean_w1) col = b.colour[i];  // (its w is the opacity, as mean_op's)
    if (fp.cov_cache) {
#pragma unroll
      for (int k = 0; k < 9; ++k) c3[k] = load_stream(b.cov3 + k * nn + i);
      if (c3[8] < 0.0f) sg.w = 0.0f;
    } else {
      rot = b.rot[i];
    }
  }
  // the record: 32 B per Gaussian (48 B with the colour for the readback)
  float4* rec = b.rec + (fp.full_record ? 3 : 2) * (size_t)i;
  uint2 rect = kEmptyRect, crect = kEmptyRect;
  uint32_t dkey = 0xFFFFFFFFu;
  if (!(sg.w <= 0.0f)) {  // codelets.cpp:456: if (g.gid <= 0) continue;
    const float* m = fp.mvp;
    // clip = mvp * mean (codelets.cpp:460)
    const float cx = mv_row(m, 0, mean.x, mean.y, mean.z, mean.w);
    const float cy = mv_row(m, 1, mean.x, mean.y, mean.z, mean.w);
    const float cz = mv_row(m, 2, mean.x, mean.y, mean.z, mean.w);
    const float cw = mv_row(m, 3, mean.x, mean.y, mean.z, mean.w);
    // Viewport::clipSpaceToViewport (viewport.hpp:21-35)
    const float s = 0.5f / cw;
    float vx = cx * s, vy = cy * s;
    vx = vx + 0.5f;
    vy = vy + 0.5f;
    vx = vx * fp.W;
    vy = vy * fp.H;
    vx = vx + 0.0f;
    vy = vy + 0.0f;
    // ComputeCov2D (ipu_geometry.hpp:333-383): t = mv * (mean.xyz, 1)
    float tx = mv_row(m, 0, mean.x, mean.y, mean.z, 1.0f);
    float ty = mv_row(m, 1, mean.x, mean.y, mean.z, 1.0f);
    const float tz = mv_row(m, 2, mean.x, mean.y, mean.z, 1.0f);
    const float limx = 1.3f * fp.tanfov;
    const float limy = 1.3f * fp.tanfov;
    const float txtz = tx / tz;
    const float tytz = ty / tz;
    tx = smin(limx, smax(-limx, txtz)) * tz;
    ty = smin(limy, smax(-limy, tytz)) * tz;
    M3 J;
    J.m[0][0] = fp.focal_x / tz;
    J.m[0][1] = 0.0f;
    J.m[0][2] = -(fp.focal_x * tx) / (tz * tz);
    J.m[1][0] = 0.0f;
    J.m[1][1] = fp.focal_y / tz;
    J.m[1][2] = -(fp.focal_y * ty) / (tz * tz);
    J.m[2][0] = 0.0f;
    J.m[2][1] = 0.0f;
    J.m[2][2] = 0.0f;
    M3 W;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r < 3; ++r) W.m[c][r] = m[c * 4 + r];
    const M3 T = m3_mul(W, J);
    if (fp.band_cull && band_culled<P2>(fp, vy, T, sg)) {
      // no tile row in this band: empty rectangle; the record is never read
      store_rects(fp, b, i, rect, crect);
      b.depth_key[i] = dkey;
      rect_out = rect;
      crect_out = crect;
      return false;
    }
    if (fp.band_cull) {
      if (!fp.mean_w1) col = b.colour[i];  // (its w is the opacity, as mean_op's)
      if (fp.cov_cache) {
#pragma unroll
        for (int k = 0; k < 9; ++k) c3[k] = b.cov3[k * nn + i];
      } else {
        rot = b.rot[i];
      }
    }
    if (fp.sh_degree >= 0 && b.sh) sh_colour(fp, b, i, mean, col);
    M3 C3;
    if (fp.cov_cache) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) C3.m[c][r] = c3[c * 3 + r];
    } else {
      C3 = cov3d(rot, div_p2<P2>(sg.x, fp.scale_div, fp.inv_sd), div_p2<P2>(sg.y, fp.scale_div, fp.inv_sd),
                 div_p2<P2>(sg.z, fp.scale_div, fp.inv_sd));
    }
    M3 cov = m3_mul(m3_mul(m3_t(T), m3_t(C3)), T);
    const float a = cov.m[0][0] + 0.3f;
    const float bb = cov.m[0][1];
    const float c = cov.m[1][1] + 0.3f;
    // ComputeEigenvalues / GetBoundingBox (ipu_geometry.hpp:247-276)
    const float det = a * c - bb * bb;
    const float mid = 0.5f * (a + c);
    const float l1 = mid + __builtin_sqrtf(smax(0.1f, mid * mid - det));
    const float l2 = mid - __builtin_sqrtf(smax(0.1f, mid * mid - det));
    const float radius = __builtin_ceilf(3.0f * __builtin_sqrtf(smax(l1, l2)));
    const float minx = vx - radius, miny = vy - radius;
    const float maxx = vx + radius, maxy = vy + radius;
    const float ddx = maxx - minx, ddy = maxy - miny;
    const bool within = __builtin_sqrtf(ddx * ddx + ddy * ddy) < fp.guard_thr;
    // ComputeConicOpacity (ipu_geometry.hpp:278-286)
    float k0 = 0.0f, k1 = 0.0f, k2 = 0.0f, k3 = 0.0f;
    const float cdet = a * c - bb * bb;
    if (!(cdet == 0.0f)) {
      const float inv = 1.0f / cdet;
      k0 = c * inv;
      k1 = -bb * inv;
      k2 = a * inv;
      k3 = col.w;
    }
    float pcut;
    uint32_t b01, b23;
    alpha_footprint(vx, vy, k0, k1, k2, k3, fp, pcut, b01, b23);
    const float4 rec0 = make_float4(vx, vy, k0, k2);
    if (fp.full_record) b.rec_tail[i] = make_float2(radius, cz);  // readback only
    if (within && cz < 0.0f) {  // codelets.cpp:493
      rendered = true;
      dkey = depth_key_of(cz);
      // converged lattice rectangle
      float fx0 = __builtin_floorf(div_p2<P2>(__builtin_floorf(minx), fp.tw, fp.inv_tw));
      float fx1 = __builtin_floorf(div_p2<P2>(__builtin_ceilf(maxx), fp.tw, fp.inv_tw));
      float fy0 = __builtin_floorf(div_p2<P2>(__builtin_floorf(miny), fp.th, fp.inv_th));
      float fy1 = __builtin_floorf(div_p2<P2>(__builtin_ceilf(maxy), fp.th, fp.inv_th));
      const float gx1 = (float)(fp.tiles_x - 1);
      if (fx0 < 0.0f) fx0 = 0.0f;
      if (fx1 > gx1) fx1 = gx1;
      // this band's rows among the absolute rows [fy0, fy1]
      int yb0, yb1;
      band_rows_of<P2>(fp, fy0, fy1, yb0, yb1);
      if (fx0 <= fx1 && yb0 <= yb1) {
        const uint32_t x0 = (uint32_t)(int)fx0, x1 = (uint32_t)(int)fx1;
        const uint32_t y0 = (uint32_t)yb0, y1 = (uint32_t)yb1;
        rect = make_uint2(x0 | (x1 << 16), y0 | (y1 << 16));
        if (fp.pair_cull) {
          // the tiles whose pixels the alpha box meets: a tile outside it has
          // no pixel where the Gaussian passes alpha >= 1/255 (blend culling),
          // so leaving it out of that tile's list changes no pixel
          const int bx0 = (int)(b01 << 16) >> 16, bx1 = (int)b01 >> 16;
          const int by0 = (int)(b23 << 16) >> 16, by1 = (int)b23 >> 16;
          const int cx0 = max((int)x0, idiv_p2<P2>(max(bx0, 0), fp.tile_w, fp.sh_tw));
          const int cx1 = min((int)x1, bx1 < 0 ? -1 : idiv_p2<P2>(bx1, fp.tile_w, fp.sh_tw));
          const float gy0 = smax(fy0, (float)idiv_p2<P2>(max(by0, 0), fp.tile_h, fp.sh_th));
          const float gy1 = smin(fy1, by1 < 0 ? -1.0f : (float)idiv_p2<P2>(by1, fp.tile_h, fp.sh_th));
          int cy0, cy1;
          band_rows_of<P2>(fp, gy0, gy1, cy0, cy1);
          crect = (cx0 <= cx1 && cy0 <= cy1 && bx0 <= bx1 && by0 <= by1)
                      ? make_uint2((uint32_t)cx0 | ((uint32_t)cx1 << 16),
                                   (uint32_t)cy0 | ((uint32_t)cy1 << 16))
                      : kEmptyRect;
        }
        if (fp.bin_global)  // fallback binning: per-tile lengths by global atomics
          for (uint32_t y = y0; y <= y1; ++y)
            for (uint32_t x = x0; x <= x1; ++x) atomicAdd(&b.tile_count[y * fp.tiles_x + x], 1u);
      }
    }
    // the blend reads the records of binned Gaussians only: the others'
    // 48 B stay unwritten (off-screen, culled, outside the band, or no tile
    // met by the alpha box); the readback pass writes every record
    // The blend takes the colour and opacity from the scene (or, with SH, from
    // col_out): a record with an empty alpha box (k3 = 0 when the conic's
    // determinant is 0, or opacity < 1/255) is never composited, so its
    // opacity never matters, and otherwise k3 == col.w
    const uint2 binned = fp.pair_cull ? crect : rect;
    if (fp.full_record) {
      rec[0] = rec0;
      rec[1] = make_float4(k1, pcut, col.x, col.y);
      rec[2] = make_float4(col.z, k3, __uint_as_float(b01), __uint_as_float(b23));
    } else if (stage) {  // (project_block stores the wave's records as whole lines)
      stage[0] = rec0;
      stage[1] = make_float4(k1, pcut, __uint_as_float(b01), __uint_as_float(b23));
      if (fp.sh_degree >= 0 && b.sh) b.col_out[i] = col;
    } else if ((binned.x & 0xFFFFu) <= (binned.x >> 16)) {
      rec[0] = rec0;
      rec[1] = make_float4(k1, pcut, __uint_as_float(b01), __uint_as_float(b23));
      if (fp.sh_degree >= 0 && b.sh) b.col_out[i] = col;
    }
  } else if (fp.full_record) {  // empty slot: never binned; a neutral record for the readback
    rec[0] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    rec[1] = make_float4(0.0f, __builtin_huge_valf(), 0.0f, 0.0f);
    rec[2] = make_float4(0.0f, 0.0f, __uint_as_float(kEmptyBox), __uint_as_float(kEmptyBox));
    b.rec_tail[i] = make_float2(0.0f, 0.0f);
  }
  store_rects(fp, b, i, rect, crect);
  b.depth_key[i] = dkey;
  if (dkey_out) *dkey_out = dkey;
  rect_out = rect;
  crect_out = fp.pair_cull ? crect : rect;
  return rendered;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// wave-wide min of lo and max of hi, each two packed u16 (v_pk_min / max_u16)
__device__ __forceinline__ void wave_minmax_u16x2(uint32_t& lo, uint32_t& hi) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t ol = (uint32_t)__shfl_xor((int)lo, d, 64), oh = (uint32_t)__shfl_xor((int)hi, d, 64);
    lo = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, lo), __builtin_bit_cast(u16x2, ol)));
    hi = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, hi), __builtin_bit_cast(u16x2, oh)));
  }
}

#if GS_PROBE
// the kernel's earliest start (each workgroup's first wave) and latest end
// (every wave) for the frame, spread over kProbeSlots (start, end) pairs
// (vector atomics on the probe ring; probe builds only)
struct ProbeScope {
  unsigned long long* p = nullptr;
  __device__ ProbeScope(const FrameParams& fp, const Buffers& b, int k) {
    if (b.probe && (threadIdx.x & 63) == 0) {
      const size_t slot = (size_t)(blockIdx.x * 4u + (threadIdx.x >> 6)) % (size_t)kProbeSlots;
      p = b.probe + 2 * (((size_t)(fp.probe_frame % kProbeFrames) * kProbeKernels + (size_t)k) * kProbeSlots + slot);
      if (threadIdx.x == 0) atomicMin(p, (unsigned long long)wall_clock64());
    }
  }
  __device__ ~ProbeScope() {
    if (p) atomicMax(p + 1, (unsigned long long)wall_clock64());
  }
};
#define GS_PROBE_SCOPE(k) ProbeScope gs_probe_scope_(fp, b, k)
#else
#define GS_PROBE_SCOPE(k) ((void)0)
#endif
enum { kPrProject = 0, kPrAggScan, kPrAggEmit, kPrCount, kPrColscan, kPrScanMulti, kPrEmitChunk, kPrSortTiles,
       kPrBlend, kPrBlendCont, kPrScan, kPrEmit, kPrBig };

// ----------------------------------------------------- aggregated binning
// FrameParams::bin_agg: the per-tile list lengths are summed by the
// projection's own workgroups and the pairs emitted with one returning
// global atomic per (workgroup, tile) -- no chunk matrix, no column scan.
// A workgroup's 256 Gaussians are neighbours (Morton device order), so their
// rectangles fall in a small box of tiles: each workgroup histograms its
// pairs over that box in LDS (the first lane of a run of equal rectangles
// adds the run's length), then adds every non-zero entry to the tile's
// 64-bit counter (binned count | reference count << 32).  A box larger than
// kAggCap tiles (Gaussians spread far apart, rare) adds per pair instead.
// gs_agg_scan_kernel turns the counters into tile starts and sort queues (and
// zeroes them for the next frame); gs_agg_emit_kernel reserves each
// (workgroup, tile) range with one returning atomic on the tile's cursor and
// places the pairs by LDS cursors.  The pairs land in a tile's segment in an
// order set by the atomics; the depth sort puts every list in its total
// (z, input index) order, so the lists and the frame are unchanged.
constexpr uint32_t kAggSpread = 0xFFFFFFFFu;  // agg_box area marker: the per-pair fallback
// a box of at most this many tiles is counted by ballots instead of LDS
// atomics (a clustered scene's workgroup puts all its pairs in a few tiles,
// where the LDS atomics of a wave serialise on the same addresses)
constexpr int kAggBallot = 16;

struct AggBox {
  int x0, y0, w, area;  // area 0: nothing binned in the workgroup
};

// the workgroup's box of tiles over the non-empty rectangles r (every
// thread of the 256-thread workgroup calls it)
__device__ __forceinline__ AggBox agg_box(uint2 r, uint32_t* s_lo, uint32_t* s_hi) {
  const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
  const bool ok = x0 <= x1 && y0 <= y1;
  uint32_t lo = ok ? (x0 | (y0 << 16)) : 0xFFFFFFFFu, hi = ok ? (x1 | (y1 << 16)) : 0u;
  wave_minmax_u16x2(lo, hi);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_lo[wave] = lo;
    s_hi[wave] = hi;
  }
  __syncthreads();
  lo = s_lo[0];
  hi = s_hi[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) {
    lo = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, lo),
                                                                 __builtin_bit_cast(u16x2, s_lo[w])));
    hi = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, hi),
                                                                 __builtin_bit_cast(u16x2, s_hi[w])));
  }
  AggBox bx;
  bx.x0 = (int)(lo & 0xFFFFu);
  bx.y0 = (int)(lo >> 16);
  const int bx1 = (int)(hi & 0xFFFFu), by1 = (int)(hi >> 16);
  const bool any = bx.x0 <= bx1 && bx.y0 <= by1;
  bx.w = any ? bx1 - bx.x0 + 1 : 0;
  bx.area = any ? bx.w * (by1 - bx.y0 + 1) : 0;
  return bx;
}

// run of equal (r, q) rectangles in this wave: is this lane its first, and
// the run's length
__device__ __forceinline__ bool rect_run(uint2 r, uint2 q, uint32_t& len) {
  const int lane = threadIdx.x & 63;
  const uint32_t px = (uint32_t)__shfl_up((int)r.x, 1, 64), py = (uint32_t)__shfl_up((int)r.y, 1, 64);
  const uint32_t qx = (uint32_t)__shfl_up((int)q.x, 1, 64), qy = (uint32_t)__shfl_up((int)q.y, 1, 64);
  const bool start = lane == 0 || r.x != px || r.y != py || q.x != qx || q.y != qy;
  const unsigned long long st = ballot64(start);
  const unsigned long long above = lane == 63 ? 0ull : (st & ~((2ull << lane) - 1ull));
  len = above ? (uint32_t)(__builtin_ctzll(above) - lane) : (uint32_t)(64 - lane);
  return start;
}

// The projection workgroup's share of the per-tile counters: r = reference
// rectangle, q = binned rectangle (q inside r) of this thread's Gaussian.
__device__ __forceinline__ void agg_count(const FrameParams& fp, const Buffers& b, uint2 r, uint2 q, int blk) {
  __shared__ uint32_t cnt[kAggCap];
  __shared__ uint32_t s_lo[4], s_hi[4];
  const AggBox bx = agg_box(r, s_lo, s_hi);
  // the box the emit uses (the reference rectangles' box, which holds the
  // binned ones): origin, width, area (kAggSpread: the per-pair fallback)
  if (threadIdx.x == 0)
    b.agg_box[blk] = make_uint4((uint32_t)bx.x0, (uint32_t)bx.y0, (uint32_t)bx.w,
                                bx.area > kAggCap ? kAggSpread : (uint32_t)bx.area);
  if (bx.area == 0) return;  // (uniform)
  uint32_t len;
  const bool start = rect_run(r, q, len);
  const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
  const uint32_t u0 = q.x & 0xFFFFu, u1 = q.x >> 16, v0 = q.y & 0xFFFFu, v1 = q.y >> 16;
  const bool mine = start && x0 <= x1;
  uint32_t* const off = b.agg_off + (size_t)blk * kAggCap;
  // one returning add per (workgroup, tile): binned | reference << 32 into
  // the tile's counter; the binned half of the old value is this
  // workgroup's offset within the tile's aggregated pairs (the emit's slots)
  auto reserve = [&](int k, uint32_t v) {
    const int y = bx.y0 + k / bx.w, x = bx.x0 + k % bx.w;
    const unsigned long long old =
        atomicAdd(&b.tile_cnt64[y * fp.tiles_x + x], ((unsigned long long)(v >> 16) << 32) | (v & 0xFFFFu));
    off[k] = (uint32_t)old;
  };
  if (bx.area <= kAggBallot) {  // (uniform) small box: per tile, ballots of the rectangles covering it
    __shared__ uint32_t s_wc[4][kAggBallot];
    const int wave = threadIdx.x >> 6;
    for (int k = 0; k < bx.area; ++k) {
      const uint32_t tx = (uint32_t)(bx.x0 + k % bx.w), ty = (uint32_t)(bx.y0 + k / bx.w);
      const bool in_r = x0 <= tx && tx <= x1 && y0 <= ty && ty <= y1;
      const bool in_q = u0 <= tx && tx <= u1 && v0 <= ty && ty <= v1;
      const uint32_t cr = (uint32_t)__popcll(ballot64(in_r)), cq = (uint32_t)__popcll(ballot64(in_q));
      if ((threadIdx.x & 63) == 0) s_wc[wave][k] = (cr << 16) | cq;
    }
    __syncthreads();
    if ((int)threadIdx.x < bx.area) {
      const int k = threadIdx.x;
      const uint32_t v = s_wc[0][k] + s_wc[1][k] + s_wc[2][k] + s_wc[3][k];
      if (v) reserve(k, v);
    }
    return;
  }
  if (bx.area > kAggCap) {  // (uniform) spread-out workgroup: per run, the fallback counters
    if (mine)
      for (uint32_t y = y0; y <= y1; ++y) {
        const bool yin = v0 <= y && y <= v1;
        for (uint32_t x = x0; x <= x1; ++x) {
          const uint32_t t = y * fp.tiles_x + x;
          if (yin && u0 <= x && x <= u1) atomicAdd(&b.tile_fb[t], len);
          atomicAdd(&b.tile_cnt64[t], (unsigned long long)len << 32);
        }
      }
    return;
  }
  for (int k = threadIdx.x; k < bx.area; k += 256) cnt[k] = 0u;
  __syncthreads();
  if (mine)
    for (uint32_t y = y0; y <= y1; ++y) {
      const bool yin = v0 <= y && y <= v1;
      const int row = ((int)y - bx.y0) * bx.w - bx.x0;
      for (uint32_t x = x0; x <= x1; ++x)
        atomicAdd(&cnt[row + (int)x], (len << 16) | ((yin && u0 <= x && x <= u1) ? len : 0u));
    }
  __syncthreads();
  for (int k = threadIdx.x; k < bx.area; k += 256) {
    const uint32_t v = cnt[k];
    if (v) reserve(k, v);
  }
}

// FrameParams::bin_direct (row bands): the projection workgroup places its
// own pairs.  Tile t's pairs go to [tile_start[t], tile_start[t + 1]): the
// layout the last scan of this view wrote (the same view bins the same
// lists, so each tile's segment is exactly its list).  The workgroup's
// reservation -- the returning add on the tile's counter that agg_count makes
// (binned | reference << 32) -- is its offset in that segment, so no scan
// has to run before any pair can be placed and no emit launch follows.  The
// same three box cases as agg_count (ballots for <= kAggBallot tiles, LDS
// cursors for <= kAggCap, a returning add per pair beyond), the emit's
// placement rules (agg_emit_block) inside each.  A pair past its segment (or
// the pair buffer) is not written and flags the frame (dir_word[1]): the
// blend's last workgroup reports it as the pair-capacity overflow, and the
// host bins that renderer's next frame with the scan and emit again.  The
// order of a tile's pairs is set by the atomics, as with agg_emit: the
// in-blend sort puts every list in its total (z, input index) order.
__device__ __forceinline__ uint32_t direct_limit(const FrameParams& fp, const Buffers& b, uint32_t t) {
  const uint32_t en = b.tile_start[t + 1];
  return (unsigned long long)en < fp.pair_cap ? en : (uint32_t)min(fp.pair_cap, 0xFFFFFFFFull);
}

__device__ __forceinline__ void agg_direct(const FrameParams& fp, const Buffers& b, uint2 r, uint2 q,
                                           unsigned long long key) {
  __shared__ uint32_t dcnt[kAggCap];
  __shared__ uint32_t dlim[kAggCap];
  __shared__ uint32_t d_lo[4], d_hi[4];
  __shared__ uint32_t d_wc[4][kAggBallot];
  const AggBox bx = agg_box(r, d_lo, d_hi);
  if (bx.area == 0) return;  // (uniform)
  const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
  const uint32_t u0 = q.x & 0xFFFFu, u1 = q.x >> 16, v0 = q.y & 0xFFFFu, v1 = q.y >> 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  bool ovf = false;
  auto put = [&](uint32_t pos, uint32_t lim) {
    if (pos < lim) b.pairs[pos] = key;
    else ovf = true;
  };
  if (bx.area <= kAggBallot) {  // (uniform) per tile: ballots of the rectangles covering it
    for (int k = 0; k < bx.area; ++k) {
      const uint32_t tx = (uint32_t)(bx.x0 + k % bx.w), ty = (uint32_t)(bx.y0 + k / bx.w);
      const bool in_r = x0 <= tx && tx <= x1 && y0 <= ty && ty <= y1;
      const bool in_q = u0 <= tx && tx <= u1 && v0 <= ty && ty <= v1;
      const uint32_t cr = (uint32_t)__popcll(ballot64(in_r)), cq = (uint32_t)__popcll(ballot64(in_q));
      if (lane == 0) d_wc[wave][k] = (cr << 16) | cq;
    }
    __syncthreads();
    if ((int)threadIdx.x < bx.area) {  // the workgroup's slots in the tile, split over its waves
      const int k = threadIdx.x;
      const uint32_t w0 = d_wc[0][k], w1 = d_wc[1][k], w2 = d_wc[2][k], w3 = d_wc[3][k];
      const uint32_t v = w0 + w1 + w2 + w3;
      uint32_t base = 0u, lim = 0u;
      if (v) {
        const uint32_t t = (uint32_t)((bx.y0 + k / bx.w) * fp.tiles_x + bx.x0 + k % bx.w);
        const uint32_t st = b.tile_start[t];
        lim = direct_limit(fp, b, t);
        base = st + (uint32_t)atomicAdd(&b.tile_cnt64[t], ((unsigned long long)(v >> 16) << 32) | (v & 0xFFFFu));
      }
      const uint32_t c0 = w0 & 0xFFFFu, c1 = w1 & 0xFFFFu, c2 = w2 & 0xFFFFu;
      d_wc[0][k] = base;
      d_wc[1][k] = base + c0;
      d_wc[2][k] = base + c0 + c1;
      d_wc[3][k] = base + c0 + c1 + c2;
      dlim[k] = lim;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int k = 0; k < bx.area; ++k) {
      const uint32_t tx = (uint32_t)(bx.x0 + k % bx.w), ty = (uint32_t)(bx.y0 + k / bx.w);
      const bool in_q = u0 <= tx && tx <= u1 && v0 <= ty && ty <= v1;
      const unsigned long long m = ballot64(in_q);
      if (in_q) put(d_wc[wave][k] + (uint32_t)__popcll(m & lt), dlim[k]);
    }
  } else if (bx.area > kAggCap) {  // (uniform) spread-out workgroup: a returning add per pair
    if (x0 <= x1)
      for (uint32_t y = y0; y <= y1; ++y) {
        const bool yin = v0 <= y && y <= v1;
        for (uint32_t x = x0; x <= x1; ++x) {
          const uint32_t t = y * fp.tiles_x + x;
          if (yin && u0 <= x && x <= u1)
            put(b.tile_start[t] + (uint32_t)atomicAdd(&b.tile_cnt64[t], (1ull << 32) | 1ull), direct_limit(fp, b, t));
          else
            atomicAdd(&b.tile_cnt64[t], 1ull << 32);
        }
      }
  } else {  // LDS histogram of the box, one returning add per (workgroup, tile), LDS cursors
    for (int k = threadIdx.x; k < bx.area; k += 256) dcnt[k] = 0u;
    uint32_t len;
    const bool start = rect_run(r, q, len);
    __syncthreads();
    if (start && x0 <= x1)
      for (uint32_t y = y0; y <= y1; ++y) {
        const bool yin = v0 <= y && y <= v1;
        const int row = ((int)y - bx.y0) * bx.w - bx.x0;
        for (uint32_t x = x0; x <= x1; ++x)
          atomicAdd(&dcnt[row + (int)x], (len << 16) | ((yin && u0 <= x && x <= u1) ? len : 0u));
      }
    __syncthreads();
    for (int k = threadIdx.x; k < bx.area; k += 256) {
      const uint32_t v = dcnt[k];
      uint32_t base = 0u, lim = 0u;
      if (v) {
        const uint32_t t = (uint32_t)((bx.y0 + k / bx.w) * fp.tiles_x + bx.x0 + k % bx.w);
        const uint32_t st = b.tile_start[t];
        lim = direct_limit(fp, b, t);
        base = st + (uint32_t)atomicAdd(&b.tile_cnt64[t], ((unsigned long long)(v >> 16) << 32) | (v & 0xFFFFu));
      }
      dcnt[k] = base;  // the workgroup's cursor in the tile's segment
      dlim[k] = lim;
    }
    __syncthreads();
    // a run of equal (reference, binned) rectangles takes its slots of each
    // binned tile with one LDS atomic by its first lane
    const unsigned long long st = ballot64(start);
    const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const int lead = 63 - __builtin_clzll(st & upto);
    const uint32_t rank = (uint32_t)(lane - lead);
    if (u0 <= u1)
      for (uint32_t y = v0; y <= v1; ++y) {
        const int row = ((int)y - bx.y0) * bx.w - bx.x0;
        for (uint32_t x = u0; x <= u1; ++x) {
          uint32_t base = 0u;
          if (start) base = atomicAdd(&dcnt[row + (int)x], len);
          put((uint32_t)__shfl((int)base, lead, 64) + rank, dlim[row + (int)x]);
        }
      }
  }
  if (ovf) atomicOr(&b.dir_word[1], 1u);
}

// GS_X_BAND (measurement builds only, tools/build_x.sh; wrong frames): what
// a row band's projection spends where.  1: every block returns after the
// cull pass; 2: no aggregated counting (and every block reports no rendered
// Gaussian, so the emit places nothing); 3: a band renderer projects only its
// first frame, later frames reuse its records, rectangles and counters (the
// aggregated scan keeps them): right frames for a fixed camera at no
// projection cost -- what the projection costs the pipelined band frame.
#ifndef GS_X_BAND
#define GS_X_BAND 0
#endif

// one block of 256 Gaussians (every thread of the workgroup calls it)
// STAGE (whole frames' lean projection): the records go out as streaming
// stores of whole 128-B lines -- each wave's 64 records (2 KB, contiguous)
// through LDS, written for every Gaussian of the wave (a record that no tile
// binned is never read, so its contents do not matter)
template <bool P2, bool STAGE = false, bool DIRECT = false>
__device__ __forceinline__ void project_block(const FrameParams& fp, const Buffers& b, int blk) {
  const int i = blk * 256 + threadIdx.x;
  bool rendered = false;
  uint2 rect = kEmptyRect, crect = kEmptyRect;
  uint32_t dkey = 0xFFFFFFFFu;
  if (fp.band_cull) {
    // the cheap band test first; a block of 256 Gaussians that it culls
    // entirely writes only its V (0): count and emit skip such blocks
    // without reading their rectangles, so nothing else needs writing.
    // (Per-block bounds before any Gaussian is read did not pay: DESIGN.md
    // §4 "Tried and dropped", the two round-2 block-test entries, and §0's
    // round-5 block list -- a launch projecting only the listed blocks)
    // (a per-wave test of the 64 Gaussians' bound before any of them is read,
    // round 6: slower -- DESIGN.md section 4 "Tried and dropped")
    bool culled = true;
    if (i < fp.n) {
      // one 16-B load (the mean and the largest scale) instead of two
      const float4 cr = b.cull[i];
      culled = !__builtin_isnan(cr.w) && band_culled_fast<P2>(fp, cr);
    }
    if (__syncthreads_count(i < fp.n && !culled) == 0 || GS_X_BAND == 1) {
      if (threadIdx.x == 0) b.block_rendered[blk] = 0u;
      return;
    }
    if (i >= fp.n) {
    } else if (culled) {  // no tile row in this band: empty rectangle, no record
      store_rects(fp, b, i, kEmptyRect, kEmptyRect);
      b.depth_key[i] = 0xFFFFFFFFu;
    } else {
      rendered = project_one<P2>(fp, b, i, rect, crect, nullptr, &dkey);
    }
  } else if constexpr (STAGE) {
    __shared__ float4 s_rec[4][128];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float4 r2[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    if (i < fp.n) rendered = project_one<P2>(fp, b, i, rect, crect, r2);
    float4* const sw = s_rec[wave];
    sw[2 * lane] = r2[0];
    sw[2 * lane + 1] = r2[1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int i0 = blk * 256 + wave * 64;  // the wave's first Gaussian
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 64 * h + lane;  // float4 k of the wave's records: record i0 + k / 2
      if (i0 + (k >> 1) < fp.n) store_stream(b.rec + 2 * (size_t)i0 + k, sw[k]);
    }
  } else if (i < fp.n) {
    rendered = project_one<P2>(fp, b, i, rect, crect);
  }
  if (fp.bin_agg && GS_X_BAND != 2) {
    if constexpr (DIRECT)  // the pairs go to the tiles' fixed segments now
      agg_direct(fp, b, rect, crect, ((unsigned long long)dkey << 32) | (uint32_t)i);
    else
      agg_count(fp, b, rect, crect, blk);
  }
  // V per workgroup (summed by the scan kernel): no single-address atomics
  const int v = __syncthreads_count(rendered);
  if (threadIdx.x == 0) b.block_rendered[blk] = (fp.band_cull && GS_X_BAND == 2) ? 0u : (uint32_t)v;
}

// one workgroup per block (a grid of workgroups walking the blocks held
// 73-113 VGPRs inside the loop instead of 51-57: config 3 7 824 against
// 8 275 frames/s).  MODE: the paths compiled into the instantiation (a smaller kernel beside
// the other frames' kernels in the CU pair's instruction cache: config 3's
// projection 35.5 -> 32.4 us, 7 782 -> 8 048 frames/s with the lean one).
// kProjLean: a whole frame's plain projection (no band cull, no aggregated
// counting, no readback record, no SH, no global-atomic binning);
// kProjBand: a row band's (band cull and aggregated counting, nothing else);
// kProjAny: every path, chosen at run time.
// kProjDirect: a direct-binned band's (kProjBand with agg_direct instead of
// agg_count: FrameParams::bin_direct).
enum { kProjAny = 0, kProjLean = 1, kProjBand = 2, kProjDirect = 3 };
template <bool P2, int MODE>
__device__ __forceinline__ void project_entry(FrameParams fp, const Buffers& b) {
  GS_PROBE_SCOPE(kPrProject);
  if constexpr (MODE != kProjAny) {
    fp.band_cull = (MODE == kProjBand || MODE == kProjDirect) ? 1 : 0;
    fp.bin_agg = (MODE == kProjBand || MODE == kProjDirect) ? 1 : 0;
    fp.full_record = 0;
    fp.sh_degree = -1;
    fp.bin_global = 0;
  }
  project_block<P2, MODE == kProjLean, MODE == kProjDirect>(fp, b, blockIdx.x);
}
// one kernel name per kind, so a profile's per-kernel counters are the
// kind's own (gs_frame_stats.paths bits GS_PATH_PROJ_BAND / _ANY)
template <bool P2>
__global__ __launch_bounds__(256) void gs_project_kernel(FrameParams fp, Buffers b) {
  project_entry<P2, kProjLean>(fp, b);
}
template <bool P2>
__global__ __launch_bounds__(256) void gs_project_band_kernel(FrameParams fp, Buffers b) {
  project_entry<P2, kProjBand>(fp, b);
}
template <bool P2>
__global__ __launch_bounds__(256) void gs_project_any_kernel(FrameParams fp, Buffers b) {
  project_entry<P2, kProjAny>(fp, b);
}
template <bool P2>
__global__ __launch_bounds__(256) void gs_project_direct_kernel(FrameParams fp, Buffers b) {
  project_entry<P2, kProjDirect>(fp, b);
}

// --------------------------------------------------------------------- scan
// One workgroup of 1024 threads, rounds of 8192 tiles (8 per thread, held in
// registers): tile_start = exclusive scan(tile_count), max list length, and
// the sort queues -- tiles too long for the one-wave register sort are
// compacted into medium_tiles / big_tiles here (no contended atomics).
__device__ __forceinline__ int sort_class(uint32_t L) {
  return L <= kSortRegCap ? 0 : (L <= (uint32_t)kSortLdsCap ? 1 : 2);
}

__global__ __launch_bounds__(1024) void gs_scan_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrScan);
  __shared__ unsigned long long wsum[16];
  __shared__ uint32_t wq[16];  // per wave: small | medium << 10 | big << 20 (<= 512 each)
  __shared__ uint32_t wmax[16];
  __shared__ uint32_t wvis[16];
  const int T = fp.n_tiles;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // V = sum of the project workgroups' counts (loads issued up front)
  uint32_t vsum = 0;
  {
    const int nb = (fp.n + 255) / 256;
    uint32_t vr[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = tid + k * 1024;
      vr[k] = i < nb ? b.block_rendered[i] : 0u;
    }
    for (int i = tid + 8 * 1024; i < nb; i += 1024) vsum += b.block_rendered[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) vsum += vr[k];
  }
  unsigned long long carry = 0;
  uint32_t sml_base = 0, med_base = 0, big_base = 0, mx = 0;
  for (int r0 = 0; r0 < T; r0 += 8192) {
    const int i0 = r0 + tid * 8;
    uint32_t c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = (i0 + j < T) ? b.tile_count[i0 + j] : 0u;
    unsigned long long sum = 0;
    uint32_t q = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sum += c[j];
      mx = max(mx, c[j]);
      const int cl = sort_class(c[j]);
      // small queue: empty tiles too -- but not the round's slots past the
      // last tile (counted, they made the small queue longer than the tiles
      // written to it, and the sort read tile ids past its end)
      if (i0 + j < T) q += cl == 0 ? 1u : (cl == 1 ? (1u << 10) : (1u << 20));
    }
    unsigned long long inc = sum;
    uint32_t qinc = q;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long o = __shfl_up(inc, d, 64);
      const uint32_t oq = __shfl_up(qinc, d, 64);
      if (lane >= d) {
        inc += o;
        qinc += oq;
      }
    }
    if (lane == 63) {
      wsum[wave] = inc;
      wq[wave] = qinc;
    }
    __syncthreads();
    unsigned long long base = carry, total = carry;
    uint32_t qb[3] = {0, 0, 0}, qt[3] = {0, 0, 0};
    for (int w = 0; w < 16; ++w) {
      const uint32_t v = wq[w];
      if (w < wave) {
        base += wsum[w];
        for (int k = 0; k < 3; ++k) qb[k] += (v >> (10 * k)) & 1023u;
      }
      total += wsum[w];
      for (int k = 0; k < 3; ++k) qt[k] += (v >> (10 * k)) & 1023u;
    }
    unsigned long long run = base + inc - sum;
    const uint32_t qx = qinc - q;  // this lane's exclusive counts in the wave
    uint32_t sml = sml_base + qb[0] + (qx & 1023u);
    uint32_t med = med_base + qb[1] + ((qx >> 10) & 1023u);
    uint32_t big = big_base + qb[2] + ((qx >> 20) & 1023u);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = i0 + j;
      if (i < T) {
        b.tile_start[i] = (uint32_t)run;
        if (fp.bin_global) b.tile_cursor[i] = (uint32_t)run;
        const int cl = sort_class(c[j]);
        if (cl == 0) b.small_tiles[sml++] = (uint32_t)i;
        if (cl == 1) b.medium_tiles[med++] = (uint32_t)i;
        if (cl == 2) b.big_tiles[big++] = (uint32_t)i;
      }
      run += c[j];
    }
    carry = total;
    sml_base += qt[0];
    med_base += qt[1];
    big_base += qt[2];
    __syncthreads();  // wsum / wq are rewritten by the next round
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) vsum += __shfl_xor(vsum, d, 64);
  if (lane == 0) {
    wvis[wave] = vsum;
    wmax[wave] = mx;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t vis = 0, m = 0;
    for (int w = 0; w < 16; ++w) {
      vis += wvis[w];
      m = max(m, wmax[w]);
    }
    // every counter of the frame is (re)set here: the chunked path needs no
    // per-frame memset (colscan writes every tile_count)
    b.counters[0] = big_base;
    b.counters[1] = 0;  // (unused)
    b.counters[8] = 0;  // medium_next
    for (int k = 10; k < 16; ++k) b.counters[k] = 0;
    b.counters[2] = vis;
    b.counters[7] = med_base;
    b.counters[9] = sml_base;
    const unsigned long long total = carry;
    b.tile_start[T] = (uint32_t)(total < 0xFFFFFFFFull ? total : 0xFFFFFFFFull);
    b.counters[3] = total > fp.pair_cap ? 1u : 0u;
    if (total > fp.pair_cap) {  // sticky until the host's sync
      *b.host_sticky = 1u;
      if (b.group_sticky) *b.group_sticky = 1u;
    }
    b.counters[4] = m;
    b.counters[5] = (uint32_t)total;
    b.counters[6] = (uint32_t)(total >> 32);
  }
}

// Aggregated binning (FrameParams::bin_agg): tile starts, the sort queues and
// the frame counters from the projection's per-tile counters (binned |
// reference << 32), which it resets to zero for the next frame.  One
// workgroup of 1024 threads, rounds of 4096 tiles (4 per thread in
// registers; 8 spilled); the histogram (reference lengths) and the counters go straight
// to the mapped host mirror and, in a row-band group, to the frame's footer.
// the aggregated scan's queues: 0 small (<= 256 keys), 1..3 medium with
// >= 1024, >= 512, > 256 keys, 4 big (> 2048)
constexpr int kAggQueues = 5;
__device__ __forceinline__ int agg_queue(uint32_t L) {
  return L <= kSortRegCap ? 0 : (L > (uint32_t)kSortLdsCap ? 4 : (L >= 1024u ? 1 : (L >= 512u ? 2 : 3)));
}

template <int NT, int PER>
__global__ __launch_bounds__(NT) void gs_agg_scan_kernel(FrameParams fp, Buffers b) {
  constexpr int NW = NT / 64, ROUND = NT * PER;
  static_assert(NW >= 2 && NW <= 16 && 64 * PER <= 1023, "wave scan by lanes < NW; 10-bit queue fields");
  GS_PROBE_SCOPE(kPrAggScan);
  // per wave of a round: pair sum, reference sum, queue counts; per wave the
  // exclusive bases (computed by lanes 0..NW-1 of wave 0), and the round totals
  __shared__ unsigned long long wsum[NW], wref[NW], wbase[NW], wq[NW];
  __shared__ uint32_t wqb[kAggQueues][NW], wvis[NW], wmax[NW];
  __shared__ unsigned long long s_tot;
  __shared__ uint32_t s_qt[3];
  __shared__ uint32_t s_c[ROUND];  // a round's binned counts (striped in, blocked out)
  __shared__ uint32_t s_a[ROUND];  // ... their aggregated parts
  const int T = fp.n_tiles;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // a round's counters, read striped (coalesced: lane-consecutive tiles);
  // the first round's are issued before the V loads (one memory round trip
  // for both)
  unsigned long long vs[PER];
  uint32_t fb[PER];
  auto load_round = [&](int r0) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = r0 + j * NT + tid;
      vs[j] = i < T ? b.tile_cnt64[i] : 0ull;
      fb[j] = i < T ? b.tile_fb[i] : 0u;
    }
  };
  load_round(0);
  // V = the projection workgroups' counts, reduced per wave at once (kept
  // live across the rounds they were spilled)
  {
    const int nb = (fp.n + 255) / 256;
    uint32_t vr[8], vsum = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = tid + k * NT;
      vr[k] = i < nb ? b.block_rendered[i] : 0u;
    }
    for (int i = tid + 8 * NT; i < nb; i += NT) vsum += b.block_rendered[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) vsum += vr[k];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) vsum += __shfl_xor(vsum, d, 64);
    if (lane == 0) wvis[wave] = vsum;
  }
  // (lanes 0..15 of wave 0) the running bases over the rounds: pairs,
  // reference pairs, small / medium / big queue lengths
  unsigned long long carry = 0, rcarry = 0;
  uint32_t qcarry[3] = {0u, 0u, 0u};
  uint32_t mx = 0;
  for (int r0 = 0; r0 < T; r0 += ROUND) {
    // the round's counters, read striped (coalesced: lane-consecutive tiles);
    // the histogram goes to tile_ref (and the group's footer) from here, the
    // counters are zeroed for the next frame, and the binned counts are
    // transposed through LDS so each thread scans 8 consecutive tiles
    unsigned long long rsum = 0;
    {
      if (r0 > 0) load_round(r0);
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int i = r0 + j * NT + tid;
        const uint32_t rf = (uint32_t)(vs[j] >> 32);
        rsum += rf;
        s_c[j * NT + tid] = (uint32_t)vs[j] + fb[j];  // the tile's binned pairs
        s_a[j * NT + tid] = (uint32_t)vs[j];          // ... of which the aggregated workgroups'
        if (i < T) {
          if (GS_X_BAND != 3) {
            b.tile_cnt64[i] = 0ull;  // zero for the next frame's projection
            b.tile_fb[i] = 0u;
          }
          b.tile_ref[i] = rf;      // the histogram (reference list lengths; the host reads it at sync)
          if (b.footer) b.footer[16 + i] = rf;
        }
      }
    }
    __syncthreads();
    const int i0 = r0 + tid * PER;
    uint32_t v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) v[j] = s_c[tid * PER + j];
    unsigned long long sum = 0, q = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t c = v[j];
      sum += c;
      mx = max(mx, c);
      if (i0 + j < T) q += 1ull << (10 * agg_queue(c));
    }
    unsigned long long inc = sum, qinc = q;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long o = __shfl_up(inc, d, 64);
      const unsigned long long oq = __shfl_up(qinc, d, 64);
      if (lane >= d) {
        inc += o;
        qinc += oq;
      }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) rsum += __shfl_xor(rsum, d, 64);
    if (lane == 63) {
      wsum[wave] = inc;
      wq[wave] = qinc;
    }
    if (lane == 0) wref[wave] = rsum;
    __syncthreads();
    if (tid < NW) {  // exclusive scan over the NW waves
      const unsigned long long ws = wsum[tid], wqv = wq[tid];
      unsigned long long si = ws, ri = wref[tid], qi = wqv;  // (queue counts: 5 fields of 10 bits, <= 64 PER each per wave)
      uint32_t qk[kAggQueues];
#pragma unroll
      for (int k = 0; k < kAggQueues; ++k) qk[k] = (uint32_t)(wqv >> (10 * k)) & 1023u;
      uint32_t qs[kAggQueues];  // (inclusive scans of the NW waves' counts; a field can pass 1023 here)
#pragma unroll
      for (int k = 0; k < kAggQueues; ++k) qs[k] = qk[k];
#pragma unroll
      for (int d = 1; d < NW; d <<= 1) {
        const unsigned long long o = __shfl_up(si, d, 64), orr = __shfl_up(ri, d, 64);
        uint32_t oq[kAggQueues];
#pragma unroll
        for (int k = 0; k < kAggQueues; ++k) oq[k] = __shfl_up(qs[k], d, 64);
        if (tid >= d) {
          si += o;
          ri += orr;
#pragma unroll
          for (int k = 0; k < kAggQueues; ++k) qs[k] += oq[k];
        }
      }
      (void)qi;
      wbase[tid] = carry + si - ws;
      uint32_t qt[kAggQueues];
#pragma unroll
      for (int k = 0; k < kAggQueues; ++k) qt[k] = __shfl(qs[k], NW - 1, 64);
      // queue bases of this round: small, big, then the medium lists longest
      // first (>= 1024, >= 512, > 256 keys: the sort, and a band's
      // longest-first blend, start the heaviest lists first)
      const uint32_t mb0 = qcarry[1], mb1 = mb0 + qt[1], mb2 = mb1 + qt[2];
      wqb[0][tid] = qcarry[0] + qs[0] - qk[0];
      wqb[1][tid] = mb0 + qs[1] - qk[1];
      wqb[2][tid] = mb1 + qs[2] - qk[2];
      wqb[3][tid] = mb2 + qs[3] - qk[3];
      wqb[4][tid] = qcarry[2] + qs[4] - qk[4];
      const unsigned long long tot = __shfl(si, NW - 1, 64), rtot = __shfl(ri, NW - 1, 64);
      carry += tot;
      rcarry += rtot;
      qcarry[0] += qt[0];
      qcarry[1] += qt[1] + qt[2] + qt[3];
      qcarry[2] += qt[4];
      if (tid == 0) {
        s_tot = carry;
#pragma unroll
        for (int k = 0; k < 3; ++k) s_qt[k] = qcarry[k];
      }
    }
    __syncthreads();
    unsigned long long run = wbase[wave] + inc - sum;
    const unsigned long long qx = qinc - q;  // this lane's exclusive counts in the wave
    uint32_t qpos[kAggQueues];
#pragma unroll
    for (int k = 0; k < kAggQueues; ++k) qpos[k] = wqb[k][wave] + ((uint32_t)(qx >> (10 * k)) & 1023u);
    __syncthreads();  // (every thread has read its counts from s_c)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = i0 + j;
      const uint32_t c = v[j];
      s_c[tid * PER + j] = (uint32_t)(run < 0xFFFFFFFFull ? run : 0xFFFFFFFFull);  // the tile start
      if (i < T) {
        const int qq = agg_queue(c);
        const uint32_t pos = qpos[qq]++;
        if (qq == 0) b.small_tiles[pos] = (uint32_t)i;
        if (qq >= 1 && qq <= 3) b.medium_tiles[pos] = (uint32_t)i;
        if (b.tile_big) b.tile_big[i] = qq == 4 ? pos : 0xFFFFFFFFu;
        if (qq == 4) b.big_tiles[pos] = (uint32_t)i;
      }
      run += c;
    }
    __syncthreads();
    // the tile starts back striped (coalesced stores)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = r0 + j * NT + tid;
      if (i < T) {
        const uint32_t st = s_c[j * NT + tid];
        b.tile_start[i] = st;
        // the fallback workgroups' pairs follow the aggregated ones'
        b.tile_cursor[i] = st + s_a[j * NT + tid];
      }
    }
    __syncthreads();  // the wave tables and s_c are rewritten by the next round
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
  if (lane == 0) wmax[wave] = mx;
  __syncthreads();
  if (tid == 0) {
    uint32_t vis = 0, m = 0;
    for (int w = 0; w < NW; ++w) {
      vis += wvis[w];
      m = max(m, wmax[w]);
    }
    const unsigned long long total = T > 0 ? s_tot : 0ull;
    // the frame counters from registers (no read-back of what was just
    // stored), 16-B stores
    const uint4 c0 = make_uint4(T > 0 ? s_qt[2] : 0u, 0u, vis, total > fp.pair_cap ? 1u : 0u);
    const uint4 c1 = make_uint4(m, (uint32_t)total, (uint32_t)(total >> 32), T > 0 ? s_qt[1] : 0u);
    // (tid 0 ran the wave scans: its rcarry is the frame's)
    const uint4 c2 = make_uint4(0u, T > 0 ? s_qt[0] : 0u, (uint32_t)rcarry, (uint32_t)(rcarry >> 32));
    const uint4 c3 = make_uint4(0u, 0u, 0u, 0u);
    if (total > fp.pair_cap) {  // sticky until the host's sync
      *b.host_sticky = 1u;
      if (b.group_sticky) *b.group_sticky = 1u;
    }
    uint4* const cv = reinterpret_cast<uint4*>(b.counters);
    cv[0] = c0;
    cv[1] = c1;
    cv[2] = c2;
    cv[3] = c3;
    b.tile_start[T] = (uint32_t)(total < 0xFFFFFFFFull ? total : 0xFFFFFFFFull);
    if (b.footer) {
      uint4* const fv = reinterpret_cast<uint4*>(b.footer);
      fv[0] = c0;
      fv[1] = c1;
      fv[2] = c2;
      fv[3] = c3;
    }
    // the host mirror: written here only when no emit follows (the emit's
    // first workgroup copies it, off this single-workgroup kernel's path)
    if (fp.n == 0) {
      const uint32_t cc[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                               c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, fp.frame_seq};
      for (int k = 0; k < 16; ++k) b.host_counters[k] = cc[k];
    }
  }
}

// Aggregated binning's emit: one workgroup per projection block of 256
// Gaussians.  The projection reserved the block's range of every tile it has
// pairs in (agg_off: its offset among the tile's aggregated pairs) over the
// box it recorded (agg_box); each pair takes the next slot of its tile's
// range: by ballot ranks for a box of <= kAggBallot tiles, else from an LDS
// cursor per tile (one atomic per run of equal rectangles).  A block whose
// box was too wide for LDS places every pair with a global cursor past the
// tile's aggregated pairs.
__device__ __forceinline__ void agg_emit_block(const FrameParams& fp, const Buffers& b, int blk, uint32_t* cnt,
                                               uint32_t (*s_wc)[kAggBallot]) {
  const int i = blk * 256 + (int)threadIdx.x;
  if (fp.band_cull && b.block_rendered[blk] == 0u) return;  // (uniform) culled block: nothing binned
  const uint4 box = b.agg_box[blk];
  if (box.w == 0u) return;  // (uniform) nothing binned
  uint2 r = kEmptyRect;
  uint32_t dk = 0u;
  if (i < fp.n) {
    r = fp.rect8 ? rect8_unpack(reinterpret_cast<const uint32_t*>(b.crect)[i]) : (fp.pair_cull ? b.crect[i] : b.rect[i]);
    dk = b.depth_key[i];
  }
  const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
  const unsigned long long key = ((unsigned long long)dk << 32) | (uint32_t)i;
  if (box.w == kAggSpread || box.z == 0u) {  // (uniform) the per-pair fallback
    if (x0 <= x1)
      for (uint32_t y = y0; y <= y1; ++y)
        for (uint32_t x = x0; x <= x1; ++x) {
          const uint32_t pos = atomicAdd(&b.tile_cursor[y * fp.tiles_x + x], 1u);
          if (pos < fp.pair_cap) b.pairs[pos] = key;
        }
    return;
  }
  const int bx0 = (int)box.x, by0 = (int)box.y, bw = (int)box.z, area = (int)box.w;
  const uint32_t* const off = b.agg_off + (size_t)blk * kAggCap;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (area <= kAggBallot) {  // (uniform) small box: ranks from ballots, no LDS atomics
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int k = 0; k < area; ++k) {
      const uint32_t tx = (uint32_t)(bx0 + k % bw), ty = (uint32_t)(by0 + k / bw);
      const bool in = x0 <= tx && tx <= x1 && y0 <= ty && ty <= y1;
      const uint32_t c = (uint32_t)__popcll(ballot64(in));
      if (lane == 0) s_wc[wave][k] = c;
    }
    __syncthreads();
    if ((int)threadIdx.x < area) {  // the block's range, split over its waves
      const int k = threadIdx.x;
      const uint32_t c0 = s_wc[0][k], c1 = s_wc[1][k], c2 = s_wc[2][k], c3 = s_wc[3][k];
      uint32_t base = 0u;
      if (c0 + c1 + c2 + c3) {
        const int y = by0 + k / bw, x = bx0 + k % bw;
        base = b.tile_start[y * fp.tiles_x + x] + off[k];
      }
      s_wc[0][k] = base;
      s_wc[1][k] = base + c0;
      s_wc[2][k] = base + c0 + c1;
      s_wc[3][k] = base + c0 + c1 + c2;
    }
    __syncthreads();
    for (int k = 0; k < area; ++k) {
      const uint32_t tx = (uint32_t)(bx0 + k % bw), ty = (uint32_t)(by0 + k / bw);
      const bool in = x0 <= tx && tx <= x1 && y0 <= ty && ty <= y1;
      const unsigned long long m = ballot64(in);
      if (in) {
        const uint32_t pos = s_wc[wave][k] + (uint32_t)__popcll(m & lt);
        if (pos < fp.pair_cap) b.pairs[pos] = key;
      }
    }
    return;
  }
  // LDS cursors seeded with the block's ranges (entries of tiles without its
  // pairs hold stale offsets, never used)
  for (int k = threadIdx.x; k < area; k += 256) {
    const int y = by0 + k / bw, x = bx0 + k % bw;
    cnt[k] = b.tile_start[y * fp.tiles_x + x] + off[k];
  }
  uint32_t len;
  const bool start = rect_run(r, r, len);
  __syncthreads();
  // a run of equal rectangles takes its slots of each tile with one LDS
  // atomic by its first lane (clustered scenes: the lanes of a wave would
  // otherwise serialise on the same few tiles' cursors)
  const unsigned long long st = ballot64(start);
  const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  const int lead = 63 - __builtin_clzll(st & upto);
  const uint32_t rank = (uint32_t)(lane - lead);
  if (x0 <= x1)
    for (uint32_t y = y0; y <= y1; ++y) {
      const int row = ((int)y - by0) * bw - bx0;
      for (uint32_t x = x0; x <= x1; ++x) {
        uint32_t base = 0u;
        if (start) base = atomicAdd(&cnt[row + (int)x], len);
        const uint32_t pos = (uint32_t)__shfl((int)base, lead, 64) + rank;
        if (pos < fp.pair_cap) b.pairs[pos] = key;
      }
    }
}

// one workgroup per projection block, or (FrameParams::emit_grid) a grid
// of that many workgroups walking the blocks
__global__ __launch_bounds__(256) void gs_agg_emit_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrAggEmit);
  __shared__ uint32_t cnt[kAggCap];
  __shared__ uint32_t s_wc[4][kAggBallot];
  // the scan's frame counters to the mapped host mirror (the next frames'
  // big-list hint, the host's counters at sync)
  // (word 15: the frame's number, for the host's direct-binning choice)
  if (blockIdx.x == 0 && threadIdx.x < 16)
    b.host_counters[threadIdx.x] = threadIdx.x == 15 ? fp.frame_seq : b.counters[threadIdx.x];
  const int nb = (fp.n + 255) / 256;
  for (int blk = blockIdx.x; blk < nb; blk += gridDim.x) {
    agg_emit_block(fp, b, blk, cnt, s_wc);
    if ((int)gridDim.x < nb) __syncthreads();  // (uniform) the next block rewrites the LDS
  }
}

// ------------------------------------------------------------ chunked binning
// The Gaussians are cut into chunks of fp.chunk_size; one 1024-thread
// workgroup per chunk keeps a private histogram over all band tiles in LDS,
// two 16-bit counters per word (a chunk adds at most chunk_size <= 65535 to a
// tile), so the contended global atomics of a plain histogram never happen.
//   count:   chunk histogram rows -> chunk_off[chunk][tile]
//   colscan: per tile, exclusive scan over chunks (in place) + tile totals
//   emit:    chunk c writes its pairs of tile t at
//            tile_start[t] + chunk_off[c][t] + (LDS slot counter)
// GS_FLAG_BAND_CULL: the projection skips every write of a 256-Gaussian block
// its cheap band test culls entirely (block_rendered = 0), so binning must not
// read such a block's rectangles
__device__ __forceinline__ bool block_live(const FrameParams& fp, const Buffers& b, int i) {
  return !fp.band_cull || b.block_rendered[i >> 8] != 0u;
}

__device__ __forceinline__ void lds_zero(uint32_t* cnt, int words) {
  for (int i = threadIdx.x; i < words; i += blockDim.x) cnt[i] = 0;
}

__global__ __launch_bounds__(1024) void gs_count_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrCount);
  extern __shared__ __attribute__((aligned(16))) uint32_t cnt[];
  const int T = fp.n_tiles;
  const int c = blockIdx.x;
  const int g0 = c * fp.chunk_size;
  const int g1 = min(fp.n, g0 + fp.chunk_size);
  // Consecutive Gaussians (Morton order) often share their whole rectangle:
  // the first lane of each run of equal rectangles adds the run length, so
  // the LDS atomics on the same counters are not serialised lane by lane.
  const int lane = threadIdx.x & 63;
  if (fp.pair_cull) {
    // one u32 per tile: binned (culled) pairs in the low half, the reference
    // list length in the high half (chunk_size <= 65535 keeps both in 16 bits)
    lds_zero(cnt, T);
    __syncthreads();
    for (int i00 = g0; i00 < g1; i00 += 4096) {  // 4 Gaussians per thread, loaded up front
      uint2 rr[4], qq[4];
      bool live[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = i00 + k * 1024 + (int)threadIdx.x;
        // band cull: a 256-Gaussian block with no rendered Gaussian (project's
        // block_rendered) has only empty rectangles; skip its loads (wave-uniform)
        live[k] = i < g1 && block_live(fp, b, i);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = i00 + k * 1024 + (int)threadIdx.x;
        if (fp.rect8) {
          rr[k] = rect8_unpack(live[k] ? reinterpret_cast<const uint32_t*>(b.rect)[i] : 0x00010001u);
          qq[k] = rect8_unpack(live[k] ? reinterpret_cast<const uint32_t*>(b.crect)[i] : 0x00010001u);
        } else {
          rr[k] = live[k] ? b.rect[i] : kEmptyRect;
          qq[k] = live[k] ? b.crect[i] : kEmptyRect;
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint2 r = rr[k], q = qq[k];
        const uint32_t px = (uint32_t)__shfl_up((int)r.x, 1, 64), py = (uint32_t)__shfl_up((int)r.y, 1, 64);
        const uint32_t qx = (uint32_t)__shfl_up((int)q.x, 1, 64), qy = (uint32_t)__shfl_up((int)q.y, 1, 64);
        const bool start = lane == 0 || r.x != px || r.y != py || q.x != qx || q.y != qy;
        const unsigned long long st = ballot64(start);
        const unsigned long long above = lane == 63 ? 0ull : (st & ~((2ull << lane) - 1ull));
        const uint32_t len = above ? (uint32_t)(__builtin_ctzll(above) - lane) : (uint32_t)(64 - lane);
        const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
        const uint32_t u0 = q.x & 0xFFFFu, u1 = q.x >> 16, v0 = q.y & 0xFFFFu, v1 = q.y >> 16;
        if (!start || x0 > x1) continue;
        for (uint32_t y = y0; y <= y1; ++y) {
          const bool yin = v0 <= y && y <= v1;
          for (uint32_t x = x0; x <= x1; ++x) {
            const uint32_t inc = (len << 16) | ((yin && u0 <= x && x <= u1) ? len : 0u);
            atomicAdd(&cnt[y * fp.tiles_x + x], inc);
          }
        }
      }
    }
    __syncthreads();
    uint32_t* row = b.chunk_off + (size_t)c * T;
    for (int t = threadIdx.x; t < T; t += 1024) row[t] = cnt[t];
    return;
  }
  lds_zero(cnt, (T + 1) >> 1);
  __syncthreads();
  for (int i0 = g0; i0 < g1; i0 += 1024) {
    const int i = i0 + (int)threadIdx.x;
    const uint2 r = (i < g1 && block_live(fp, b, i)) ? b.rect[i] : kEmptyRect;
    const uint32_t px = (uint32_t)__shfl_up((int)r.x, 1, 64), py = (uint32_t)__shfl_up((int)r.y, 1, 64);
    const bool start = lane == 0 || r.x != px || r.y != py;
    const unsigned long long st = ballot64(start);
    const unsigned long long above = lane == 63 ? 0ull : (st & ~((2ull << lane) - 1ull));
    const uint32_t len = above ? (uint32_t)(__builtin_ctzll(above) - lane) : (uint32_t)(64 - lane);
    const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
    if (!start || x0 > x1) continue;
    for (uint32_t y = y0; y <= y1; ++y)
      for (uint32_t x = x0; x <= x1; ++x) {
        const uint32_t t = y * fp.tiles_x + x;
        atomicAdd(&cnt[t >> 1], len << ((t & 1u) * 16u));
      }
  }
  __syncthreads();
  uint32_t* row = b.chunk_off + (size_t)c * T;
  for (int t = threadIdx.x; t < T; t += 1024) row[t] = (cnt[t >> 1] >> ((t & 1) * 16)) & 0xFFFFu;
}

// 64 tiles per workgroup (one per lane), the chunk rows split over 16 waves
// (n_chunks <= 256: at most 16 rows per wave, held in registers; a larger
// scene's rows past a wave's 16th are read twice, summed then rewritten).
__global__ __launch_bounds__(1024) void gs_colscan_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrColscan);
  __shared__ uint32_t wsum[16][64], whsum[16][64];
  const int T = fp.n_tiles, NC = fp.n_chunks;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = blockIdx.x * 64 + lane;
  const int rows = (NC + 15) / 16;
  const int c0 = wave * rows, c1 = min(NC, c0 + rows);
  // pair_cull: entries hold binned | reference << 16; the offsets scan the
  // binned counts, the reference counts are only summed (the histogram)
  const uint32_t lo_mask = fp.pair_cull ? 0xFFFFu : 0xFFFFFFFFu;
  uint32_t v[16];
  uint32_t sum = 0, hsum = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t e = (t < T && c0 + k < c1) ? b.chunk_off[(size_t)(c0 + k) * T + t] : 0u;
    v[k] = e & lo_mask;
    sum += v[k];
    hsum += fp.pair_cull ? e >> 16 : e;
  }
  for (int cc0 = c0 + 16; cc0 < c1; cc0 += 8) {  // (n_chunks > 256 only) 8 loads in flight
    uint32_t e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = (t < T && cc0 + k < c1) ? b.chunk_off[(size_t)(cc0 + k) * T + t] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sum += e[k] & lo_mask;
      hsum += fp.pair_cull ? e[k] >> 16 : e[k];
    }
  }
  wsum[wave][lane] = sum;
  whsum[wave][lane] = hsum;
  __syncthreads();
  uint32_t run = 0;
  for (int w = 0; w < wave; ++w) run += wsum[w][lane];
  if (t < T) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (c0 + k < c1) b.chunk_off[(size_t)(c0 + k) * T + t] = run;
      run += v[k];
    }
    for (int cc0 = c0 + 16; cc0 < c1; cc0 += 8) {
      uint32_t e[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = cc0 + k < c1 ? b.chunk_off[(size_t)(cc0 + k) * T + t] & lo_mask : 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (cc0 + k < c1) b.chunk_off[(size_t)(cc0 + k) * T + t] = run;
        run += e[k];
      }
    }
    if (wave == 15) b.tile_count[t] = run;
  }
  if (wave == 15) {  // this workgroup's 64 tiles, summarised for gs_scan_multi_kernel
    const bool ok = t < T;
    uint32_t href = 0;  // the reference list length: the histogram, straight to host memory
    for (int w = 0; w < 16; ++w) href += whsum[w][lane];
    if (ok) b.host_counters[16 + t] = href;
    if (ok && b.footer) b.footer[16 + t] = href;
    unsigned long long rsum = ok ? href : 0u;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) rsum += __shfl_xor(rsum, d, 64);
    if (lane == 0) b.tile_agg[2 * blockIdx.x + 1] = make_uint4((uint32_t)rsum, (uint32_t)(rsum >> 32), 0u, 0u);
    const uint32_t L = ok ? run : 0u;
    unsigned long long sum = L;
    uint32_t mx = L;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      sum += __shfl_xor(sum, d, 64);
      mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
    }
    const int cl = sort_class(L);
    const uint32_t ns = (uint32_t)__popcll(ballot64(ok && cl == 0));
    const uint32_t nm = (uint32_t)__popcll(ballot64(ok && cl == 1));
    const uint32_t nb = (uint32_t)__popcll(ballot64(ok && cl == 2));
    if (lane == 0)
      b.tile_agg[2 * blockIdx.x] = make_uint4((uint32_t)sum, (uint32_t)(sum >> 32), ns | (nm << 8) | (nb << 16), mx);
  }
}

// Chunked path: tile starts and sort queues from the colscan's per-64-tile
// summaries.  One workgroup per 64 tiles: it scans the summaries of the
// workgroups before it (all of them are in memory already, no chaining),
// then its 64 tiles in one wave.  Workgroup 0 also writes the frame counters.
// Counters and list lengths also go straight to the mapped host mirror, so a
// frame needs no device-to-host copy.
__global__ __launch_bounds__(256) void gs_scan_multi_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrScanMulti);
  __shared__ unsigned long long s_sum[3][4];
  __shared__ uint32_t s_q[2][4][3], s_mx[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x, G = gridDim.x, T = fp.n_tiles;
  unsigned long long ps = 0, ts = 0, rs = 0;
  uint32_t pq[3] = {0, 0, 0}, tq[3] = {0, 0, 0}, mx = 0;
  for (int i = tid; i < G; i += 256) {
    const uint4 a = b.tile_agg[2 * i];
    const uint4 ar = b.tile_agg[2 * i + 1];
    rs += (unsigned long long)ar.x | ((unsigned long long)ar.y << 32);
    const unsigned long long sm = (unsigned long long)a.x | ((unsigned long long)a.y << 32);
    const uint32_t q[3] = {a.z & 255u, (a.z >> 8) & 255u, (a.z >> 16) & 255u};
    ts += sm;
    if (i < g) ps += sm;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      tq[k] += q[k];
      if (i < g) pq[k] += q[k];
    }
    mx = max(mx, a.w);
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    ps += __shfl_xor(ps, d, 64);
    ts += __shfl_xor(ts, d, 64);
    rs += __shfl_xor(rs, d, 64);
    mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pq[k] += __shfl_xor(pq[k], d, 64);
      tq[k] += __shfl_xor(tq[k], d, 64);
    }
  }
  if (lane == 0) {
    s_sum[0][wave] = ps;
    s_sum[1][wave] = ts;
    s_sum[2][wave] = rs;
    s_mx[wave] = mx;
    for (int k = 0; k < 3; ++k) {
      s_q[0][wave][k] = pq[k];
      s_q[1][wave][k] = tq[k];
    }
  }
  __syncthreads();
  ps = s_sum[0][0] + s_sum[0][1] + s_sum[0][2] + s_sum[0][3];
  ts = s_sum[1][0] + s_sum[1][1] + s_sum[1][2] + s_sum[1][3];
  rs = s_sum[2][0] + s_sum[2][1] + s_sum[2][2] + s_sum[2][3];
  for (int k = 0; k < 3; ++k) {
    pq[k] = s_q[0][0][k] + s_q[0][1][k] + s_q[0][2][k] + s_q[0][3][k];
    tq[k] = s_q[1][0][k] + s_q[1][1][k] + s_q[1][2][k] + s_q[1][3][k];
  }
  mx = max(max(s_mx[0], s_mx[1]), max(s_mx[2], s_mx[3]));
  if (wave == 0) {
    const int t = g * 64 + lane;
    const bool ok = t < T;
    const uint32_t c = ok ? b.tile_count[t] : 0u;
    unsigned long long inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    const unsigned long long start = ps + inc - c;
    const int cl = sort_class(c);
    const unsigned long long lt = (1ull << lane) - 1ull;
    const unsigned long long m0 = ballot64(ok && cl == 0), m1 = ballot64(ok && cl == 1),
                             m2 = ballot64(ok && cl == 2);
    if (ok) {
      b.tile_start[t] = (uint32_t)(start < 0xFFFFFFFFull ? start : 0xFFFFFFFFull);
      if (cl == 0) b.small_tiles[pq[0] + (uint32_t)__popcll(m0 & lt)] = (uint32_t)t;
      if (cl == 1) b.medium_tiles[pq[1] + (uint32_t)__popcll(m1 & lt)] = (uint32_t)t;
      if (cl == 2) b.big_tiles[pq[2] + (uint32_t)__popcll(m2 & lt)] = (uint32_t)t;
      if (b.tile_big) b.tile_big[t] = cl == 2 ? pq[2] + (uint32_t)__popcll(m2 & lt) : 0xFFFFFFFFu;
    }
  }
  if (g == 0) {  // frame counters (every counter of the frame is reset here)
    uint32_t vsum = 0;
    const int nb = (fp.n + 255) / 256;
    for (int i0 = 0; i0 < nb; i0 += 256 * 8) {  // 8 independent loads in flight per thread
      uint32_t vr[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = i0 + k * 256 + tid;
        vr[k] = i < nb ? b.block_rendered[i] : 0u;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) vsum += vr[k];
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) vsum += __shfl_xor(vsum, d, 64);
    __syncthreads();
    if (lane == 0) s_mx[wave] = vsum;
    __syncthreads();
    if (tid == 0) {
      b.counters[0] = tq[2];
      b.counters[1] = 0;
      b.counters[2] = s_mx[0] + s_mx[1] + s_mx[2] + s_mx[3];
      b.counters[3] = ts > fp.pair_cap ? 1u : 0u;
      if (ts > fp.pair_cap) {  // sticky until the host's sync
        *b.host_sticky = 1u;
        if (b.group_sticky) *b.group_sticky = 1u;
      }
      b.counters[4] = mx;
      b.counters[5] = (uint32_t)ts;
      b.counters[6] = (uint32_t)(ts >> 32);
      b.counters[7] = tq[1];
      b.counters[8] = 0;
      b.counters[9] = tq[0];
      b.counters[10] = (uint32_t)rs;
      b.counters[11] = (uint32_t)(rs >> 32);
      for (int k = 12; k < 16; ++k) b.counters[k] = 0;
      b.tile_start[T] = (uint32_t)(ts < 0xFFFFFFFFull ? ts : 0xFFFFFFFFull);
      for (int k = 0; k < 16; ++k) b.host_counters[k] = b.counters[k];
      if (b.footer)
        for (int k = 0; k < 16; ++k) b.footer[k] = b.counters[k];
    }
  }
}

__global__ __launch_bounds__(1024) void gs_emit_chunk_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrEmitChunk);
  extern __shared__ __attribute__((aligned(16))) uint32_t cnt[];
  const int T = fp.n_tiles;
  const int c = blockIdx.x;
  const int g0 = c * fp.chunk_size;
  const int g1 = min(fp.n, g0 + fp.chunk_size);
  const uint32_t* row = b.chunk_off + (size_t)c * T;
  const int lane = threadIdx.x & 63;
  if (fp.emit_wide) {
    // one u32 cursor per tile, seeded with the chunk's first slot of the
    // tile: a single LDS atomic returns the pair's final position
    for (int t0 = 0; t0 < T; t0 += 1024 * 8) {  // loads first: 16 in flight per thread
      uint32_t st[8], ro[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int t = t0 + k * 1024 + (int)threadIdx.x;
        st[k] = t < T ? b.tile_start[t] : 0u;
        ro[k] = t < T ? row[t] : 0u;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int t = t0 + k * 1024 + (int)threadIdx.x;
        if (t < T) cnt[t] = st[k] + ro[k];
      }
    }
    __syncthreads();
    const uint2* __restrict__ rects = fp.pair_cull ? b.crect : b.rect;
    for (int i0 = g0; i0 < g1; i0 += 4096) {  // 4 Gaussians per thread, loaded up front
      uint2 r[4];
      uint32_t dk[4];
      bool live[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = i0 + k * 1024 + (int)threadIdx.x;
        live[k] = i < g1 && block_live(fp, b, i);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = i0 + k * 1024 + (int)threadIdx.x;
        if (fp.rect8)
          r[k] = rect8_unpack(live[k] ? reinterpret_cast<const uint32_t*>(b.crect)[i] : 0x00010001u);
        else
          r[k] = live[k] ? rects[i] : kEmptyRect;
        dk[k] = live[k] ? b.depth_key[i] : 0u;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // Runs of equal rectangles among the wave's lanes (consecutive
        // Gaussians in Morton order often bin into the same tiles, as in the
        // count): the run's first lane reserves the run's slots in each tile
        // with one LDS atomic and the run's lanes take consecutive slots
        // (coalesced 8-B stores).  The run's lanes share the rectangle, so
        // they walk the tile loops in step and the leader's reservation is
        // read in the same iteration.  Slots within a tile are the atomics'
        // order either way; the sort sets the list order.
        const uint2 rk = r[k];
        const uint32_t px = (uint32_t)__shfl_up((int)rk.x, 1, 64), py = (uint32_t)__shfl_up((int)rk.y, 1, 64);
        const bool start = lane == 0 || rk.x != px || rk.y != py;
        const unsigned long long st = ballot64(start);
        const unsigned long long upto = lane == 63 ? st : (st & ((2ull << lane) - 1ull));
        const int leader = 63 - __builtin_clzll(upto);  // (bit 0 is always set)
        const unsigned long long above = lane == 63 ? 0ull : (st & ~((2ull << lane) - 1ull));
        const uint32_t len = above ? (uint32_t)(__builtin_ctzll(above) - lane) : (uint32_t)(64 - lane);
        const uint32_t rank = (uint32_t)(lane - leader);
        const uint32_t x0 = rk.x & 0xFFFFu, x1 = rk.x >> 16, y0 = rk.y & 0xFFFFu, y1 = rk.y >> 16;
        const unsigned long long key = ((unsigned long long)dk[k] << 32) | (uint32_t)(i0 + k * 1024 + (int)threadIdx.x);
        if (x0 > x1) continue;
        for (uint32_t y = y0; y <= y1; ++y)
          for (uint32_t x = x0; x <= x1; ++x) {
            uint32_t base = 0u;
            if (start) base = atomicAdd(&cnt[y * fp.tiles_x + x], len);
            base = (uint32_t)__builtin_amdgcn_ds_bpermute(leader << 2, (int)base);
            const uint32_t pos = base + rank;
            if (pos < fp.pair_cap) b.pairs[pos] = key;
          }
      }
    }
    return;
  }
  lds_zero(cnt, (T + 1) >> 1);
  __syncthreads();
  for (int i = g0 + (int)threadIdx.x; i < g1; i += 1024) {
    if (!block_live(fp, b, i)) continue;
    const uint2 r = fp.pair_cull ? b.crect[i] : b.rect[i];
    const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
    if (x0 > x1) continue;
    const unsigned long long key = ((unsigned long long)b.depth_key[i] << 32) | (uint32_t)i;
    for (uint32_t y = y0; y <= y1; ++y)
      for (uint32_t x = x0; x <= x1; ++x) {
        const uint32_t t = y * fp.tiles_x + x;
        const uint32_t sh = (t & 1u) * 16u;
        const uint32_t slot = (atomicAdd(&cnt[t >> 1], 1u << sh) >> sh) & 0xFFFFu;
        const uint32_t pos = b.tile_start[t] + row[t] + slot;
        if (pos < fp.pair_cap) b.pairs[pos] = key;
      }
  }
}

// --------------------------------------------------------------------- emit
// Fallback emit (tile grids too large for an LDS histogram): global cursors.
__global__ __launch_bounds__(256) void gs_emit_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrEmit);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= fp.n) return;
  if (!block_live(fp, b, i)) return;
  const uint2 r = b.rect[i];
  const uint32_t x0 = r.x & 0xFFFFu, x1 = r.x >> 16, y0 = r.y & 0xFFFFu, y1 = r.y >> 16;
  if (x0 > x1) return;
  const unsigned long long key = ((unsigned long long)b.depth_key[i] << 32) | (uint32_t)i;
  for (uint32_t y = y0; y <= y1; ++y)
    for (uint32_t x = x0; x <= x1; ++x) {
      const uint32_t pos = atomicAdd(&b.tile_cursor[y * fp.tiles_x + x], 1u);
      if (pos < fp.pair_cap) b.pairs[pos] = key;
    }
}

// --------------------------------------------------------------------- sort
// DIRECT (FrameParams::bin_direct frames, gs_blend_direct_kernel only): the
// tile's fixed segment; its pairs past the segment were dropped (overflow)
template <bool DIRECT = false>
__device__ __forceinline__ void tile_segment(const FrameParams& fp, const Buffers& b, int t,
                                             uint32_t& s, uint32_t& L) {
  if constexpr (DIRECT) {  // (the segment of the view's last scan; the list this frame placed in it)
    const uint32_t c = (uint32_t)b.tile_cnt64[t];
    const uint32_t en = direct_limit(fp, b, (uint32_t)t);
    uint32_t st = b.tile_start[t];
    if (st > en) st = en;
    s = st;
    L = c < en - st ? c : en - st;
    return;
  }
  uint32_t st = b.tile_start[t], en = b.tile_start[t + 1];
  const unsigned long long cap = fp.pair_cap;
  if (en > cap) en = (uint32_t)cap;
  if (st > en) st = en;
  s = st;
  L = en - st;
}

// Register bitonic sort of E*64 keys held by one wave: element i = lane*E + e
// (each lane owns E consecutive keys).  Strides < E compare two registers of
// the same lane; strides >= E exchange register e with lane ^ (j / E)
// (ds_bpermute).  No LDS arrays, no barriers.  The k / j loops stay rolled (the
// network runs once per wave); wave_bitonic unrolls the whole network at
// compile time for E <= GS_SORT_UNROLL_E.
template <int E, int J>
__device__ __forceinline__ void reg_stage(unsigned long long (&v)[E], int i0, int k) {
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int pe = e ^ J;
    if (pe > e) {
      const bool asc = ((i0 + e) & k) == 0;  // i0 = global index of the lane's first key
      const unsigned long long a = v[e], c = v[pe];
      const bool sw = (a > c) == asc;
      v[e] = sw ? c : a;
      v[pe] = sw ? a : c;
    }
  }
}

// Value of lane ^ lj (lj = 1 .. 32, wave-uniform) without an LDS round trip:
// DPP quad_perm for 1 / 2, bank-masked row_shl / row_shr for 4, row_ror for 8,
// v_permlane16_swap / v_permlane32_swap for 16 / 32.
template <int LJ>
__device__ __forceinline__ uint32_t xor_lane_u32(uint32_t x, int lane) {
  if constexpr (LJ == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  } else if constexpr (LJ == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  } else if constexpr (LJ == 4) {
    // row_shl:4 into banks 0 / 2 (lanes 0-3, 8-11 of a row), row_shr:4 into
    // banks 1 / 3: two DPP moves, no select
    const int up = __builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xF, 0x5, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(up, (int)x, 0x114, 0xF, 0xA, false);
  } else if constexpr (LJ == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
  } else if constexpr (LJ == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (lane & 16) ? p[0] : p[1];
  } else {
    const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (lane & 32) ? p[0] : p[1];
  }
}

template <int LJ>
__device__ __forceinline__ unsigned long long xor_lane_u64(unsigned long long x, int lane) {
  const uint32_t lo = xor_lane_u32<LJ>((uint32_t)x, lane);
  const uint32_t hi = xor_lane_u32<LJ>((uint32_t)(x >> 32), lane);
  return ((unsigned long long)hi << 32) | lo;
}

// One cross-lane stage: every register exchanged with lane ^ LJ.
template <int E, int LJ>
__device__ __forceinline__ void lane_stage(unsigned long long (&v)[E], int lane, int ibase, int k) {
  const bool lower = (lane & LJ) == 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = ibase + lane * E + e;
    const unsigned long long o = xor_lane_u64<LJ>(v[e], lane);
    const bool asc = (i & k) == 0;
    const bool take_min = lower == asc;
    const bool gt = v[e] > o;
    v[e] = (take_min == gt) ? o : v[e];
  }
}

// In-wave stages j = jmax .. 1 of bitonic step k; ibase = global index of this
// wave's first key (the direction of a compare depends on the global index).
template <int E>
__device__ __forceinline__ void wave_merge(unsigned long long (&v)[E], int lane, int ibase, int k,
                                           int jmax) {
  for (int j = jmax; j > 0; j >>= 1) {
    if (j < E) {
      const int i0 = ibase + lane * E;
      switch (j) {
        case 1: if constexpr (E > 1) reg_stage<E, 1>(v, i0, k); break;
        case 2: if constexpr (E > 2) reg_stage<E, 2>(v, i0, k); break;
        case 4: if constexpr (E > 4) reg_stage<E, 4>(v, i0, k); break;
        default: break;
      }
    } else {
      switch (j / E) {
        case 1: lane_stage<E, 1>(v, lane, ibase, k); break;
        case 2: lane_stage<E, 2>(v, lane, ibase, k); break;
        case 4: lane_stage<E, 4>(v, lane, ibase, k); break;
        case 8: lane_stage<E, 8>(v, lane, ibase, k); break;
        case 16: lane_stage<E, 16>(v, lane, ibase, k); break;
        default: lane_stage<E, 32>(v, lane, ibase, k); break;
      }
    }
  }
}

// Fully unrolled network (E <= 2: 21 or 28 stages, short enough to unroll):
// stage (K, J) of step K, compile-time, no per-stage branches.
template <int E, int K, int J>
struct BitonicStages {
  __device__ __forceinline__ static void run(unsigned long long (&v)[E], int lane) {
    if constexpr (J < E) {
      reg_stage<E, J>(v, lane * E, K);
    } else {
      lane_stage<E, J / E>(v, lane, 0, K);
    }
    if constexpr (J > 1) BitonicStages<E, K, J / 2>::run(v, lane);
  }
};
template <int E, int K>
struct BitonicSteps {
  __device__ __forceinline__ static void run(unsigned long long (&v)[E], int lane) {
    BitonicStages<E, K, K / 2>::run(v, lane);
    if constexpr (2 * K <= 64 * E) BitonicSteps<E, 2 * K>::run(v, lane);
  }
};

template <int E>
__device__ __forceinline__ void wave_bitonic(unsigned long long (&v)[E], int lane) {
  constexpr int n = E * 64;
  if constexpr (E <= GS_SORT_UNROLL_E) {
    BitonicSteps<E, 2>::run(v, lane);
  } else {
    for (int k = 2; k <= n; k <<= 1) wave_merge<E>(v, lane, 0, k, k >> 1);
  }
}

// Keys: (orderable clip z << 32) | device index, as the emit writes them.
// The list order is (z, INPUT index) (the oracle's stable order), which the
// device index gives too except among equal depths (the device order is 3D
// Morton).  So a sorted list is checked for neighbours of equal depth; only a
// list that has some (rare: exactly equal clip z in one tile) is re-keyed with
// the input index (perm[]) and sorted again, and its list written through
// inv_perm[].  The common case writes the low words: no gather.
constexpr unsigned long long kDepthMask = 0xFFFFFFFF00000000ull;

__device__ __forceinline__ unsigned long long rekey_input(const Buffers& b, unsigned long long k) {
  return (k & kDepthMask) | b.perm[(uint32_t)k];
}

// Writes the list of sorted device-index keys k[0, L) (positions t, t + stride,
// ... of this thread).  A key without an equal-depth neighbour is in place.
// A run of equal depths shorter than kTieRun is put in input-index order: a
// member's place is the run's start plus its input index's rank within the
// run (perm[], only for these).  Returns true when this thread met a longer
// run (e.g. a plane facing the camera): the caller re-sorts the list.  At
// 1M/1080p clip z has only 943 k distinct values over 1M Gaussians; 182 of
// the 8160 lists have equal depths, nearly all in runs of 2 (re-sorting those
// lists cost the sort launch 13 us).
constexpr uint32_t kTieRun = 16;

__device__ __forceinline__ bool write_tied_list(const Buffers& b, uint32_t s, uint32_t L,
                                                const unsigned long long* k, uint32_t t,
                                                uint32_t stride) {
  bool longrun = false;
  for (uint32_t p = t; p < L; p += stride) {
    const unsigned long long kp = k[p];
    const uint32_t hi = (uint32_t)(kp >> 32);
    const bool tp = p > 0u && (uint32_t)(k[p - 1] >> 32) == hi;
    const bool tn = p + 1u < L && (uint32_t)(k[p + 1] >> 32) == hi;
    if (!tp && !tn) {
      b.list[s + p] = (uint32_t)kp;
      continue;
    }
    uint32_t a = p, e = p + 1u;
    while (a > 0u && p - a < kTieRun && (uint32_t)(k[a - 1] >> 32) == hi) --a;
    while (e < L && e - p < kTieRun && (uint32_t)(k[e] >> 32) == hi) ++e;
    if (e - a >= kTieRun) {
      longrun = true;
      continue;
    }
    const uint32_t me = b.perm[(uint32_t)kp];
    uint32_t rank = 0;
    for (uint32_t j = a; j < e; ++j) rank += b.perm[(uint32_t)k[j]] < me ? 1u : 0u;
    b.list[s + a + rank] = (uint32_t)kp;
  }
  return longrun;
}

// The rare path of a small list with equal depths: input-index keys, the
// rolled network, one copy for every E (the hot unrolled networks stay
// compact in the instruction cache: a copy per E inside them doubled the
// kernel's code and cost the isolated sort 13 us).
__device__ __forceinline__ void wave_sort_tile_input(const Buffers& b, const unsigned long long* src,
                                                     uint32_t s, uint32_t L, int lane) {
  constexpr int E = 4;  // L <= kSortRegCap = 256
  unsigned long long v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t i = (uint32_t)(lane * E + e);
    v[e] = i < L ? rekey_input(b, src[i]) : ~0ull;
  }
  for (int k = 2; k <= 64 * E; k <<= 1) wave_merge<E>(v, lane, 0, k, k >> 1);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t i = (uint32_t)(lane * E + e);
    if (i < L) b.list[s + i] = b.inv_perm[(uint32_t)v[e]];
  }
}

// Sorts the keys src[0, L) and writes the list at list[s, s + L).  Returns
// false (nothing written; the sorted keys are left in slice[0, L)) when the
// list has equal depths.
template <int E>
__device__ __forceinline__ bool wave_sort_tile(const Buffers& b, const unsigned long long* src, uint32_t s,
                                               uint32_t L, int lane, unsigned long long* slice) {
  unsigned long long v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t i = (uint32_t)(lane * E + e);
    v[e] = i < L ? src[i] : ~0ull;
  }
  wave_bitonic<E>(v, lane);
  // key i - 1 of key i: this lane's previous register, or lane - 1's last
  const uint32_t prev_hi = (uint32_t)__shfl_up((int)(uint32_t)(v[E - 1] >> 32), 1, 64);
  bool tie = false;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t i = (uint32_t)(lane * E + e);
    const uint32_t ph = e > 0 ? (uint32_t)(v[e - 1] >> 32) : prev_hi;
    tie = tie || (i > 0u && i < L && ph == (uint32_t)(v[e] >> 32));
  }
  if (ballot64(tie) != 0ull) {
#pragma unroll
    for (int e = 0; e < E; ++e) slice[lane * E + e] = v[e];
    return false;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t i = (uint32_t)(lane * E + e);
    if (i < L) b.list[s + i] = (uint32_t)v[e];
  }
  return true;
}

// Medium lists (kSortRegCap < L <= kSortLdsCap), one NT-thread workgroup:
// the waves sort RUN = 64 E-key runs in registers (wave_bitonic<E>), then
// log2(runs) merge-path levels run in LDS.  At every level each thread
// produces K = ceil(npad / NT) consecutive outputs: a co-rank binary search
// finds where its first output comes from, then it merges sequentially,
// holding the outputs in registers across the barrier (the merge is in
// place).  The last level writes the list.  Work is O(L log L) over L rounded
// up to RUN, against O(L log^2 L) over L rounded up to a power of two for a
// bitonic network.  E = 2 (128-key runs, one more merge level than 256-key
// runs): the register bitonic phase was 80 % of a medium sort (per-workgroup
// timestamps, tools/sort_times.py), and E = 2 took the sort from 45.0 to
// 43.2 us; E = 1 took 49.1.
// SRC: where the keys come from (kSrcPairs: the tile's pairs; kSrcRekey: the
// pairs re-keyed with the input index; kSrcLds: lds[0, L) already holds them;
// kSrcAlt: pairs_alt; kSrcAltRekey: pairs_alt re-keyed).  kOutLds leaves the
// sorted keys in lds[0, L).
// OUT: kOutKeys writes the sorted keys back to the pairs (a big list's
// segment); kOutInput writes the list from input-index keys (inv_perm);
// kOutDevice writes the list from device-index keys, checking equal depths
// first (see wave_sort_tile) and re-sorting with input-index keys if any.
// kOutDevice returns false (nothing written) when the list has equal depths.
enum { kSrcPairs = 0, kSrcRekey = 1, kSrcLds = 2, kSrcAlt = 3, kSrcAltRekey = 4 };
enum { kOutKeys = 0, kOutInput = 1, kOutDevice = 2, kOutLds = 3 };

template <int NT, int E, int OUT, int SRC = kSrcPairs>
__device__ __forceinline__ bool merge_sort_tile(const Buffers& b, uint32_t s, uint32_t L,
                                                unsigned long long* lds) {
  constexpr int RUN = 64 * E, NW = NT / 64;
  constexpr int KMAX = (kSortLdsCap + NT - 1) / NT;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int runs = (int)((L + (uint32_t)RUN - 1u) / (uint32_t)RUN);
  const int npad = runs * RUN;
  for (int r = wave; r < runs; r += NW) {
    unsigned long long v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t i = (uint32_t)(r * RUN + lane * E + e);
      if constexpr (SRC == kSrcRekey) v[e] = i < L ? rekey_input(b, b.pairs[s + i]) : ~0ull;
      else if constexpr (SRC == kSrcLds) v[e] = i < L ? lds[i] : ~0ull;  // run r: this wave's own slots
      else if constexpr (SRC == kSrcAlt) v[e] = i < L ? b.pairs_alt[s + i] : ~0ull;
      else if constexpr (SRC == kSrcAltRekey) v[e] = i < L ? rekey_input(b, b.pairs_alt[s + i]) : ~0ull;
      else v[e] = i < L ? b.pairs[s + i] : ~0ull;
    }
    wave_bitonic<E>(v, lane);
#pragma unroll
    for (int e = 0; e < E; ++e) lds[r * RUN + lane * E + e] = v[e];
  }
  __syncthreads();
  const int K = (npad + NT - 1) / NT;
  const int d0 = (int)threadIdx.x * K;
  for (int w = RUN;; w <<= 1) {  // runs == 1 degenerates to a copy
    unsigned long long out[KMAX];
    int i = 0, j = 0, la = 0, lb = 0, abase = 0, bbase = 0;
    unsigned long long av = 0ull, bv = 0ull;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int d = d0 + k;
      if (k < K && d < npad) {
        if (k == 0 || (d & (2 * w - 1)) == 0) {  // (re)locate: first output or a new pair
          abase = d & ~(2 * w - 1);
          bbase = abase + w;
          la = min(w, npad - abase);
          lb = max(0, min(w, npad - bbase));
          const int dd = d - abase;
          int lo = max(0, dd - lb), hi = min(dd, la);
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (lds[abase + mid] <= lds[bbase + dd - 1 - mid]) lo = mid + 1;
            else hi = mid;
          }
          i = lo;
          j = dd - lo;
          av = i < la ? lds[abase + i] : ~0ull;
          bv = j < lb ? lds[bbase + j] : ~0ull;
        }
        const bool ta = j >= lb || (i < la && av <= bv);
        out[k] = ta ? av : bv;
        if (ta) {
          ++i;
          av = i < la ? lds[abase + i] : ~0ull;
        } else {
          ++j;
          bv = j < lb ? lds[bbase + j] : ~0ull;
        }
      }
    }
    __syncthreads();
    if (2 * w < npad || OUT == kOutDevice || OUT == kOutLds) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K && d0 + k < npad) lds[d0 + k] = out[k];
      __syncthreads();
      if (2 * w < npad) continue;
    } else {
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < K && d0 + k < (int)L) {
          if constexpr (OUT == kOutKeys) b.pairs[s + d0 + k] = out[k];  // a big list's sorted segment
          else b.list[s + d0 + k] = b.inv_perm[(uint32_t)out[k]];
        }
      return true;
    }
    break;
  }
  if constexpr (OUT == kOutDevice) {
    // the sorted keys are in lds[0, L)
    if (__syncthreads_or(write_tied_list(b, s, L, lds, threadIdx.x, NT))) return false;
  }
  return true;
}

// Large lists (> kSortLdsCap, clustered scenes): a block-wide stable LSD
// radix sort (8 x 8-bit passes) over the tile's segment in global memory,
// pairs <-> pairs_alt, by one NT-thread workgroup.  One sweep first builds the
// digit histograms of all 8 passes (the histogram of a digit does not depend
// on the order); passes whose digit is the same for every key are skipped.
// A pass walks the list in rounds of NT * KPL keys: wave w takes the round's
// keys [w * 64 KPL, (w + 1) * 64 KPL) in KPL steps of 64, all loaded up front,
// and ranks each step with a wave64 ballot multisplit (8 ballots give each
// lane the mask of lanes with its digit) plus the wave's running per-digit
// count in LDS; one cross-wave prefix per digit and the scatter follow, so a
// round costs 3 barriers (the first version ranked 256 keys per 4 barriers,
// with each chunk's global load exposed: 5.4 ms per frame on config 5's
// 162 k-key tiles).
// The device-index keys [s, s + L) of the pairs (FROM_ALT: of pairs_alt) are
// re-keyed with the input index into the other buffer and sorted there; the
// list [s, s + L) is written.
template <int NT, int KPL, bool FROM_ALT>
__device__ __forceinline__ void radix_sort_seg(const Buffers& b, uint32_t s, uint32_t L,
                                               uint32_t* hist, uint32_t* base,
                                               uint32_t (*wcnt)[256]) {
  constexpr int NW = NT / 64, RK = NT * KPL;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  unsigned long long* src = (FROM_ALT ? b.pairs : b.pairs_alt) + s;
  unsigned long long* dst = (FROM_ALT ? b.pairs_alt : b.pairs) + s;
  // input-index keys (the order among equal depths), written to the other
  // buffer and sorted from there
  for (uint32_t i = tid; i < L; i += NT) src[i] = rekey_input(b, dst[i]);
  // hist[p * 256 + d]: keys whose pass-p digit is d (one sweep for all passes)
  for (int k = tid; k < 8 * 256; k += NT) hist[k] = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < L; c0 += RK) {
    unsigned long long key[KPL];
#pragma unroll
    for (int e = 0; e < KPL; ++e) {
      const uint32_t i = c0 + (uint32_t)(e * NT + tid);
      key[e] = i < L ? src[i] : 0ull;
    }
#pragma unroll
    for (int e = 0; e < KPL; ++e) {
      if (c0 + (uint32_t)(e * NT + tid) < L) {
#pragma unroll
        for (int p = 0; p < 8; ++p) atomicAdd(&hist[p * 256 + ((uint32_t)(key[e] >> (8 * p)) & 255u)], 1u);
      }
    }
  }
  __syncthreads();
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = pass * 8;
    const uint32_t* h = hist + pass * 256;
    const bool trivial = L == 0 || h[(uint32_t)(src[0] >> shift) & 255u] == L;
    if (trivial) continue;  // every key has the same digit: order unchanged (uniform branch)
    if (wave == 0) {  // exclusive scan of 256 bins, 4 per lane
      uint32_t v[4], tot = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] = h[lane * 4 + k];
        tot += v[k];
      }
      uint32_t inc = tot;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
      }
      uint32_t run = inc - tot;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        base[lane * 4 + k] = run;
        run += v[k];
      }
    }
    __syncthreads();
    for (uint32_t c0 = 0; c0 < L; c0 += RK) {
      const uint32_t w0 = c0 + (uint32_t)(wave * 64 * KPL);
      unsigned long long key[KPL];
#pragma unroll
      for (int e = 0; e < KPL; ++e) {
        const uint32_t i = w0 + (uint32_t)(e * 64 + lane);
        key[e] = i < L ? src[i] : 0ull;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) wcnt[wave][lane * 4 + k] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      uint32_t rank[KPL];
#pragma unroll
      for (int e = 0; e < KPL; ++e) {
        const bool valid = w0 + (uint32_t)(e * 64 + lane) < L;
        const uint32_t d = (uint32_t)(key[e] >> shift) & 255u;
        unsigned long long m = ballot64(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
          const bool set = (d >> bit) & 1u;
          const unsigned long long bb = ballot64(set);
          m &= set ? bb : ~bb;
        }
        const uint32_t before = wcnt[wave][d];
        rank[e] = before + (uint32_t)__popcll(m & lt_mask);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (valid && (m & lt_mask) == 0ull) wcnt[wave][d] = before + (uint32_t)__popcll(m);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      __syncthreads();
      uint32_t round_tot = 0;  // NT >= 256: one digit per thread
      for (int k = tid; k < 256; k += NT) {
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const uint32_t c = wcnt[w][k];
          wcnt[w][k] = run;
          run += c;
        }
        round_tot = run;
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < KPL; ++e) {
        const uint32_t d = (uint32_t)(key[e] >> shift) & 255u;
        if (w0 + (uint32_t)(e * 64 + lane) < L) dst[base[d] + wcnt[wave][d] + rank[e]] = key[e];
      }
      __syncthreads();
      if (tid < 256) base[tid] += round_tot;
      __syncthreads();
    }
    unsigned long long* tmp = src;
    src = dst;
    dst = tmp;
  }
  for (uint32_t i = tid; i < L; i += NT) b.list[s + i] = b.inv_perm[(uint32_t)src[i]];
}

template <int NT, int KPL, bool DIRECT = false>
__device__ __forceinline__ void radix_sort_tile(const FrameParams& fp, const Buffers& b, int t,
                                                uint32_t* hist, uint32_t* base,
                                                uint32_t (*wcnt)[256]) {
  uint32_t s, L;
  tile_segment<DIRECT>(fp, b, t, s, L);
  radix_sort_seg<NT, KPL, false>(b, s, L, hist, base, wcnt);
}

// One wave sorts a list of L <= kSortRegCap keys src[0, L) in registers and
// writes it at list[s, s + L) (equal depths: see write_tied_list).
// (EMAX: the largest register network compiled in -- L <= 64 EMAX keys)
template <int EMAX = 4>
__device__ __forceinline__ void wave_sort_list(const Buffers& b, const unsigned long long* src, uint32_t s,
                                               uint32_t L, int lane, unsigned long long* slice) {
  bool done;
  if constexpr (EMAX == 1) {
    done = wave_sort_tile<1>(b, src, s, L, lane, slice);
  } else {
    if (L <= 64u)
      done = wave_sort_tile<1>(b, src, s, L, lane, slice);
    else if (L <= 128u)
      done = wave_sort_tile<2>(b, src, s, L, lane, slice);
    else
      done = wave_sort_tile<4>(b, src, s, L, lane, slice);
  }
  if (!done) {  // equal depths (wave-uniform)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool longrun = write_tied_list(b, s, L, slice, (uint32_t)lane, 64u);
    if (ballot64(longrun) != 0ull) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // after the stores above
      wave_sort_tile_input(b, src, s, L, lane);
    }
  }
}

// Big, medium and small lists in one launch, longest first: workgroups
// [0, n_big) radix-sort one big list each (> kSortLdsCap); the next n_medium
// each sort one medium list (kSortRegCap < L <= kSortLdsCap, merge_sort_tile);
// the rest give each of their waves one small list (L <= kSortRegCap, sorted
// in one wave's registers).  Keys are unique (the input index is in the low
// word), so the order is total and deterministic.  NT = 256: 8 workgroups
// per CU.  (1024-thread workgroups, 16 waves per list, cut a 1000-key list's
// sort from ~24 to ~12 us when alone, but hold one workgroup per CU and ran
// no faster in a row band and 2.4x slower on the full frame.)
template <int NT>
__device__ __forceinline__ void sort_tiles(const FrameParams& fp, const Buffers& b) {
  constexpr int NW = NT / 64;
  // the radix path's histograms alias the merge path's key buffer (a
  // workgroup takes one path)
  constexpr int kRadixWords = 8 * 256 + 256 + NW * 256;
  constexpr int kWords = 2 * kSortLdsCap > kRadixWords ? 2 * kSortLdsCap : kRadixWords;
  __shared__ unsigned long long keys[kWords / 2];
  uint32_t* const r_hist = (uint32_t*)keys;
  uint32_t* const r_base = r_hist + 8 * 256;
  uint32_t(*const r_wcnt)[256] = (uint32_t(*)[256])(r_hist + 9 * 256);
  // big lists: radix-sorted here (4 keys per lane and round) unless the
  // segmented merge sort has taken them this frame (FrameParams::big_separate)
  const uint32_t n_big = fp.big_separate ? 0u : b.counters[0];
  // FrameParams::blend_seg: each list's (tile, start, length) at its blend
  // slot (the queues' order: big, medium, small)
  auto put_seg = [&](uint32_t slot, uint32_t t, uint32_t s, uint32_t L) {
    if (fp.blend_seg && (threadIdx.x & 63) == 0) b.blend_seg[slot] = make_uint4(t, s, L, 0u);
  };
  if (blockIdx.x < n_big) {  // the longest lists first
    const uint32_t t = b.big_tiles[blockIdx.x];
    if (fp.blend_seg && threadIdx.x == 0) {
      uint32_t s, L;
      tile_segment(fp, b, (int)t, s, L);
      put_seg(blockIdx.x, t, s, L);
    }
    radix_sort_tile<NT, 4>(fp, b, (int)t, r_hist, r_base, r_wcnt);
    return;
  }
  const uint32_t n_med = b.counters[7], n_small = b.counters[9];
  const uint32_t item = blockIdx.x - n_big;
  if (item < n_med) {
    uint32_t s, L;
    const uint32_t t = b.medium_tiles[item];
    tile_segment(fp, b, (int)t, s, L);
    if (threadIdx.x == 0) put_seg(n_big + item, t, s, L);
    if (!merge_sort_tile<NT, 2, kOutDevice>(b, s, L, keys)) {
      __syncthreads();  // a long run of equal depths: again with input-index keys
      merge_sort_tile<NT, 2, kOutInput, kSrcRekey>(b, s, L, keys);
    }
    return;
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t k = (item - n_med) * (uint32_t)NW + (uint32_t)wave;
  if (k >= n_small) return;
  const int lane = threadIdx.x & 63;
  uint32_t s, L;
  const uint32_t t = b.small_tiles[k];
  tile_segment(fp, b, (int)t, s, L);
  put_seg(n_big + n_med + k, t, s, L);
  // this wave's slice of the (here unused) merge buffer, for a list with
  // equal depths
  static_assert(NW * kSortRegCap <= kWords / 2, "small-list slices fit the merge buffer");
  unsigned long long* const slice = keys + wave * kSortRegCap;
  wave_sort_list(b, b.pairs + s, s, L, lane, slice);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_sort_tiles_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrSortTiles);
  sort_tiles<256>(fp, b);
}

// ---- big lists as a segmented merge sort over many workgroups
// (FrameParams::big_separate).  A list > kSortLdsCap is cut into 2048-key
// segments; every segment is sorted by one workgroup (the medium path, keys
// written back in place), then merge passes p = 0, 1, ... each merge pairs of
// sorted runs of 2048 << p keys, pairs <-> pairs_alt, every workgroup making
// 2048 outputs of one list (merge path: two co-rank searches in global memory,
// the two input ranges staged in LDS, 8 outputs per thread).  The pass whose
// pair covers the whole list writes the list itself (device indices); later
// passes skip it.  Work items are (big list j, segment c), numbered through
// big_chunk_off (tile_cursor, unused by the chunked binning) and walked
// grid-stride, so any grid size is correct.
constexpr int kBigSeg = 2048;

// sample sort of the big lists: buckets of ~kBktAvg keys, at most kBktMax
// per list (their splitters are staged in LDS)
constexpr uint32_t kBktAvg = 1024, kBktMax = 2048;
// lazy big lists: the sorted prefix holds ~this many keys (see gs_big_select_kernel);
// the continuation's window the next ~kLazyWindow (gs_big_cont_kernel)
constexpr uint32_t kLazyPrefix = 1024, kLazyWindow = 1536;
__device__ __forceinline__ uint32_t big_buckets(uint32_t L) {
  return min(kBktMax, (L + kBktAvg - 1u) / kBktAvg);
}

// one workgroup: segment counts of the big lists -> exclusive prefix
__global__ __launch_bounds__(1024) void gs_big_prefix_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  __shared__ uint32_t wsum[16], wsum_b[16];
  __shared__ uint32_t s_maxl;
  const uint32_t n_big = b.counters[0];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool keep_buckets = fp.lazy && fp.big_pass != 0;
  // pass 2: nothing to do unless a continuation wave outlived its window
  if (fp.big_pass == 2 && b.counters[1] == 0u) {
    if (tid == 0) b.counters[12] = 0u;
    return;
  }
  if (tid == 0) s_maxl = 0;
  uint32_t carry = 0, carry_b = 0, maxl = 0;
  for (uint32_t j0 = 0; j0 < n_big; j0 += 1024) {
    const uint32_t j = j0 + (uint32_t)tid;
    uint32_t c = 0, nb = 0;
    if (j < n_big) {
      uint32_t s, L;
      tile_segment(fp, b, (int)b.big_tiles[j], s, L);
      // pass 2 (lazy frames): only the lists whose continuation outlived its window
      const bool use = fp.big_pass == 0 || (fp.big_pass == 1 ? b.big_flag[j] : b.big_flag2[j]) != 0u;
      c = use ? (L + kBigSeg - 1) / kBigSeg : 0u;
      nb = (use || keep_buckets) ? big_buckets(L) : 0u;
      maxl = use ? max(maxl, L) : maxl;
      if (fp.lazy && fp.big_pass == 0) {
        b.big_flag[j] = 0u;
        b.big_cnt[j] = 0u;
        b.big_flag2[j] = 0u;
        b.big_cnt2[j] = 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) b.cont_flag[4 * j + q] = 0u;
      }
    }
    uint32_t inc = c, inc_b = nb;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d, 64), ob = __shfl_up(inc_b, d, 64);
      if (lane >= d) {
        inc += o;
        inc_b += ob;
      }
    }
    if (lane == 63) {
      wsum[wave] = inc;
      wsum_b[wave] = inc_b;
    }
    __syncthreads();
    uint32_t before = 0, tot = 0, before_b = 0, tot_b = 0;
    for (int w = 0; w < 16; ++w) {
      before += w < wave ? wsum[w] : 0u;
      tot += wsum[w];
      before_b += w < wave ? wsum_b[w] : 0u;
      tot_b += wsum_b[w];
    }
    if (j < n_big) {
      const uint32_t off = carry + before + inc - c;
      b.tile_cursor[j] = off;
      for (uint32_t q = 0; q < c; ++q) b.big_item[off + q] = j;  // segment -> list slot
      // the list's first bucket (the continuation of lazy frames keeps the
      // numbering -- and the splitters -- of the frame's first pass)
      if (!keep_buckets) b.bk_off[j] = carry_b + before_b + inc_b - nb;
    }
    carry += tot;
    carry_b += tot_b;
    __syncthreads();
  }
  atomicMax(&s_maxl, maxl);
  __syncthreads();
  if (tid == 0) {
    b.counters[12] = carry;   // segments of all big lists
    b.counters[13] = s_maxl;  // the longest big list (passes beyond it are no-ops)
    b.counters[14] = carry_b; // sample-sort buckets of all big lists
  }
}

// work item k -> (big list j, segment c), from the prefix kernel's tables
__device__ __forceinline__ void big_item(const Buffers& b, uint32_t n_big, uint32_t k, uint32_t& j,
                                         uint32_t& c) {
  j = b.big_item[k];
  c = k - b.tile_cursor[j];
}


// ---- big lists as a sample sort (FrameParams::big_separate, the default):
// per list, splitters from a sorted regular sample of its keys cut it into
// buckets of ~1024 keys; one pass counts the keys per bucket, a scan turns
// the counts into bucket starts, one pass scatters the keys (input-index
// keys, pairs -> pairs_alt) and every bucket is then sorted by one workgroup
// (the medium path; the radix path for a bucket > kSortLdsCap) straight into
// its place in the list.  Buckets split the lists by depth only (keys of
// equal depth share one), so the buckets sort device-index keys and put runs
// of equal depth in input order like the medium lists.  The splitters only
// set the buckets' sizes, never the order.  Every key is read 4 times and
// written twice, against ~8 + 16 per key for the segmented merge sort's
// seven passes at config 5's 162 k-key lists.

// one workgroup per big list (grid-stride): sample, sort it, pick splitters;
// zero the list's bucket counters
__global__ __launch_bounds__(256) void gs_big_split_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  __shared__ unsigned long long keys[kSortLdsCap];
  const uint32_t n_big = b.counters[0];
  const uint32_t tid = threadIdx.x;
  const bool bound = fp.lazy && fp.big_pass == 0;
  for (uint32_t j = blockIdx.x; j < n_big; j += gridDim.x) {
    if (fp.big_pass == 1 && b.big_flag[j] == 0u) continue;  // (uniform)
    uint32_t s, L;
    tile_segment(fp, b, (int)b.big_tiles[j], s, L);
    const uint32_t B = big_buckets(L), bo = b.bk_off[j];
    const uint32_t S = min((uint32_t)kSortLdsCap, min(L, 16u * B));  // sample size
    for (uint32_t k = tid; k < S; k += 256u) {
      const uint32_t p = (uint32_t)(((2ull * k + 1ull) * L) / (2ull * S));
      keys[k] = b.pairs[s + p];
    }
    __syncthreads();
    merge_sort_tile<256, 2, kOutLds, kSrcLds>(b, 0u, S, keys);
    if (bound) {
      // the prefix: keys of lower depth than the sample's kLazyPrefix / L
      // quantile (~kLazyPrefix keys; more than kSortLdsCap sends the whole
      // list to the continuation)
      if (tid == 0u) {
        const uint32_t q = (uint32_t)(((unsigned long long)kLazyPrefix * S) / L);
        b.big_thr[j] = (uint32_t)(keys[min(q, S - 1u)] >> 32);
        // the continuation's window: up to the (prefix + window) / L quantile,
        // or the list's end (~0) when that reaches past the sample
        const uint32_t q2 = (uint32_t)(((unsigned long long)(kLazyPrefix + kLazyWindow) * S) / L);
        b.big_thr2[j] = kLazyPrefix + kLazyWindow < L && q2 < S ? (uint32_t)(keys[q2] >> 32) : 0xFFFFFFFFu;
      }
      // and the buckets of the full sort the continuation may need, from this
      // (larger) sample: the continuation's sample sort then needs no split
      // pass of its own (splitters only size the buckets, never the order)
      for (uint32_t t = tid; t < B; t += 256u) {
        if (t + 1u < B) b.bk_spl[bo + t] = keys[((unsigned long long)(t + 1u) * S) / B - 1u];
        b.bk_cnt[bo + t] = 0u;
        b.bk_list[bo + t] = j;
      }
      __syncthreads();
      continue;
    }
    for (uint32_t t = tid; t < B; t += 256u) {
      if (t + 1u < B) b.bk_spl[bo + t] = keys[((unsigned long long)(t + 1u) * S) / B - 1u];
      b.bk_cnt[bo + t] = 0u;
      b.bk_list[bo + t] = j;
    }
    __syncthreads();
  }
}

// ---- lazy big lists (FrameParams::lazy): the blend rarely needs more than
// the nearest ~2 k keys of a big list -- a tile's pixels saturate (the
// reference's `break`) after a few hundred records in front (config 5: 6.5 %
// of the big-list keys are ever composited).  So before the blend only each
// list's prefix of keys below a depth bound is sorted (split: the bound from
// the sample; select: the keys below it; psort: one workgroup sorts them into
// the list).  A blend wave that reaches the end of the prefix with live pixels
// saves their state and flags the list; after the blend the flagged lists are
// sorted in full by the sample sort (big_pass 1) and the saved waves continue
// from the prefix's end (blend_cont).  Every key below the bound precedes
// every other in the total order (ties share a depth, so they share a side),
// so each pixel composites exactly the list's records in order: the frame is
// the same bit for bit.
// one workgroup per 2048-key work item (pass 0: every big list): append the
// item's keys below the list's bound to the list's prefix (pairs_alt[s, ...))
// The keys of the continuation's window [bound, bound2) go to the END of the
// list's pairs_alt region (from s + L - 1 down): the prefix takes at most the
// keys below the bound from the front, so the two never meet.
__global__ __launch_bounds__(256) void gs_big_select_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  __shared__ uint32_t s_par[6];
  __shared__ uint32_t s_n, s_base, s_n2, s_base2;
  const uint32_t n_big = b.counters[0], total = n_big ? b.counters[12] : 0u;
  const uint32_t tid = threadIdx.x;
  constexpr int Q = kBigSeg / 256;
  for (uint32_t k = blockIdx.x; k < total; k += gridDim.x) {
    if (tid == 0) {
      uint32_t j, c;
      big_item(b, n_big, k, j, c);
      uint32_t s, L;
      tile_segment(fp, b, (int)b.big_tiles[j], s, L);
      s_par[0] = s;
      s_par[1] = L;
      s_par[2] = c;
      s_par[3] = b.big_thr[j];
      s_par[4] = j;
      s_par[5] = b.big_thr2[j];
      s_n = 0u;
      s_n2 = 0u;
    }
    __syncthreads();
    const uint32_t s = s_par[0], L = s_par[1], c = s_par[2], thr = s_par[3], j = s_par[4], thr2 = s_par[5];
    unsigned long long key[Q];
    uint32_t rk[Q], rk2[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t i = c * (uint32_t)kBigSeg + (uint32_t)q * 256u + tid;
      key[q] = i < L ? b.pairs[s + i] : ~0ull;
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t i = c * (uint32_t)kBigSeg + (uint32_t)q * 256u + tid;
      const uint32_t z = (uint32_t)(key[q] >> 32);
      rk[q] = (i < L && z < thr) ? atomicAdd(&s_n, 1u) : 0xFFFFFFFFu;
      rk2[q] = (fp.lazy && i < L && z >= thr && (thr2 == 0xFFFFFFFFu || z < thr2)) ? atomicAdd(&s_n2, 1u)
                                                                                 : 0xFFFFFFFFu;
    }
    __syncthreads();
    if (tid == 0) {
      s_base = s_n ? atomicAdd(&b.big_cnt[j], s_n) : 0u;
      s_base2 = s_n2 ? atomicAdd(&b.big_cnt2[j], s_n2) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t pos = s_base + rk[q];
      if (rk[q] != 0xFFFFFFFFu && pos < (uint32_t)kSortLdsCap) b.pairs_alt[s + pos] = key[q];
      if (rk2[q] != 0xFFFFFFFFu) b.pairs_alt[s + L - 1u - (s_base2 + rk2[q])] = key[q];
    }
    __syncthreads();
  }
}

// one workgroup per big list (grid-stride): sort its prefix into list[s, s + n)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_big_psort_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  __shared__ unsigned long long keys[kSortLdsCap];
  const uint32_t n_big = b.counters[0];
  for (uint32_t j = blockIdx.x; j < n_big; j += gridDim.x) {
    uint32_t s, L;
    tile_segment(fp, b, (int)b.big_tiles[j], s, L);
    const uint32_t n = b.big_cnt[j];
    const bool ok = n > 0u && n <= (uint32_t)kSortLdsCap;  // else: all of it in the continuation
    if (ok && !merge_sort_tile<256, 2, kOutDevice, kSrcAlt>(b, s, n, keys)) {
      __syncthreads();  // a long run of equal depths: again with input-index keys
      merge_sort_tile<256, 2, kOutInput, kSrcAltRekey>(b, s, n, keys);
    }
    if (threadIdx.x == 0) b.big_len[j] = ok ? n : 0u;
    __syncthreads();
  }
}

// the box of the live pixels of a big list's saved waves (the union of their boxes)
__device__ __forceinline__ void cont_live_box(const Buffers& b, uint32_t j, int& x0, int& x1, int& y0, int& y1) {
  x0 = 0x7FFFFFFF, x1 = -1, y0 = 0x7FFFFFFF, y1 = -1;
  for (int w = 0; w < 4; ++w)
    if (b.cont_flag[4 * j + w]) {
      const uint2 cb = b.cont_box[4 * j + w];
      x0 = min(x0, (int)(cb.x & 0xFFFFu));
      x1 = max(x1, (int)(cb.x >> 16));
      y0 = min(y0, (int)(cb.y & 0xFFFFu));
      y1 = max(y1, (int)(cb.y >> 16));
    }
}

// Lazy continuation, pass 1: one workgroup per big list the blend flagged.
// The window's keys (depth in [bound, bound2), kept by the prefix select)
// whose alpha box meets the saved waves' live pixels are sorted into the
// list's front; the continued blend walks them.  The list is complete when
// the window reached its end (bound2 = ~0); otherwise a wave that outlives
// the window flags the list for pass 2, the full sample sort of the keys of
// depth >= cont_thr.  A window whose filtered keys overflow one workgroup's
// sort is skipped (cont_len 0): pass 2 then takes every key past the prefix.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_big_cont_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  __shared__ unsigned long long keys[kSortLdsCap];
  __shared__ uint32_t s_m;
  const uint32_t n_big = b.counters[0];
  const uint32_t tid = threadIdx.x;
  for (uint32_t j = blockIdx.x; j < n_big; j += gridDim.x) {
    if (b.big_flag[j] == 0u) continue;  // (uniform)
    uint32_t s, L;
    tile_segment(fp, b, (int)b.big_tiles[j], s, L);
    // the prefix was sorted (else the keys past it start at depth 0)
    const bool pre = b.big_len[j] != 0u;
    const uint32_t thr = pre ? b.big_thr[j] : 0u, thr2 = b.big_thr2[j];
    const uint32_t n2 = pre ? min(b.big_cnt2[j], L) : 0u;
    int lx0, lx1, ly0, ly1;
    cont_live_box(b, j, lx0, lx1, ly0, ly1);
    if (tid == 0u) s_m = 0u;
    __syncthreads();
    // U keys per thread in flight: all key loads, then all box gathers
    constexpr int U = 8;
    for (uint32_t k0 = 0; k0 < n2; k0 += 256u * U) {
      unsigned long long key[U];
      uint2 bx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t k = k0 + (uint32_t)u * 256u + tid;
        key[u] = k < n2 ? b.pairs_alt[s + L - 1u - k] : ~0ull;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        bx[u] = key[u] != ~0ull ? rec_box(fp, b, (uint32_t)key[u])
                                : make_uint2(kEmptyBox, kEmptyBox);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rx0 = (int)(bx[u].x << 16) >> 16, rx1 = (int)bx[u].x >> 16;
        const int ry0 = (int)(bx[u].y << 16) >> 16, ry1 = (int)bx[u].y >> 16;
        if (rx0 <= lx1 && rx1 >= lx0 && ry0 <= ly1 && ry1 >= ly0) {
          const uint32_t p = atomicAdd(&s_m, 1u);
          if (p < (uint32_t)kSortLdsCap) keys[p] = key[u];
        }
      }
    }
    __syncthreads();
    const uint32_t m = s_m;
    const bool ok = pre && m <= (uint32_t)kSortLdsCap;
    if (ok && m > 0u && !merge_sort_tile<256, 2, kOutDevice, kSrcLds>(b, s, m, keys)) {
      // equal depths: the sorted device-index keys are in keys[0, m); again
      // with input-index keys
      __syncthreads();
      for (uint32_t k = tid; k < m; k += 256u) keys[k] = rekey_input(b, keys[k]);
      __syncthreads();
      merge_sort_tile<256, 2, kOutInput, kSrcLds>(b, s, m, keys);
    }
    if (tid == 0u) {
      b.cont_len[j] = ok ? m : 0u;
      b.cont_full[j] = ok && thr2 == 0xFFFFFFFFu ? 1u : 0u;
      b.cont_thr[j] = ok ? thr2 : thr;  // where pass 2 starts
    }
    __syncthreads();
  }
}

// the bucket of key k: the number of splitters of lower DEPTH (keys of equal
// depth share a bucket, so the bucket sort puts their runs in input order)
__device__ __forceinline__ uint32_t big_bucket_of(const unsigned long long* spl, uint32_t nspl,
                                                  unsigned long long k) {
  const uint32_t kz = (uint32_t)(k >> 32);
  uint32_t lo = 0u, hi = nspl;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((uint32_t)(spl[mid] >> 32) < kz) lo = mid + 1u;
    else hi = mid;
  }
  return lo;
}

// one workgroup per 2048-key work item: count the keys per bucket (LDS
// histogram, then one global add per non-empty bucket)
// SCATTER: the second pass -- reserve each bucket's range and write the keys
// to pairs_alt at bucket start + reserved base + rank
template <bool SCATTER>
__device__ __forceinline__ void big_bucket_pass(const FrameParams& fp, const Buffers& b) {
  __shared__ unsigned long long s_spl[kBktMax];
  __shared__ uint32_t s_h[kBktMax], s_base[SCATTER ? kBktMax : 1];
  __shared__ uint32_t s_par[9];
  const uint32_t n_big = b.counters[0], total = n_big ? b.counters[12] : 0u;
  const uint32_t tid = threadIdx.x;
  constexpr int Q = kBigSeg / 256;
  // lazy continuation (pass 2): only the keys past the window (cont_thr) whose
  // alpha box meets the list's live pixels (the saved waves' boxes) are sorted
  const bool filt = fp.lazy && fp.big_pass == 2;
  for (uint32_t k = blockIdx.x; k < total; k += gridDim.x) {
    if (tid == 0) {
      uint32_t j, c;
      big_item(b, n_big, k, j, c);
      uint32_t s, L;
      tile_segment(fp, b, (int)b.big_tiles[j], s, L);
      s_par[0] = s;
      s_par[1] = L;
      s_par[2] = c;
      s_par[3] = b.bk_off[j];
      if (filt) {
        int bx0, bx1, by0, by1;
        cont_live_box(b, j, bx0, bx1, by0, by1);
        s_par[4] = (uint32_t)bx0;
        s_par[5] = (uint32_t)bx1;
        s_par[6] = (uint32_t)by0;
        s_par[7] = (uint32_t)by1;
        // keys below cont_thr were composited by the prefix blend and the
        // window's continuation (gs_big_cont_kernel)
        s_par[8] = b.cont_thr[j];
      }
    }
    __syncthreads();
    const uint32_t s = s_par[0], L = s_par[1], c = s_par[2], bo = s_par[3];
    const uint32_t B = big_buckets(L);
    for (uint32_t t = tid; t < B; t += 256u) {
      if (t + 1u < B) s_spl[t] = b.bk_spl[bo + t];
      s_h[t] = 0u;
    }
    __syncthreads();
    unsigned long long key[Q];
    uint32_t bk[Q], rk[Q];
    bool use[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t i = c * (uint32_t)kBigSeg + (uint32_t)q * 256u + tid;
      key[q] = i < L ? b.pairs[s + i] : 0ull;
      use[q] = i < L;
    }
    if (filt) {
      const int lx0 = (int)s_par[4], lx1 = (int)s_par[5], ly0 = (int)s_par[6], ly1 = (int)s_par[7];
      const uint32_t thr = s_par[8];
      uint2 bx[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q)  // the record's alpha box (its 3rd float4's z, w)
        bx[q] = (use[q] && (uint32_t)(key[q] >> 32) >= thr)
                    ? rec_box(fp, b, (uint32_t)key[q])
                    : make_uint2(kEmptyBox, kEmptyBox);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int rx0 = (int)(bx[q].x << 16) >> 16, rx1 = (int)bx[q].x >> 16;
        const int ry0 = (int)(bx[q].y << 16) >> 16, ry1 = (int)bx[q].y >> 16;
        use[q] = use[q] && (uint32_t)(key[q] >> 32) >= thr && rx0 <= lx1 && rx1 >= lx0 && ry0 <= ly1 && ry1 >= ly0;
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (use[q]) {
        bk[q] = big_bucket_of(s_spl, B - 1u, key[q]);
        rk[q] = atomicAdd(&s_h[bk[q]], 1u);
      }
    }
    __syncthreads();
    for (uint32_t t = tid; t < B; t += 256u) {
      const uint32_t n = s_h[t];
      if constexpr (SCATTER) s_base[t] = n ? b.bk_start[bo + t] + atomicAdd(&b.bk_cnt[bo + t], n) : 0u;
      else if (n) atomicAdd(&b.bk_cnt[bo + t], n);
    }
    __syncthreads();
    if constexpr (SCATTER) {
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (use[q]) b.pairs_alt[s + s_base[bk[q]] + rk[q]] = key[q];
    }
  }
}

__global__ __launch_bounds__(256) void gs_big_count_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  big_bucket_pass<false>(fp, b);
}

__global__ __launch_bounds__(256) void gs_big_scatter_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  big_bucket_pass<true>(fp, b);
}

// one wave per big list: bucket counts -> bucket starts (exclusive, within the
// list); the counters are reset for the scatter's reservations
__global__ __launch_bounds__(256) void gs_big_bscan_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  const uint32_t n_big = b.counters[0];
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * 4u;
  if (fp.big_pass == 2 && b.counters[1] == 0u) return;  // no list outlived its window
  for (uint32_t j = blockIdx.x * 4u + (threadIdx.x >> 6); j < n_big; j += nw) {
    if (fp.big_pass == 2 && b.big_flag2[j] == 0u) continue;  // (wave-uniform)
    uint32_t s, L;
    tile_segment(fp, b, (int)b.big_tiles[j], s, L);
    const uint32_t B = big_buckets(L), bo = b.bk_off[j];
    uint32_t carry = 0u;
    for (uint32_t t0 = 0; t0 < B; t0 += 64u) {
      const uint32_t t = t0 + (uint32_t)lane;
      const uint32_t n = t < B ? b.bk_cnt[bo + t] : 0u;
      uint32_t inc = n;
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
      }
      if (t < B) {
        b.bk_start[bo + t] = carry + inc - n;
        b.bk_cnt[bo + t] = 0u;
      }
      carry += (uint32_t)__shfl(inc, 63, 64);
    }
    if (fp.lazy && fp.big_pass == 2 && lane == 0) b.cont_len[j] = carry;  // the filtered keys
  }
}

// one workgroup per bucket (grid-stride): sort it into its place in the list
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_big_bsort_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBig);
  constexpr int NT = 256, NW = NT / 64;
  constexpr int kRadixWords = 8 * 256 + 256 + NW * 256;
  constexpr int kWords = 2 * kSortLdsCap > kRadixWords ? 2 * kSortLdsCap : kRadixWords;
  __shared__ unsigned long long keys[kWords / 2];
  uint32_t* const r_hist = (uint32_t*)keys;
  uint32_t* const r_base = r_hist + 8 * 256;
  uint32_t(*const r_wcnt)[256] = (uint32_t(*)[256])(r_hist + 9 * 256);
  const uint32_t n_bk = (b.counters[0] && (fp.big_pass != 2 || b.counters[1])) ? b.counters[14] : 0u;
  for (uint32_t k = blockIdx.x; k < n_bk; k += gridDim.x) {
    const uint32_t j = b.bk_list[k];
    if (fp.big_pass == 2 && b.big_flag2[j] == 0u) continue;  // (uniform) lazy continuation: flagged lists only
    uint32_t s, L;
    tile_segment(fp, b, (int)b.big_tiles[j], s, L);
    const uint32_t bo = b.bk_off[j], B = big_buckets(L);
    const uint32_t Lk = (fp.lazy && fp.big_pass == 2) ? b.cont_len[j] : L;  // (pass 2: the filtered keys)
    const uint32_t st = b.bk_start[k], en = k + 1u < bo + B ? b.bk_start[k + 1u] : Lk;
    const uint32_t n = en - st;
    if (n == 0u) continue;  // (uniform)
    if (n > (uint32_t)kSortLdsCap) {
      radix_sort_seg<NT, 4, true>(b, s + st, n, r_hist, r_base, r_wcnt);
    } else if (!merge_sort_tile<NT, 2, kOutDevice, kSrcAlt>(b, s + st, n, keys)) {
      __syncthreads();  // a long run of equal depths: again with input-index keys
      merge_sort_tile<NT, 2, kOutInput, kSrcAltRekey>(b, s + st, n, keys);
    }
    __syncthreads();
  }
}

// -------------------------------------------------------------------- blend

typedef float f32x2 __attribute__((ext_vector_type(2)));

// v_writelane_b32 x2: lanes L and L + 1 of v take the wave-uniform words lo,
// hi -- a ballot's two halves.  The s_nop gives the two wait states a VALU
// read of an SGPR needs after the VALU compare that wrote it (the compiler
// inserts them for its own code, not inside inline asm).
template <int L>
__device__ __forceinline__ uint32_t writelane2(uint32_t v, uint32_t lo, uint32_t hi) {
  asm("s_nop 1\n\tv_writelane_b32 %0, %1, %3\n\tv_writelane_b32 %0, %2, %4"
      : "+v"(v)
      : "s"(lo), "s"(hi), "n"(L), "n"(L + 1));
  return v;
}

// The ballots of spans [lo, lo + sp] over positions C = 0 .. N - 1, written
// into lanes 2 (B + C) (low word) and 2 (B + C) + 1 (high word) of tab
template <int B, int C, int N>
struct BallotTab {
  __device__ __forceinline__ static void run(uint32_t& tab, int lo, int sp) {
    if constexpr (C < N) {
      const unsigned long long bc = ballot64((uint32_t)(C - lo) <= (uint32_t)sp);
      tab = writelane2<2 * (B + C)>(tab, (uint32_t)bc, (uint32_t)(bc >> 32));
      BallotTab<B, C + 1, N>::run(tab, lo, sp);
    }
  }
};

// Per-pixel blend state: position, transmittance, accumulated colour, and
// whether the pixel has saturated (the reference's `break`).
struct Px {
  f32x2 p;         // pixel centre (x, y)
  float T;
  f32x2 c01, c23;  // colour accumulators (r, g), (b, a)
  bool done;
};

// GS_X_EXPM (measurement builds, tools/build_x.sh): 1 = rint and the integer
// exponent from the magic-number addition
#ifndef GS_X_EXPM
#define GS_X_EXPM 0
#endif
__device__ __forceinline__ float gs_expf_inrange(float x) {
  // gs_expf for x in [-80, 0]: the same ops minus the clamps / selects, which
  // are no-ops there.  Outside that range the result is unused (selected away).
#if GS_X_EXPM
  // rint by the 1.5 * 2^23 addition (exact for |t| < 2^22, ties to even as
  // v_rndne_f32), and the integer k from the sum's low mantissa bits: two
  // full-rate adds and an integer add instead of v_rndne and v_cvt_i32
  // (~4.1 SIMD cycles each), the same values
  const float t = x * 1.44269502162933349609f;
  const float sm = t + 12582912.0f;
  const float k = sm - 12582912.0f;
  const int ki = (int)(__float_as_uint(sm) - 0x4B400000u);
#else
  const float k = __builtin_rintf(x * 1.44269502162933349609f);
  const int ki = (int)k;
#endif
  float r = __builtin_fmaf(k, -0.693145751953125f, x);
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
  return __builtin_amdgcn_ldexpf(p, ki);  // == p * 2^k: k in [-115, 0], p in [0.7, 1.5]
}

// GS_FLAG_FAST_EXP: e^x = 2^t with t = x log2(e) split into t + lo by an fma
// (lo carries the product's rounding error), then 2^(t + lo) = 2^t (1 + lo ln 2)
// with the hardware exp2.  A few ulp, for every x (NaN in, NaN out; large
// negative x -> 0); not the oracle's bits, so opt-in only.
__device__ __forceinline__ float gs_expf_hw(float x) {
  const float t = x * 1.44269502162933349609f;
  const float lo = __builtin_fmaf(x, 1.925963033500011079e-08f, __builtin_fmaf(x, 1.44269502162933349609f, -t));
  const float p = __builtin_amdgcn_exp2f(t);
  return __builtin_fmaf(p * lo, 0.693147182464599609375f, p);
}

// exponential variants of the blend loop
enum BlendExp { kExpExact = 0, kExpInRange = 1, kExpHw = 2 };

// One staged record (48 B, see the project kernel):
//   r0 = (mx, my, k0, k2)   r1 = (k1, pcut, r, g)   r2 = (b, opacity, box_x, box_y)
// One pixel's front-to-back step for one record (renderTile inner loop,
// codelets.cpp:385-411), split in two: blend_power_exp (independent of the
// pixel's state) and blend_composite (the decisions, then the state update).
// All scalar fp32 (the build disables SLP packing: packed fp32 chains were
// 15 % slower).  kExpInRange: the batch's records all have pcut >= -80, so
// any power the update accepts lies in [-80, 0], where gs_expf_inrange ==
// gs_expf bit for bit; kExpHw: GS_FLAG_FAST_EXP.
// The staging stores h0 = -0.5 k0 and h2 = -0.5 k2, so power = (h0 dx dx +
// h2 dy dy) - k1 dx dy saves the reference's multiply by -0.5 per step.
// Scaling by a power of two commutes with rounding, so every product and the
// sum are the reference's values times -0.5 exactly -- except below the
// normal range, where only powers of magnitude < 1e-37 can differ: those give
// expf = 1 and the same sign tests either way.  (A/B: blend 75.1 -> 74.0 us
// with the loads issued up front; parity tests bit-exact.)
template <int EXP>
__device__ __forceinline__ float blend_power_exp(const Px& q, const float4& r0, const float4& r1,
                                                 float& power) {
  const float dx = r0.x - q.p.x, dy = r0.y - q.p.y;
  const float h0 = r0.z, h2 = r0.w, k1 = r1.x;  // h0 = -0.5 k0, h2 = -0.5 k2 (staged)
  power = (h0 * dx * dx + h2 * dy * dy) - k1 * dx * dy;
  return EXP == kExpHw ? gs_expf_hw(power) : (EXP == kExpInRange ? gs_expf_inrange(power) : gs_expf(power));
}

__device__ __forceinline__ void blend_composite(Px& q, float power, float e, const float4& r1,
                                                const float4& r2, bool ok) {
  const float pcut = r1.y, op = r2.y;
  const float v = op * e;
  const float alpha = (v < 0.99f) ? v : 0.99f;  // glm::min(0.99f, v)
  const float test_T = q.T * (1.0f - alpha);
  // power > 0: skipped; power < pcut: alpha < 1/255 guaranteed (`continue`)
  const bool hit =
      ok && !q.done && !(power > 0.0f) && !(power < pcut) && !(alpha < 1.0f / 255.0f);
  const bool brk = hit && test_T < 0.0001f;  // break (codelets.cpp:406-408)
  const bool upd = hit && !brk;
  if (__builtin_expect(upd, 0)) {
    q.c01.x = q.c01.x + (r1.z * alpha) * q.T;  // colour += gCont * alpha * T
    q.c01.y = q.c01.y + (r1.w * alpha) * q.T;
    q.c23.x = q.c23.x + (r2.x * alpha) * q.T;
    q.c23.y = q.c23.y + (op * alpha) * q.T;
    q.T = test_T;
  }
  q.done = q.done || brk;
}

// the pixel's RGBA f32 value (+0: a -0 sum stored as +0, as the oracle)
__device__ __forceinline__ float4 pixel_rgba(const Px& q) {
  return make_float4(0.0f + q.c01.x, 0.0f + q.c01.y, 0.0f + q.c23.x, 0.0f + q.c23.y);
}

// row: the pixel's row in this band's output
__device__ __forceinline__ void store_bgr(const FrameParams& fp, const Buffers& b, int px, int row, const Px& q) {
  const float4 o = pixel_rgba(q);
  uint8_t* dst = b.bgr + (size_t)row * fp.bgr_pitch + 3 * (size_t)px;
  dst[0] = to_u8(o.z);  // RGBA2BGR
  dst[1] = to_u8(o.y);
  dst[2] = to_u8(o.x);
}

// one pixel per lane: a wave's 16-B stores cover whole 128-B lines (the
// 8-pixel rows of an 8x8 block, the 16-pixel rows of a 16x4 one), so the
// streaming stores write each line once (the quad-row runs of other tile
// shapes, BQW = 0, may start or end mid-line)
__device__ __forceinline__ void store_pixel(const FrameParams& fp, const Buffers& b, int px, int row,
                                            const Px& q) {
  if (fp.write_rgba) store_stream(b.rgba + (size_t)row * fp.width + px, pixel_rgba(q));
  store_bgr(fp, b, px, row, q);
}

// The records of a lane's batch mask (bit k = staged record k), one per
// iteration in list order, so the wave's iteration count is the largest
// number of records of any lane.  (Round 3: one record per step instead of
// two with independent exponentials -- a lane with an odd count no longer
// evaluates a dead second record and the walk is simpler: blend 78.2 -> 75.6
// us, 7 527 -> 7 728 frames/s, three interleaved A/B repeats, bit-exact.)
// The lane stops as soon as its pixel has saturated (the reference's `break`).
template <int EXP>
__device__ __forceinline__ void blend_records(Px& q, float4 (*st)[64], uint32_t w, uint32_t h) {
  unsigned long long m = ((unsigned long long)h << 32) | w;
  while (m) {
    const int ja = __builtin_ctzll(m);
    m &= m - 1ull;
    const float4 a0 = st[0][ja], a1 = st[1][ja], a2 = st[2][ja];
    asm volatile("" ::"v"(a1.z), "v"(a1.w), "v"(a2.x), "v"(a2.y));  // all loads issued up front
    float pa;
    const float ea = blend_power_exp<EXP>(q, a0, a1, pa);
    blend_composite(q, pa, ea, a1, a2, true);
    m = q.done ? 0ull : m;
  }
}

// One wave = 16 pixel quads (2x2) of one tile, one lane per pixel: a block of
// bqw x (16 / bqw) quads (8x8 or 16x4 pixels) when the tile is a multiple of
// it, else 16 consecutive quads in quad-row-major order.  Every quad keeps its
// own record queue.  The wave walks the tile's depth-sorted list in batches
// of 64 (the next batch's indices and records are loaded while this one is
// blended): the records are staged in wave-private LDS and each record's
// footprint box is turned into the set of quads it touches (16 ballots, one
// 64-bit mask per quad).  Each quad then evaluates only its records, in list
// order, reading the next record from LDS while the current one is blended;
// a quad stops when its four pixels have saturated and the wave when all
// quads have.  The per-pixel arithmetic and record order are those of
// renderTile (codelets.cpp:385-411): a record is skipped for a quad only when
// no pixel of the quad can take it ("blend culling").
// profiled frames (FrameParams::count_records): the records a blend wave
// staged, for the bench's algorithmic bytes (lane 0 of the wave)
__device__ __forceinline__ void blend_count_store(const FrameParams& fp, const Buffers& b, int wid,
                                                  uint32_t staged) {
  if (fp.count_records && (threadIdx.x & 63) == 0) {
    if (fp.blend_cont && fp.big_pass == 2) b.blend_count_cont[wid] += staged;  // (after pass 1's)
    else (fp.blend_cont ? b.blend_count_cont : b.blend_count)[wid] = staged;
  }
}

// A list entry.  With the sort in the blend (FrameParams::blend_sort) the
// lists were written by this launch's own workgroups: agent-scope loads, so
// a line of a neighbouring tile's list that another workgroup of the CU
// pulled into the vector L1 before this tile's list was written is never
// read from there.
__device__ __forceinline__ uint32_t blend_idx(const FrameParams& fp, const uint32_t* list, uint32_t L, uint32_t k) {
  uint32_t g = 0xFFFFFFFFu;
  if (k < L) g = fp.blend_sort ? __hip_atomic_load(list + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : list[k];
  return g < (uint32_t)fp.n ? g : 0xFFFFFFFFu;  // defensive: never read past the records
}

// the tile of blend slot `slot`: the tile order, or (blend_lpt) the sort
// queues' order -- big, medium (longest first), then small and empty lists
__device__ __forceinline__ int blend_tile_of(const FrameParams& fp, const Buffers& b, int slot) {
  if (!fp.blend_lpt) return slot;
  const uint32_t nb = b.counters[0], nm = b.counters[7], u = (uint32_t)slot;
  return (int)(u < nb ? b.big_tiles[u] : (u < nb + nm ? b.medium_tiles[u - nb] : b.small_tiles[u - nb - nm]));
}

// wid = the wave's (tile slot, 8x8 block) item; st: the wave's LDS staging
// of one batch (3 x 64 float4)
template <int BQW, bool HWEXP, bool DIRECT = false>
__device__ __forceinline__ void blend_wave(const FrameParams& fp, const Buffers& b, int wid, float4 (*st)[64]) {
  const int slot = wid / fp.chunks_per_tile;
  const int chunk = wid - slot * fp.chunks_per_tile;
  if (slot >= fp.n_tiles) return;
  // lazy big lists: jb = the tile's big-list slot.  The continuation's waves
  // are (slot, chunk) of the flagged lists whose state was saved.
  uint32_t jb = 0xFFFFFFFFu;
  if (fp.blend_cont) {
    // pass 1: the waves the prefix blend saved; pass 2: those of them that
    // outlived their window too
    if ((uint32_t)slot >= b.counters[0] || b.cont_flag[4 * slot + chunk] == 0u ||
        (fp.big_pass == 2 && b.big_flag2[slot] == 0u)) {
      if (fp.big_pass == 1) blend_count_store(fp, b, wid, 0u);
      return;
    }
    jb = (uint32_t)slot;
  }
  // row bands: longest lists first (the sort queues: big, medium, then small
  // and empty tiles), so the heaviest tiles' waves start at once instead of
  // where the tile order puts them (8 bands: blend 35.7 -> 29.3 us).  The
  // full frame keeps the tile order (neighbouring tiles share records in L2:
  // 75.1 against 76.1 us in queue order).
  const int tile = DIRECT ? slot : (fp.blend_cont ? (int)b.big_tiles[jb] : blend_tile_of(fp, b, slot));
  const int lane = threadIdx.x & 63;
  const int myq = lane >> 2;
  const int tx = tile % fp.tiles_x, tyb = tile / fp.tiles_x;
  const int tile_x0 = tx * fp.tile_w;
  const int tile_y0 = (fp.band_ty0 + tyb * fp.band_stride) * fp.tile_h;
  constexpr int bqw = BQW;  // 4 | 8: block of quads; 0: quad-row-major run

  // the wave's first quad (tile-local pixel coordinates) and quad count
  int q_x, q_y, nq_wave;
  const int qw = (fp.tile_w + 1) >> 1;
  if constexpr (BQW != 0) {
    const int bpr = fp.tile_w / (2 * bqw);
    q_x = (chunk % bpr) * (2 * bqw);
    q_y = (chunk / bpr) * (32 / bqw);
    nq_wave = 16;
  } else {
    const int nq = qw * ((fp.tile_h + 1) >> 1);
    const int qi0 = chunk * 16;
    q_x = (qi0 % qw) << 1;
    q_y = (qi0 / qw) << 1;
    nq_wave = min(16, nq - qi0);
  }
  // this lane's pixel
  int lqx, lqy;
  if constexpr (BQW != 0) {
    lqx = q_x + ((myq % bqw) << 1);
    lqy = q_y + ((myq / bqw) << 1);
  } else {
    const int qi = chunk * 16 + myq;
    lqx = (qi % qw) << 1;
    lqy = (qi / qw) << 1;
  }
  const int lx = lqx + (lane & 1), ly = lqy + ((lane >> 1) & 1);
  const int px = tile_x0 + lx, py = tile_y0 + ly;
  const bool valid = myq < nq_wave && lx < fp.tile_w && ly < fp.tile_h && px < fp.width &&
                     py < fp.height;
  Px q;
  q.p = f32x2{(float)px, (float)py};
  q.T = 1.0f;
  q.c01 = f32x2{0.0f, 0.0f};
  q.c23 = f32x2{0.0f, 0.0f};
  q.done = !valid;

  uint32_t s, L;
  uint32_t k0 = 0u, Lfull;
  tile_segment<DIRECT>(fp, b, tile, s, L);
  Lfull = L;
  // lazy big list: this pass composites the sorted prefix [0, big_len), the
  // continuation the rest [big_len, L) from the saved state
  if (fp.lazy && !fp.blend_cont) jb = b.tile_big[tile];
  if (jb != 0xFFFFFFFFu) {
    const uint32_t np = min(b.big_len[jb], L);
    if (fp.blend_cont) {
      // the list now holds, from its start, the keys past the prefix whose
      // alpha box meets the live pixels (big-list pass 1), in list order
      L = min(b.cont_len[jb], L);
      k0 = 0u;
      float* sv = b.cont_state + (size_t)(4 * jb + chunk) * 6 * 64 + lane;
      q.T = sv[0];
      q.c01 = f32x2{sv[64], sv[128]};
      q.c23 = f32x2{sv[192], sv[256]};
      q.done = sv[320] != 0.0f;
    } else {
      L = np;
    }
  }
  const uint32_t* __restrict__ list = b.list + s + k0;
  L -= k0;

  // software pipeline: records of batch `base`, index of batch `base + 64`
  auto load_idx = [&](uint32_t k) -> uint32_t { return blend_idx(fp, list, L, k); };
  // a record (32 B) and its colour + opacity (the scene's, or gs_set_sh's
  // view-dependent one), assembled as the staged 48-B layout
  const float4* __restrict__ ccol = (fp.sh_degree >= 0 && b.sh) ? b.col_out : b.colour;
  auto load_rec = [&](uint32_t g, float4& r0, float4& r1, float4& r2) {
    const float4* qq = b.rec + 2 * (size_t)g;
    r0 = qq[0];
    const float4 t = qq[1];    // k1 pcut boxx boxy
    const float4 c = ccol[g];  // r g b opacity
    r1 = make_float4(t.x, t.y, c.x, c.y);
    r2 = make_float4(c.z, c.w, t.z, t.w);
  };
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0;
  uint32_t g_cur = load_idx(lane);
  if (g_cur != 0xFFFFFFFFu) load_rec(g_cur, a0, a1, a2);
  uint32_t g_next = load_idx(64 + lane);

  uint32_t staged = 0;  // records staged (profiled frames)
  for (uint32_t base = 0; base < L; base += 64) {
    if (ballot64(!q.done) == 0ull) break;
    staged += min(64u, L - base);
    // stage this batch
    const bool have = g_cur != 0xFFFFFFFFu;
    st[0][lane] = make_float4(a0.x, a0.y, -0.5f * a0.z, -0.5f * a0.w);
    st[1][lane] = a1;
    st[2][lane] = a2;
    const uint32_t boxx = __float_as_uint(a2.z), boxy = __float_as_uint(a2.w);
    const int rx0 = (int)(boxx << 16) >> 16, rx1 = (int)boxx >> 16;
    const int ry0 = (int)(boxy << 16) >> 16, ry1 = (int)boxy >> 16;
    const bool rok = have && !(a2.y == 0.0f) &&  // con_o.w == 0 (codelets.cpp:389)
                     rx0 <= rx1 && ry0 <= ry1;
    // the batch takes the clamp-free exponential when every record's pcut
    // is >= -80 (wave-uniform, so the record loop carries no per-step test)
    const bool fast = ballot64(rok && !(a1.y >= -80.0f)) == 0ull;
    // prefetch the next batch
    g_cur = g_next;
    a0 = a1 = a2 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g_cur != 0xFFFFFFFFu) load_rec(g_cur, a0, a1, a2);
    g_next = load_idx(base + 128 + lane);

    // m = the batch's records whose box touches this lane's quad (bit k =
    // record k).  Blocks: per quad column / row one ballot, then each lane
    // ANDs its column's and row's masks; quad runs: one ballot per quad.
    unsigned long long m = 0ull;
    if constexpr (BQW != 0) {
      // Pixel columns and rows of the block: one ballot per column / row,
      // each a single unsigned compare (c - lo <= span; a lane without a
      // record never matches), then each lane selects its column's and row's
      // masks and ANDs them.  (Quad-granular masks: round 2, 21 % more
      // evaluations.)
      constexpr int NC = 2 * bqw, NR = 32 / bqw;
      const int bx = tile_x0 + q_x, by = tile_y0 + q_y;
      const int xlo = rok ? rx0 - bx : 0x40000000, xsp = rok ? (rx1 - bx) - xlo : 0;
      const int ylo = rok ? ry0 - by : 0x40000000, ysp = rok ? (ry1 - by) - ylo : 0;
      const int mycol = lx - q_x, myrow = ly - q_y;
      // the ballots (wave-uniform) go into one VGPR, lanes 2c / 2c + 1 for
      // column c and 2 (NC + w) / + 1 for row w; each lane then reads its
      // column's and row's words back with ds_bpermute (4 crossbar reads
      // instead of a select chain of 4 VALU per ballot)
      static_assert(2 * (NC + NR) <= 64, "one VGPR holds every ballot");
      uint32_t tab = 0u;
      BallotTab<0, 0, NC>::run(tab, xlo, xsp);
      BallotTab<NC, 0, NR>::run(tab, ylo, ysp);
      const int ac = 8 * mycol, ar = 8 * (NC + myrow);  // byte addresses of the lanes' words
      const uint32_t mcl = (uint32_t)__builtin_amdgcn_ds_bpermute(ac, (int)tab);
      const uint32_t mch = (uint32_t)__builtin_amdgcn_ds_bpermute(ac + 4, (int)tab);
      const uint32_t mrl = (uint32_t)__builtin_amdgcn_ds_bpermute(ar, (int)tab);
      const uint32_t mrh = (uint32_t)__builtin_amdgcn_ds_bpermute(ar + 4, (int)tab);
      m = ((unsigned long long)(mch & mrh) << 32) | (unsigned long long)(mcl & mrl);
    } else {
      int cx = q_x, cy = q_y;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int X0 = tile_x0 + cx, Y0 = tile_y0 + cy;
        const bool h = rok && t < nq_wave && !(rx0 > X0 + 1 || rx1 < X0 || ry0 > Y0 + 1 || ry1 < Y0);
        const unsigned long long bt = ballot64(h);
        m = (myq == t) ? bt : m;
        cx += 2;
        if (cx >= (qw << 1)) {
          cx = 0;
          cy += 2;
        }
      }
    }
    // the lanes' LDS stores precede the reads below (same wave)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // list order = ascending bits: the low word's records, then the high word's.
    // Each lane leaves as soon as its own pixel has saturated.
    const uint32_t m_lo = q.done ? 0u : (uint32_t)m, m_hi = (uint32_t)(m >> 32);
    if (HWEXP) {
      blend_records<kExpHw>(q, st, m_lo, q.done ? 0u : m_hi);
    } else if (fast) {
      blend_records<kExpInRange>(q, st, m_lo, q.done ? 0u : m_hi);
    } else {
      blend_records<kExpExact>(q, st, m_lo, q.done ? 0u : m_hi);
    }
    // the next batch's LDS stores come after every lane's reads of this one
    __builtin_amdgcn_wave_barrier();
  }
  // the list goes on past what this pass walked: the prefix blend's sorted
  // prefix, or a continuation window that did not reach the list's end
  bool more = false;
  if (jb != 0xFFFFFFFFu) more = fp.blend_cont ? (fp.big_pass == 1 && b.cont_full[jb] == 0u) : L < Lfull;
  if (more && ballot64(!q.done) != 0ull) {
    // the walk ended with live pixels: save the wave's state, flag the list
    float* sv = b.cont_state + (size_t)(4 * jb + chunk) * 6 * 64 + lane;
    sv[0] = q.T;
    sv[64] = q.c01.x;
    sv[128] = q.c01.y;
    sv[192] = q.c23.x;
    sv[256] = q.c23.y;
    sv[320] = q.done ? 1.0f : 0.0f;
    // the live pixels' box: the continuation's list keeps only the records
    // whose alpha box meets it (the others cannot touch a live pixel)
    uint32_t blo = q.done ? 0xFFFFFFFFu : ((uint32_t)px | ((uint32_t)py << 16));
    uint32_t bhi = q.done ? 0u : ((uint32_t)px | ((uint32_t)py << 16));
    wave_minmax_u16x2(blo, bhi);
    if (lane == 0) {
      b.cont_box[4 * jb + chunk] = make_uint2((blo & 0xFFFFu) | (bhi << 16), (blo >> 16) | (bhi & 0xFFFF0000u));
      b.cont_flag[4 * jb + chunk] = 1u;
      if (!fp.blend_cont) {
        b.big_flag[jb] = 1u;
      } else {  // pass 1 -> pass 2
        b.big_flag2[jb] = 1u;
        b.counters[1] = 1u;
      }
    }
    blend_count_store(fp, b, wid, staged);
    return;  // the continuation stores these pixels
  }
  if (fp.blend_cont && lane == 0) b.cont_flag[4 * jb + chunk] = 0u;  // this wave is done
  blend_count_store(fp, b, wid, staged);
  if (valid) store_pixel(fp, b, px, tyb * fp.tile_h + ly, q);
}

// Two pixels per lane (FrameParams::blend_px2, 16x16 tiles, no lazy big
// lists): a wave covers a 16x8 half of the tile, lane l the pixels
// (2 (l & 7), l >> 3) and the one right of it, with one mask per lane: the
// records whose alpha box meets either pixel (8 pixel-pair column ballots and
// 8 row ballots).  Per record the lane runs two independent chains (power,
// exponential, composite) -- the record's LDS reads, the mask walk and the
// h2 dy dy term are shared, each pixel's arithmetic is renderTile's in its
// order (codelets.cpp:385-411) -- and a tile takes two waves, not four, so
// its records are staged twice instead of four times.  A record is also
// evaluated for the lane's pixel whose column it does not meet: power <
// pcut there, so it is skipped exactly as the reference skips it.
// GS_LANES builds: a lane's record steps, live-pixel evaluations, those whose
// record's alpha box holds the pixel, and hits
struct LaneCount {
  uint32_t steps = 0, evals = 0, box = 0, hits = 0;
};

template <int EXP>
__device__ __forceinline__ void blend_records_px2(Px& qa, Px& qb, float4 (*st)[64], uint32_t w, uint32_t h,
                                                  LaneCount& lc) {
  unsigned long long m = ((unsigned long long)h << 32) | w;
  while (m) {
    const int ja = __builtin_ctzll(m);
    m &= m - 1ull;
    const float4 a0 = st[0][ja], a1 = st[1][ja], a2 = st[2][ja];
    asm volatile("" ::"v"(a1.z), "v"(a1.w), "v"(a2.x), "v"(a2.y));  // all loads issued up front
    if constexpr (GS_LANES != 0) {
      const uint32_t bx = __float_as_uint(a2.z), by = __float_as_uint(a2.w);
      const int x0 = (int)(bx << 16) >> 16, x1 = (int)bx >> 16, y0 = (int)(by << 16) >> 16, y1 = (int)by >> 16;
      const int xa = (int)qa.p.x, xb = (int)qb.p.x, y = (int)qa.p.y;
      const bool yin = y0 <= y && y <= y1;
      lc.steps += 1u;
      lc.evals += (qa.done ? 0u : 1u) + (qb.done ? 0u : 1u);
      lc.box += ((!qa.done && yin && x0 <= xa && xa <= x1) ? 1u : 0u) + ((!qb.done && yin && x0 <= xb && xb <= x1) ? 1u : 0u);
    }
    const float h0 = a0.z, h2 = a0.w, k1 = a1.x;  // h0 = -0.5 k0, h2 = -0.5 k2 (staged)
    const float dy = a0.y - qa.p.y;               // (one row: the same dy for both pixels)
    const float h2dd = h2 * dy * dy;
    const float dxa = a0.x - qa.p.x, dxb = a0.x - qb.p.x;
    const float pa = (h0 * dxa * dxa + h2dd) - k1 * dxa * dy;
    const float pb = (h0 * dxb * dxb + h2dd) - k1 * dxb * dy;
    const float ea = EXP == kExpHw ? gs_expf_hw(pa) : (EXP == kExpInRange ? gs_expf_inrange(pa) : gs_expf(pa));
    const float eb = EXP == kExpHw ? gs_expf_hw(pb) : (EXP == kExpInRange ? gs_expf_inrange(pb) : gs_expf(pb));
    // Both pixels' decisions (blend_composite's, same operations) before
    // either update branch: the compiler otherwise sinks pixel b's whole
    // chain below pixel a's update branch, so the two chains ran one after
    // the other instead of side by side.
    const float pcut = a1.y, op = a2.y;
    const float va = op * ea, vb = op * eb;
    const float ala = (va < 0.99f) ? va : 0.99f, alb = (vb < 0.99f) ? vb : 0.99f;
    const float tta = qa.T * (1.0f - ala), ttb = qb.T * (1.0f - alb);
    asm volatile("" ::"v"(ala), "v"(alb), "v"(tta), "v"(ttb));
    const bool hita = !qa.done && !(pa > 0.0f) && !(pa < pcut) && !(ala < 1.0f / 255.0f);
    const bool hitb = !qb.done && !(pb > 0.0f) && !(pb < pcut) && !(alb < 1.0f / 255.0f);
    const bool brka = hita && tta < 0.0001f, brkb = hitb && ttb < 0.0001f;
    const bool upda = hita && !brka, updb = hitb && !brkb;
    if constexpr (GS_LANES != 0) lc.hits += (hita ? 1u : 0u) + (hitb ? 1u : 0u);
    // (the update branches in line: some lane updates in most steps -- laid
    // out of line behind __builtin_expect, 74.3 -> 73.9 us, +0.6 % frames)
    if (upda) {
      qa.c01.x = qa.c01.x + (a1.z * ala) * qa.T;
      qa.c01.y = qa.c01.y + (a1.w * ala) * qa.T;
      qa.c23.x = qa.c23.x + (a2.x * ala) * qa.T;
      qa.c23.y = qa.c23.y + (op * ala) * qa.T;
      qa.T = tta;
    }
    if (updb) {
      qb.c01.x = qb.c01.x + (a1.z * alb) * qb.T;
      qb.c01.y = qb.c01.y + (a1.w * alb) * qb.T;
      qb.c23.x = qb.c23.x + (a2.x * alb) * qb.T;
      qb.c23.y = qb.c23.y + (op * alb) * qb.T;
      qb.T = ttb;
    }
    qa.done = qa.done || brka;
    qb.done = qb.done || brkb;
    m = (qa.done && qb.done) ? 0ull : m;
  }
}

// wid = (tile slot) * 2 + half; st: the wave's LDS staging of one batch
template <bool HWEXP>
__device__ __forceinline__ void blend_wave_px2(const FrameParams& fp, const Buffers& b, int wid, float4 (*st)[64]) {
  const int slot = wid >> 1, half = wid & 1;
  if (slot >= fp.n_tiles) return;
  int tile;
  uint32_t s, L;
  if (fp.blend_seg) {
    // the slot's tile and list segment in one load (the sort launch's);
    // otherwise the queue entry, then the tile's start and end
    const uint4 sg = b.blend_seg[slot];
    tile = (int)sg.x;
    s = sg.y;
    L = sg.z;
  } else {
    tile = blend_tile_of(fp, b, slot);
    tile_segment(fp, b, tile, s, L);
  }
  const int lane = threadIdx.x & 63;
  const int tx = tile % fp.tiles_x, tyb = tile / fp.tiles_x;
  const int tile_x0 = tx * fp.tile_w;
  const int tile_y0 = (fp.band_ty0 + tyb * fp.band_stride) * fp.tile_h;
  const int pc = lane & 7, row = lane >> 3;  // pixel-pair column, row of the 16x8 half
  const int lx = 2 * pc, ly = 8 * half + row;
  const int px = tile_x0 + lx, py = tile_y0 + ly;
  Px qa, qb;
  qa.p = f32x2{(float)px, (float)py};
  qb.p = f32x2{(float)(px + 1), (float)py};
  qa.T = qb.T = 1.0f;
  qa.c01 = qa.c23 = qb.c01 = qb.c23 = f32x2{0.0f, 0.0f};
  const bool va = py < fp.height && px < fp.width, vb = py < fp.height && px + 1 < fp.width;
  qa.done = !va;
  qb.done = !vb;

  const uint32_t* __restrict__ list = b.list + s;
  auto load_idx = [&](uint32_t k) -> uint32_t { return blend_idx(fp, list, L, k); };
  const float4* __restrict__ ccol = (fp.sh_degree >= 0 && b.sh) ? b.col_out : b.colour;
  auto load_rec = [&](uint32_t g, float4& r0, float4& r1, float4& r2) {
    const float4* qq = b.rec + 2 * (size_t)g;
    r0 = qq[0];
    const float4 t = qq[1];    // k1 pcut boxx boxy
    const float4 c = ccol[g];  // r g b opacity
    r1 = make_float4(t.x, t.y, c.x, c.y);
    r2 = make_float4(c.z, c.w, t.z, t.w);
  };
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0;
  uint32_t g_cur = load_idx(lane);
  if (g_cur != 0xFFFFFFFFu) load_rec(g_cur, a0, a1, a2);
  uint32_t g_next = load_idx(64 + lane);

  uint32_t staged = 0;
  LaneCount lc;
  uint32_t wave_steps = 0, batches = 0;  // (GS_LANES builds)
  for (uint32_t base = 0; base < L; base += 64) {
    if (ballot64(!(qa.done && qb.done)) == 0ull) break;
    staged += min(64u, L - base);
    const bool have = g_cur != 0xFFFFFFFFu;
    st[0][lane] = make_float4(a0.x, a0.y, -0.5f * a0.z, -0.5f * a0.w);
    st[1][lane] = a1;
    st[2][lane] = a2;
    const uint32_t boxx = __float_as_uint(a2.z), boxy = __float_as_uint(a2.w);
    const int rx0 = (int)(boxx << 16) >> 16, rx1 = (int)boxx >> 16;
    const int ry0 = (int)(boxy << 16) >> 16, ry1 = (int)boxy >> 16;
    const bool rok = have && !(a2.y == 0.0f) && rx0 <= rx1 && ry0 <= ry1;
    const bool fast = ballot64(rok && !(a1.y >= -80.0f)) == 0ull;
    g_cur = g_next;
    a0 = a1 = a2 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g_cur != 0xFFFFFFFFu) load_rec(g_cur, a0, a1, a2);
    g_next = load_idx(base + 128 + lane);
    // pixel-pair column c meets the box iff floor((rx0 - bx) / 2) <= c <=
    // floor((rx1 - bx) / 2); rows per pixel
    const int bx = tile_x0, by = tile_y0 + 8 * half;
    const int xlo = rok ? (rx0 - bx) >> 1 : 0x40000000, xsp = rok ? ((rx1 - bx) >> 1) - xlo : 0;
    const int ylo = rok ? ry0 - by : 0x40000000, ysp = rok ? (ry1 - by) - ylo : 0;
    uint32_t tab = 0u;
    BallotTab<0, 0, 8>::run(tab, xlo, xsp);
    BallotTab<8, 0, 8>::run(tab, ylo, ysp);
    const int ac = 8 * pc, ar = 8 * (8 + row);
    const uint32_t mcl = (uint32_t)__builtin_amdgcn_ds_bpermute(ac, (int)tab);
    const uint32_t mch = (uint32_t)__builtin_amdgcn_ds_bpermute(ac + 4, (int)tab);
    const uint32_t mrl = (uint32_t)__builtin_amdgcn_ds_bpermute(ar, (int)tab);
    const uint32_t mrh = (uint32_t)__builtin_amdgcn_ds_bpermute(ar + 4, (int)tab);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool both = qa.done && qb.done;
    const uint32_t m_lo = both ? 0u : (mcl & mrl), m_hi = both ? 0u : (mch & mrh);
    const uint32_t steps0 = lc.steps;
    if (HWEXP) {
      blend_records_px2<kExpHw>(qa, qb, st, m_lo, m_hi, lc);
    } else if (fast) {
      blend_records_px2<kExpInRange>(qa, qb, st, m_lo, m_hi, lc);
    } else {
      blend_records_px2<kExpExact>(qa, qb, st, m_lo, m_hi, lc);
    }
    if constexpr (GS_LANES != 0) {  // the batch's wave steps: its longest lane walk
      uint32_t d = lc.steps - steps0;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) d = max(d, (uint32_t)__shfl_xor((int)d, o, 64));
      wave_steps += d;
      ++batches;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (GS_LANES != 0) {
    if (b.lanes) {
      unsigned long long v[4] = {lc.steps, lc.evals, lc.box, lc.hits};
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v[k] += (unsigned long long)__shfl_xor((long long)v[k], o, 64);
      if (lane == 0) {
        atomicAdd(&b.lanes[0], (unsigned long long)wave_steps);
        for (int k = 0; k < 4; ++k) atomicAdd(&b.lanes[1 + k], v[k]);
        atomicAdd(&b.lanes[5], (unsigned long long)batches);
        atomicAdd(&b.lanes[6], 1ull);
      }
    }
  }
  // profiled frames: the staged records at this tile's wave slots 0 / 1 (2 / 3
  // unused: zeroed, the host takes the tile's largest)
  if (fp.count_records && lane == 0) {
    b.blend_count[4 * slot + half] = staged;
    b.blend_count[4 * slot + 2 + half] = 0u;
  }
  // RGBA f32 through the wave's (now idle) staging LDS: a lane's two pixels
  // are neighbours, so storing them directly would write every other 16 B of
  // a line per instruction, and streaming stores do not merge the halves in
  // L2 (PMC WRITE_SIZE 40.9 -> 73.6 MB per launch at config 3).  Row-major in
  // LDS, each store instruction covers four whole 256-B pixel rows.
  if (fp.write_rgba) {
    float4* const sp = &st[0][0];  // st[0], st[1]: the half tile's 128 pixels
    sp[row * 16 + lx] = pixel_rgba(qa);
    sp[row * 16 + lx + 1] = pixel_rgba(qb);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 64 * h + lane, r = k >> 4, c = k & 15;
      const int x = tile_x0 + c, y = tile_y0 + 8 * half + r;
      if (y < fp.height && x < fp.width)
        store_stream(b.rgba + (size_t)(tyb * fp.tile_h + 8 * half + r) * fp.width + x, sp[k]);
    }
  }
  const bool dw = tile_x0 + 16 <= fp.width && ((uintptr_t)b.bgr & 3u) == 0u && (fp.bgr_pitch & 3) == 0;
  if (dw) {
    uint8_t* const sb = reinterpret_cast<uint8_t*>(&st[2][0]);  // 8 rows x 48 B (st[2] is idle)
    const float4 oa = pixel_rgba(qa), ob = pixel_rgba(qb);
    uint8_t* const d = sb + row * 48 + 3 * lx;
    d[0] = to_u8(oa.z);  // RGBA2BGR
    d[1] = to_u8(oa.y);
    d[2] = to_u8(oa.x);
    d[3] = to_u8(ob.z);
    d[4] = to_u8(ob.y);
    d[5] = to_u8(ob.x);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 64 * h + lane;  // dword k of the half tile's 96: row k / 12, dword k % 12
      if (k < 96) {
        const int r = k / 12, c = k - 12 * r;
        if (tile_y0 + 8 * half + r < fp.height)
          *reinterpret_cast<uint32_t*>(b.bgr + (size_t)(tyb * fp.tile_h + 8 * half + r) * fp.bgr_pitch +
                                       3 * (size_t)tile_x0 + 4 * c) = reinterpret_cast<const uint32_t*>(sb)[k];
      }
    }
  } else {
    if (va) store_bgr(fp, b, px, tyb * fp.tile_h + ly, qa);
    if (vb) store_bgr(fp, b, px + 1, tyb * fp.tile_h + ly, qb);
  }
}

template <bool HWEXP>
__global__ __launch_bounds__(64 * GS_PX2_WPG) void gs_blend_px2_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBlend);
  __shared__ float4 s_rec[GS_PX2_WPG][3][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  blend_wave_px2<HWEXP>(fp, b, blockIdx.x * GS_PX2_WPG + wave, s_rec[wave]);
}

// The sort inside the blend (FrameParams::blend_sort; one workgroup = the
// four 8x8 blocks of one 16x16 tile): the workgroup first sorts its tile's
// list -- as gs_sort_tiles_kernel would: <= 64 keys in wave 0's registers,
// <= kSortLdsCap by the four waves (128-key register runs, then
// merge-path levels in LDS), equal depths re-sorted by input index, a list
// > kSortLdsCap radix-sorted here unless the big-list launches took it --
// then its four waves blend it.  No sort launch, and the list is read back
// while it is still in L2.  The LDS of the sort is then reused as the
// waves' record staging.
constexpr int kBlendLdsWords = 2 * kSortLdsCap;  // u32 words (16 KB)
static_assert(GS_BLEND_WPG == 4, "blend_sort: one workgroup per 16x16 tile (the renderer's chunks_per_tile == 4)");
static_assert(kBlendLdsWords * 4 >= GS_BLEND_WPG * 3 * 64 * 16, "the staging fits the sort's LDS");
static_assert(kBlendLdsWords >= 8 * 256 + 256 + 4 * 256, "the radix histograms fit the sort's LDS");

template <bool DIRECT = false>
__device__ __forceinline__ void blend_sort_tile(const FrameParams& fp, const Buffers& b, int tile,
                                                unsigned long long* keys) {
  uint32_t s, L;
  tile_segment<DIRECT>(fp, b, tile, s, L);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (L > (uint32_t)kSortLdsCap) {
    // a big list: sorted by the big-list launches (big_separate), else here
    if (!fp.big_separate) {
      uint32_t* const hist = (uint32_t*)keys;
      radix_sort_tile<256, 1, DIRECT>(fp, b, tile, hist, hist + 8 * 256, (uint32_t(*)[256])(hist + 9 * 256));  // (1 key per lane and round: compact code for this rare path)
    }
    return;
  }
  // (two of the sort launch's networks only: the kernel's code stays small)
  if (L <= 64u) {
    if (wave == 0) wave_sort_list<1>(b, b.pairs + s, s, L, lane, keys);
    return;
  }
  const bool ok = merge_sort_tile<256, 2, kOutDevice>(b, s, L, keys);
  if (!ok) {
    __syncthreads();  // a long run of equal depths: again with input-index keys
    merge_sort_tile<256, 2, kOutInput, kSrcRekey>(b, s, L, keys);
  }
}

// FrameParams::bin_direct: what the scan would have written.  Each of the
// blend's workgroups leaves its tile's list lengths and takes a ticket; the
// last one sums the frame's counters as gs_agg_scan_kernel lays them out,
// writes them to the device, the mapped host mirror and the footer, and
// resets the ticket and the overflow flag.
// The per-tile values reach the totals write-through (system scope, past the
// XCDs' L2s, sc0 sc1 loads and stores), so no workgroup releases its L2 with
// a fence (MI355X_MICROARCH.md, the hand-off table's first row)
__device__ __forceinline__ uint32_t direct_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int NT>
__device__ __forceinline__ void direct_totals(const FrameParams& fp, const Buffers& b, uint32_t* lds) {
  constexpr int NW = NT / 64;
  const int T = fp.n_tiles, nb = (fp.n + 255) / 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned long long sum = 0, rsum = 0;
  uint32_t mx = 0, n_big = 0, n_med = 0, n_small = 0, vis = 0;
  // (four loads in flight per thread: one workgroup, latency-bound)
  for (int t0 = tid; t0 < T; t0 += 4 * NT) {
    uint32_t Lr[4], Rr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = t0 + j * NT;
      Lr[j] = t < T ? direct_load(&b.tile_count[t]) : 0u;
      Rr[j] = t < T ? direct_load(&b.tile_ref[t]) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t L = Lr[j];
      sum += L;
      rsum += Rr[j];
      mx = max(mx, L);
      n_big += L > (uint32_t)kSortLdsCap ? 1u : 0u;
      n_med += (L > kSortRegCap && L <= (uint32_t)kSortLdsCap) ? 1u : 0u;
      n_small += (t0 + j * NT < T && L <= kSortRegCap) ? 1u : 0u;
    }
  }
  // (16 loads in flight per thread: 1M Gaussians' 3 907 block counts in one round)
  for (int k0 = tid; k0 < nb; k0 += 16 * NT) {
    uint32_t vr[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) vr[j] = k0 + j * NT < nb ? b.block_rendered[k0 + j * NT] : 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j) vis += vr[j];
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    sum += (unsigned long long)__shfl_xor((long long)sum, d, 64);
    rsum += (unsigned long long)__shfl_xor((long long)rsum, d, 64);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
    n_big += (uint32_t)__shfl_xor((int)n_big, d, 64);
    n_med += (uint32_t)__shfl_xor((int)n_med, d, 64);
    n_small += (uint32_t)__shfl_xor((int)n_small, d, 64);
    vis += (uint32_t)__shfl_xor((int)vis, d, 64);
  }
  unsigned long long* const w64 = reinterpret_cast<unsigned long long*>(lds);  // [NW][2]
  uint32_t* const w32 = lds + 4 * NW;                                          // [NW][5]
  __syncthreads();
  if (lane == 0) {
    w64[2 * wave] = sum;
    w64[2 * wave + 1] = rsum;
    w32[5 * wave] = mx;
    w32[5 * wave + 1] = n_big;
    w32[5 * wave + 2] = n_med;
    w32[5 * wave + 3] = n_small;
    w32[5 * wave + 4] = vis;
  }
  __syncthreads();
  if (tid == 0) {
    unsigned long long tot = 0, rtot = 0;
    uint32_t m = 0, nbg = 0, nmd = 0, nsm = 0, v = 0;
    for (int w = 0; w < NW; ++w) {
      tot += w64[2 * w];
      rtot += w64[2 * w + 1];
      m = max(m, w32[5 * w]);
      nbg += w32[5 * w + 1];
      nmd += w32[5 * w + 2];
      nsm += w32[5 * w + 3];
      v += w32[5 * w + 4];
    }
    const bool ovf = b.dir_word[1] != 0u || tot > fp.pair_cap;
    const uint4 c0 = make_uint4(nbg, 0u, v, ovf ? 1u : 0u);
    const uint4 c1 = make_uint4(m, (uint32_t)tot, (uint32_t)(tot >> 32), nmd);
    const uint4 c2 = make_uint4(0u, nsm, (uint32_t)rtot, (uint32_t)(rtot >> 32));
    const uint4 c3 = make_uint4(0u, 0u, 0u, 0u);
    if (ovf) {  // sticky until the host's sync
      *b.host_sticky = 1u;
      if (b.group_sticky) *b.group_sticky = 1u;
    }
    uint4* const cv = reinterpret_cast<uint4*>(b.counters);
    cv[0] = c0;
    cv[1] = c1;
    cv[2] = c2;
    cv[3] = c3;
    if (b.footer) {
      uint4* const fv = reinterpret_cast<uint4*>(b.footer);
      fv[0] = c0;
      fv[1] = c1;
      fv[2] = c2;
      fv[3] = c3;
    }
    const uint32_t cc[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                             c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, fp.frame_seq};
    for (int k = 0; k < 16; ++k) b.host_counters[k] = cc[k];
    b.dir_word[1] = 0u;
  }
}

// the tile's counter (c: read by thread 0 before the sort), zeroed for the
// next frame's projection once every wave is past its reads of it; its
// reference length (the histogram) and binned length (for the totals), stored
// write-through and acknowledged before the ticket (a relaxed agent-scope
// add).  An agent-scope release per workgroup instead (buffer_wbl2: the XCD's
// L2 written back) made band 3's blend 44 -> 57 us; the totals in a
// one-workgroup kernel after the blend cost 8.6 us more per frame than here.
__device__ __forceinline__ void direct_finish(const FrameParams& fp, const Buffers& b, int tile, unsigned long long c,
                                              uint32_t* lds) {
#ifndef GS_X_DIRECT_FIN
#define GS_X_DIRECT_FIN 0
#endif
#if GS_X_DIRECT_FIN  // (measurement builds, wrong stats: 1 no ticket or totals; 2 nor the barrier)
  if (GS_X_DIRECT_FIN == 1) __syncthreads();
  if (threadIdx.x == 0) {
    b.tile_cnt64[tile] = 0ull;
    b.tile_ref[tile] = (uint32_t)(c >> 32);
    b.tile_count[tile] = (uint32_t)c;
  }
  return;
#endif
  __shared__ uint32_t s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t ref = (uint32_t)(c >> 32);
    b.tile_cnt64[tile] = 0ull;
    if (b.footer) b.footer[16 + tile] = ref;
    __hip_atomic_store(&b.tile_ref[tile], ref, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&b.tile_count[tile], (uint32_t)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_waitcnt(0);  // both acknowledged before the ticket
    const uint32_t tk = __hip_atomic_fetch_add(&b.dir_word[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = tk == (uint32_t)fp.n_tiles - 1u ? 1u : 0u;
  }
  __syncthreads();
  if (s_last) {
    direct_totals<256>(fp, b, lds);
    if (threadIdx.x == 0) b.dir_word[0] = 0u;
  }
}

// HWEXP: GS_FLAG_FAST_EXP (its own kernel: the default path's code is unchanged)
template <int BQW, bool HWEXP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GS_BLEND_WPE, 8))) void gs_blend_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBlend);
  __shared__ float4 s_rec[GS_BLEND_WPG][3][64];
  const int wave = GS_BLEND_WPG == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  blend_wave<BQW, HWEXP>(fp, b, blockIdx.x * GS_BLEND_WPG + wave, s_rec[wave]);
}

// The blend with the tile sort inside (FrameParams::blend_sort, 16x16 tiles):
// its own symbol, so the whole-frame blend does not carry the sort's ~20 KB
// of code (the CU pair's instruction cache is shared with the other frames'
// kernels: config 3 7 703 -> 7 839 frames/s, blend 79.2 -> 76.7 us without it)
#ifndef GS_X_BSORT
#define GS_X_BSORT 0
#endif
#if GS_X_BSORT
__device__ uint32_t g_x_bsort_frames = 0;
#endif
template <bool HWEXP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GS_BLEND_WPE, 8))) void gs_blend_sort_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBlend);
  __shared__ __attribute__((aligned(16))) uint32_t lds[kBlendLdsWords];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int slot = (int)blockIdx.x;  // (chunks_per_tile == GS_BLEND_WPG)
  if (slot >= fp.n_tiles) return;
#if GS_X_BSORT
  // (measurement builds: 1 = no sort after a renderer's first frames -- a
  // fixed camera's lists are the previous frame's -- 2 = no blend walk)
  const bool x_sort = GS_X_BSORT == 2 || __hip_atomic_load(&g_x_bsort_frames, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 8u;
  if (x_sort)
#endif
  blend_sort_tile(fp, b, blend_tile_of(fp, b, slot), reinterpret_cast<unsigned long long*>(lds));
  // the list's stores are done (s_waitcnt in the barrier) before any wave
  // reads it, and the sort's LDS is free for the staging
  __syncthreads();
#if GS_X_BSORT
  if (slot == 0 && threadIdx.x == 0) atomicAdd(&g_x_bsort_frames, 1u);
  if (GS_X_BSORT == 2) return;
#endif
  blend_wave<4, HWEXP>(fp, b, slot * GS_BLEND_WPG + wave, reinterpret_cast<float4(*)[64]>(lds) + 3 * wave);
}

// The blend with the sort inside for a direct-binned band (FrameParams::
// bin_direct): a workgroup per tile, the tile's pairs from its segment, then
// direct_finish.  Its own symbol (the other kernels keep their
// code; profiles tell it apart).
template <bool HWEXP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GS_BLEND_WPE, 8))) void gs_blend_direct_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBlend);
  __shared__ __attribute__((aligned(16))) uint32_t lds[kBlendLdsWords];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // (chunks_per_tile == GS_BLEND_WPG; tile order: the longest-lists-first
  // order of the view's last scan took band 3's pipelined frame 28.7 -> 33.5 us)
  const int tile = (int)blockIdx.x;
  const unsigned long long c = threadIdx.x == 0 ? b.tile_cnt64[tile] : 0ull;
#ifndef GS_X_DSPLIT
#define GS_X_DSPLIT 0
#endif
  // (GS_X_DSPLIT measurement builds, wrong frames: 1 no sort, 2 no blend walk)
  if (GS_X_DSPLIT != 1) blend_sort_tile<true>(fp, b, tile, reinterpret_cast<unsigned long long*>(lds));
  __syncthreads();
  if (GS_X_DSPLIT != 2)
    blend_wave<4, HWEXP, true>(fp, b, tile * GS_BLEND_WPG + wave, reinterpret_cast<float4(*)[64]>(lds) + 3 * wave);
  direct_finish(fp, b, tile, c, lds);
}


// the lazy big lists' continuation (its own symbol, so profiles tell it from
// the prefix blend).  A grid-stride loop over the waves of the big lists
// only: a grid of every tile's waves, nearly all of which exit at once, cost
// ~70 us at config 5 (32 400 short-lived workgroups, each waiting on its
// counters load, 4 resident per CU).
template <bool HWEXP>
__global__ __launch_bounds__(256) void gs_blend_cont_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrBlendCont);
  __shared__ float4 s_rec[GS_BLEND_WPG][3][64];
  if (fp.big_pass == 2 && b.counters[1] == 0u) return;  // no list outlived its window
  const int wave = GS_BLEND_WPG == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nblk = (int)((b.counters[0] * (uint32_t)fp.chunks_per_tile + GS_BLEND_WPG - 1) / GS_BLEND_WPG);
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x)
    blend_wave<4, HWEXP>(fp, b, blk * GS_BLEND_WPG + wave, s_rec[wave]);
}


__global__ __launch_bounds__(64) void gs_copy_word_kernel(uint32_t* dst, const uint32_t* src) {
  // a device-scope load: the word was written by other kernels on other streams
  if (threadIdx.x == 0) *dst = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

void launch_copy_word(hipStream_t s, uint32_t* dst, const uint32_t* src) {
  gs_copy_word_kernel<<<1, 64, 0, s>>>(dst, src);
}

// FrameParams::cov_cache: ComputeCov3D (ipu_geometry.hpp:315-323, the scales
// divided by fxy[1], codelets.cpp:463) of every Gaussian, once per fxy[1]:
// the same function on the same inputs as the projection's, so the same
// bits.  It depends on the rotation, the scales and fxy[1] only -- never on
// the camera -- and took ~29 % of the projection's VALU per frame.
namespace {
template <bool P2>
__global__ __launch_bounds__(256) void gs_cov3d_kernel(FrameParams fp, Buffers b) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= fp.n) return;
  const size_t nn = (size_t)fp.n;
  const float4 sg = b.scale_gid[i];
  if (sg.w <= 0.0f) {  // (an empty slot: the projection skips it)
    b.cov3[8 * nn + i] = -1.0f;
    return;
  }
  const float4 rot = b.rot[i];
  const M3 C3 = cov3d(rot, div_p2<P2>(sg.x, fp.scale_div, fp.inv_sd), div_p2<P2>(sg.y, fp.scale_div, fp.inv_sd),
                      div_p2<P2>(sg.z, fp.scale_div, fp.inv_sd));
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) b.cov3[(size_t)(c * 3 + r) * nn + i] = C3.m[c][r];
}
}  // namespace

void launch_cov3d(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  if (fp.n == 0) return;
  const int nb = (fp.n + 255) / 256;
  if (fp.pow2)
    gs_cov3d_kernel<true><<<nb, 256, 0, s>>>(fp, b);
  else
    gs_cov3d_kernel<false><<<nb, 256, 0, s>>>(fp, b);
}

int project_kind(const FrameParams& fp, const Buffers& b) {
  const bool plain = !fp.full_record && !(fp.sh_degree >= 0 && b.sh) && !fp.bin_global;
  if (fp.pow2 && plain && !fp.band_cull && !fp.bin_agg) return kProjLean;
  if (fp.pow2 && plain && fp.band_cull && fp.bin_agg) return fp.bin_direct ? kProjDirect : kProjBand;
  return kProjAny;
}

void launch_project(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  if (fp.n == 0) return;
  const int nb = (fp.n + 255) / 256;
  const int kind = project_kind(fp, b);
  if (kind == kProjLean) {
    gs_project_kernel<true><<<nb, 256, 0, s>>>(fp, b);
  } else if (kind == kProjBand) {
    if (GS_X_BAND == 3) {  // (measurement builds: one projection per renderer)
      static std::vector<const void*> seen;
      if (std::find(seen.begin(), seen.end(), (const void*)b.rec) != seen.end()) return;
      seen.push_back(b.rec);
    }
    gs_project_band_kernel<true><<<nb, 256, 0, s>>>(fp, b);
  } else if (kind == kProjDirect) {
    gs_project_direct_kernel<true><<<nb, 256, 0, s>>>(fp, b);
  } else if (fp.pow2) {
    gs_project_any_kernel<true><<<nb, 256, 0, s>>>(fp, b);
  } else {
    gs_project_any_kernel<false><<<nb, 256, 0, s>>>(fp, b);
  }
}

size_t bin_lds_bytes(int n_tiles) { return (size_t)((n_tiles + 1) / 2) * 4; }

bool bin_lds_fits(int n_tiles) { return bin_lds_bytes(n_tiles) <= kBinLdsMax; }

hipError_t init_kernel_attributes() {
  hipError_t e = hipFuncSetAttribute((const void*)gs_count_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBinLdsMax);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)gs_emit_chunk_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBinLdsMax);
}

void launch_scan(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  if (fp.bin_agg && fp.bin_direct) return;  // (the blend's workgroups write the counters)
  if (fp.bin_agg) {
    // (1024 threads, 4 tiles each; 256 threads x 8 -- a workgroup easier to
    // place beside the other frames' waves -- ran the scan stage 10.5 ->
    // 15.7 us and 8 bands of config 4 38.1 -> 39.7 us per frame)
    gs_agg_scan_kernel<1024, 4><<<1, 1024, 0, s>>>(fp, b);
    return;
  }
  if (!fp.bin_global && fp.n_chunks > 0 && fp.n_tiles > 0) {
    const size_t lds = fp.pair_cull ? (size_t)fp.n_tiles * 4 : bin_lds_bytes(fp.n_tiles);
    gs_count_kernel<<<fp.n_chunks, 1024, lds, s>>>(fp, b);
    gs_colscan_kernel<<<(fp.n_tiles + 63) / 64, 1024, 0, s>>>(fp, b);
    gs_scan_multi_kernel<<<(fp.n_tiles + 63) / 64, 256, 0, s>>>(fp, b);
    return;
  }
  gs_scan_kernel<<<1, 1024, 0, s>>>(fp, b);
}

void launch_emit(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  if (fp.n == 0) return;
  if (fp.bin_agg && fp.bin_direct) return;  // (the projection placed the pairs)
  if (fp.bin_agg) {
    const int nb = (fp.n + 255) / 256;
    gs_agg_emit_kernel<<<fp.emit_grid > 0 ? std::min(nb, fp.emit_grid) : nb, 256, 0, s>>>(fp, b);
    return;
  }
  if (!fp.bin_global) {
    if (fp.n_chunks > 0 && fp.n_tiles > 0)
      gs_emit_chunk_kernel<<<fp.n_chunks, 1024,
                             fp.emit_wide ? (size_t)fp.n_tiles * 4 : bin_lds_bytes(fp.n_tiles), s>>>(fp, b);
    return;
  }
  gs_emit_kernel<<<(fp.n + 255) / 256, 256, 0, s>>>(fp, b);
}

// the sample sort's bucket passes (every big list, or the flagged ones);
// grid-stride kernels, so any grid is correct
void launch_big_buckets(const FrameParams& fp, const Buffers& b, hipStream_t s, unsigned grid) {
  gs_big_count_kernel<<<grid, 256, 0, s>>>(fp, b);
  gs_big_bscan_kernel<<<256, 256, 0, s>>>(fp, b);
  gs_big_scatter_kernel<<<grid, 256, 0, s>>>(fp, b);
  gs_big_bsort_kernel<<<grid, 256, 0, s>>>(fp, b);
}

void launch_sort(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  launch_sort_big(fp, b, s);
  launch_sort_tiles(fp, b, s);
}

void launch_sort_big(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  if (fp.n_tiles == 0) return;
  if (fp.big_separate) {
    // work items = 2048-key segments of the big lists; the passes run until a
    // run covers the longest list the pair buffer can hold (passes after a
    // list's last one skip it)
    gs_big_prefix_kernel<<<1, 1024, 0, s>>>(fp, b);
    gs_big_split_kernel<<<2048, 256, 0, s>>>(fp, b);  // (one workgroup per list: 1024 -> 2048, sort stage -10 us at config 5)
    if (fp.lazy) {  // only the prefixes now; the rest after the blend (launch_blend_cont)
      gs_big_select_kernel<<<4096, 256, 0, s>>>(fp, b);
      gs_big_psort_kernel<<<2048, 256, 0, s>>>(fp, b);
    } else {
      launch_big_buckets(fp, b, s, 4096);
    }
  }
}

void launch_sort_tiles(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  if (fp.n_tiles == 0 || fp.blend_sort) return;  // (blend_sort: each blend workgroup sorts its tile)
  // big + medium + ceil(small / waves) <= n_tiles + 1 workgroups do work
  gs_sort_tiles_kernel<<<fp.n_tiles + (fp.n_tiles + 3) / 4, 256, 0, s>>>(fp, b);
}

void launch_blend(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  const long waves = (long)fp.n_tiles * fp.chunks_per_tile;
  if (waves == 0) return;
  const unsigned grid = (unsigned)((waves + GS_BLEND_WPG - 1) / GS_BLEND_WPG);
  const unsigned block = 64 * GS_BLEND_WPG;
  if (fp.blend_px2) {  // (16x16 tiles, whole frames without lazy lists: two waves per tile)
    const unsigned g2 = (unsigned)((2L * fp.n_tiles + GS_PX2_WPG - 1) / GS_PX2_WPG);
    if (fp.fast_exp)
      gs_blend_px2_kernel<true><<<g2, 64 * GS_PX2_WPG, 0, s>>>(fp, b);
    else
      gs_blend_px2_kernel<false><<<g2, 64 * GS_PX2_WPG, 0, s>>>(fp, b);
    return;
  }
  if (fp.blend_sort && fp.bin_direct) {  // (a direct-binned band: its own kernel)
    if (fp.fast_exp)
      gs_blend_direct_kernel<true><<<grid, block, 0, s>>>(fp, b);
    else
      gs_blend_direct_kernel<false><<<grid, block, 0, s>>>(fp, b);
    return;
  }
  if (fp.blend_sort) {  // (blend_bqw == 4, chunks_per_tile == GS_BLEND_WPG: one workgroup per tile)
    if (fp.fast_exp)
      gs_blend_sort_kernel<true><<<grid, block, 0, s>>>(fp, b);
    else
      gs_blend_sort_kernel<false><<<grid, block, 0, s>>>(fp, b);
    return;
  }
  if (fp.fast_exp) {
    if (fp.blend_bqw == 4)
      gs_blend_kernel<4, true><<<grid, block, 0, s>>>(fp, b);
    else if (fp.blend_bqw == 8)
      gs_blend_kernel<8, true><<<grid, block, 0, s>>>(fp, b);
    else
      gs_blend_kernel<0, true><<<grid, block, 0, s>>>(fp, b);
  } else {
    if (fp.blend_bqw == 4)
      gs_blend_kernel<4, false><<<grid, block, 0, s>>>(fp, b);
    else if (fp.blend_bqw == 8)
      gs_blend_kernel<8, false><<<grid, block, 0, s>>>(fp, b);
    else
      gs_blend_kernel<0, false><<<grid, block, 0, s>>>(fp, b);
  }
}

void launch_blend_cont(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  const long waves = (long)fp.n_tiles * fp.chunks_per_tile;
  if (waves == 0 || !fp.lazy) return;
  const unsigned grid = (unsigned)std::min<long>((waves + GS_BLEND_WPG - 1) / GS_BLEND_WPG, 2048);
  const unsigned block = 64 * GS_BLEND_WPG;
  // the big lists whose blend outlived the prefix: sorted in full, then
  // their saved waves continue (nothing to do when none was flagged)
  // pass 1: the flagged lists' windows, sorted, then their saved waves
  // continue; pass 2 (no-ops unless a wave outlived its window): those lists
  // sorted in full past the window, and their waves continue again
  FrameParams f1 = fp;
  f1.big_pass = 1;
  gs_big_cont_kernel<<<2048, 256, 0, s>>>(f1, b);
  f1.blend_cont = 1;
  if (fp.fast_exp)
    gs_blend_cont_kernel<true><<<grid, block, 0, s>>>(f1, b);
  else
    gs_blend_cont_kernel<false><<<grid, block, 0, s>>>(f1, b);
  // Pass 2 runs for a few lists per frame (config 5: ~3 of ~110 continued
  // lists); its kernels return at once when counters[1] says no list
  // outlived its window.  Full grids: 256-workgroup grid-stride grids made
  // the frames that do have pass-2 lists slower (config 5: continuation
  // 204 -> 246 us, 1 535 -> 1 492 frames/s)
  FrameParams f2 = fp;
  f2.big_pass = 2;
  gs_big_prefix_kernel<<<1, 1024, 0, s>>>(f2, b);
  // (the splitters of every big list were chosen by the frame's first split pass)
  const unsigned g2 = 4096u;
  launch_big_buckets(f2, b, s, g2);
  f2.blend_cont = 1;
  const unsigned grid2 = std::min(grid, g2);
  if (fp.fast_exp)
    gs_blend_cont_kernel<true><<<grid2, block, 0, s>>>(f2, b);
  else
    gs_blend_cont_kernel<false><<<grid2, block, 0, s>>>(f2, b);
}

}  // namespace gsk
