// gs_oracle.cpp -- CPU ORACLE (test infrastructure only; see gs_oracle.h).
//
// Independent restatement of the reference rasteriser, written line by line
// from the reference sources cited at each function.  It shares NO code with
// the product (gaussian_splat_ipu_amd/csrc); agreement between the two is the
// parity evidence.  Compile with -ffp-contract=off (no FMA contraction) so the
// expression order below is the arithmetic that happens.
#include "gs_oracle.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#include <sched.h>
#endif

namespace {

// ---------------------------------------------------------------- glm restatement
// glm 0.9.9 is column-major: m[c][r].  (submodule external/glm is empty in the
// reference snapshot, .gitmodules:1-3; version unpinned -> see DESIGN.md)
struct V4 { float x, y, z, w; };
struct M4 { float m[4][4]; };
struct M3 { float m[3][3]; };

// glm::transpose(glm::make_mat4(p)) -- codelets.cpp:625-628
M4 m4_from_rowmajor(const float* rm) {
  M4 a;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) a.m[c][r] = rm[r * 4 + c];
  return a;
}

// glm mat4 * mat4: Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3]
M4 m4_mul(const M4& A, const M4& B) {
  M4 R;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) {
      float s = A.m[0][r] * B.m[c][0];
      s = s + A.m[1][r] * B.m[c][1];
      s = s + A.m[2][r] * B.m[c][2];
      s = s + A.m[3][r] * B.m[c][3];
      R.m[c][r] = s;
    }
  return R;
}

// glm mat4 * vec4: (m0*x + m1*y) + (m2*z + m3*w)
V4 m4_mul_v4(const M4& m, V4 v) {
  float o[4];
  for (int r = 0; r < 4; ++r) {
    float a = m.m[0][r] * v.x + m.m[1][r] * v.y;
    float b = m.m[2][r] * v.z + m.m[3][r] * v.w;
    o[r] = a + b;
  }
  return V4{o[0], o[1], o[2], o[3]};
}

// glm mat3 * mat3: Result[c][r] = (A[0][r]*B[c][0] + A[1][r]*B[c][1]) + A[2][r]*B[c][2]
M3 m3_mul(const M3& A, const M3& B) {
  M3 R;
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) {
      float s = A.m[0][r] * B.m[c][0];
      s = s + A.m[1][r] * B.m[c][1];
      s = s + A.m[2][r] * B.m[c][2];
      R.m[c][r] = s;
    }
  return R;
}

M3 m3_transpose(const M3& A) {
  M3 R;
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) R.m[c][r] = A.m[r][c];
  return R;
}

// splat::Gaussian3D::min/max and Gaussian2D::max (ipu_geometry.hpp:242-244,325-331)
inline float smax(float a, float b) { return a > b ? a : b; }
inline float smin(float a, float b) { return a < b ? a : b; }

// Gaussian3D::ComputeCov3D (ipu_geometry.hpp:315-323)
M3 compute_cov3d(const float rot[4], const float scale[3]) {
  // glm::quat q(w=rot.x, x=rot.y, y=rot.z, z=rot.w)
  const float qw = rot[0], qx = rot[1], qy = rot[2], qz = rot[3];
  // glm::normalize(quat): len = sqrt(dot(q,q)), dot = (ww + xx) + (yy + zz)
  const float dot = (qw * qw + qx * qx) + (qy * qy + qz * qz);
  const float len = std::sqrt(dot);
  float w, x, y, z;
  if (len <= 0.0f) {
    w = 1.0f; x = 0.0f; y = 0.0f; z = 0.0f;
  } else {
    const float inv = 1.0f / len;
    w = qw * inv; x = qx * inv; y = qy * inv; z = qz * inv;
  }
  // glm::mat3_cast
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
  std::memset(&S, 0, sizeof(S));
  S.m[0][0] = or_expf(scale[0]);
  S.m[1][1] = or_expf(scale[1]);
  S.m[2][2] = or_expf(scale[2]);
  // R * S * transpose(S) * transpose(R), left to right
  return m3_mul(m3_mul(m3_mul(R, S), m3_transpose(S)), m3_transpose(R));
}

struct FrameC {
  M4 mvp;
  float tanfov, focal_x, focal_y, guard_thr;
  float W, H, tw, th;
  int tiles_x, tiles_y, by0, by1;
};

FrameC make_frame(const or_frame* f) {
  FrameC c;
  const M4 view = m4_from_rowmajor(f->view_rm);
  const M4 proj = m4_from_rowmajor(f->proj_rm);
  c.mvp = m4_mul(proj, view);  // codelets.cpp:443 and ipu_geometry.hpp:336
  or_frame_scalars(f, &c.tanfov, &c.focal_x, &c.focal_y, &c.guard_thr);
  c.W = (float)f->width;
  c.H = (float)f->height;
  c.tw = (float)f->tile_w;
  c.th = (float)f->tile_h;
  c.tiles_x = (f->width + f->tile_w - 1) / f->tile_w;    // ceil grid (SURVEY §7 partial tiles)
  c.tiles_y = (f->height + f->tile_h - 1) / f->tile_h;
  c.by0 = f->band_ty0;
  c.by1 = (f->band_ty1 > f->band_ty0) ? f->band_ty1 : c.tiles_y;
  if (c.by1 > c.tiles_y) c.by1 = c.tiles_y;
  return c;
}

// Gaussian3D::ComputeCov2D (ipu_geometry.hpp:333-383) -- clip-space "EWA"
void compute_cov2d(const M4& mv, const float mean[4], const float rot[4], const float scale[3],
                   float tan_fov, float fx, float fy, float out[3]) {
  V4 t4 = m4_mul_v4(mv, V4{mean[0], mean[1], mean[2], 1.0f});
  float tx = t4.x, ty = t4.y, tz = t4.z;
  const float limx = 1.3f * tan_fov;
  const float limy = 1.3f * tan_fov;
  const float txtz = tx / tz;
  const float tytz = ty / tz;
  tx = smin(limx, smax(-limx, txtz)) * tz;
  ty = smin(limy, smax(-limy, tytz)) * tz;
  M3 J;
  J.m[0][0] = fx / tz;  J.m[0][1] = 0.0f;      J.m[0][2] = -(fx * tx) / (tz * tz);
  J.m[1][0] = 0.0f;     J.m[1][1] = fy / tz;   J.m[1][2] = -(fy * ty) / (tz * tz);
  J.m[2][0] = 0.0f;     J.m[2][1] = 0.0f;      J.m[2][2] = 0.0f;
  M3 W;  // glm::mat3(mv): upper-left, no transpose
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) W.m[c][r] = mv.m[c][r];
  const M3 T = m3_mul(W, J);
  const M3 cov3d = compute_cov3d(rot, scale);
  M3 cov = m3_mul(m3_mul(m3_transpose(T), m3_transpose(cov3d)), T);
  cov.m[0][0] += 0.3f;
  cov.m[1][1] += 0.3f;
  out[0] = cov.m[0][0];
  out[1] = cov.m[0][1];
  out[2] = cov.m[1][1];
}

void project_one(const float* g, const FrameC& c, float scale_div, or_proj* o) {
  std::memset(o, 0, sizeof(*o));
  o->rect[0] = 1; o->rect[2] = 0;  // empty
  const float* mean = g + 0;    // Gaussian3D::mean   (ipu_geometry.hpp:307)
  const float* colour = g + 4;  // Gaussian3D::colour
  const float* rot = g + 8;     // Gaussian3D::rot
  const float* scale = g + 12;  // Gaussian3D::scale
  const float gid = g[15];      // Gaussian3D::gid
  if (gid <= 0) return;         // codelets.cpp:456-458
  // codelets.cpp:460-461
  const V4 clip = m4_mul_v4(c.mvp, V4{mean[0], mean[1], mean[2], mean[3]});
  // Viewport::clipSpaceToViewport (viewport.hpp:21-35), viewport (0,0,W,H)
  float vx = clip.x, vy = clip.y;
  const float s = 0.5f / clip.w;
  vx = vx * s; vy = vy * s;
  vx = vx + 0.5f; vy = vy + 0.5f;
  vx = vx * c.W; vy = vy * c.H;
  vx = vx + 0.0f; vy = vy + 0.0f;
  o->mean2d[0] = vx; o->mean2d[1] = vy;
  o->clip_z = clip.z;
  // codelets.cpp:463: g.scale = g.scale / fxy[1]
  const float sc[3] = {scale[0] / scale_div, scale[1] / scale_div, scale[2] / scale_div};
  compute_cov2d(c.mvp, mean, rot, sc, c.tanfov, c.focal_x, c.focal_y, o->cov2d);
  const float a = o->cov2d[0], b = o->cov2d[1], cc = o->cov2d[2];
  // Gaussian2D::ComputeEigenvalues (ipu_geometry.hpp:247-261)
  const float det = a * cc - b * b;
  const float mid = 0.5f * (a + cc);
  const float l1 = mid + std::sqrt(smax(0.1f, mid * mid - det));
  const float l2 = mid - std::sqrt(smax(0.1f, mid * mid - det));
  // GetBoundingBox (ipu_geometry.hpp:263-276)
  const float radius = std::ceil(3.0f * std::sqrt(smax(l1, l2)));
  o->radius = radius;
  const float minx = vx - radius, miny = vy - radius;
  const float maxx = vx + radius, maxy = vy + radius;
  // withinGuardBand (codelets.cpp:470)
  const float dx = maxx - minx, dy = maxy - miny;
  const float blen = std::sqrt(dx * dx + dy * dy);
  const bool within = blen < c.guard_thr;
  // ComputeConicOpacity (ipu_geometry.hpp:278-286)
  const float cdet = a * cc - b * b;
  if (cdet == 0.0f) {
    o->conic[0] = o->conic[1] = o->conic[2] = o->conic[3] = 0.0f;
  } else {
    const float inv = 1.0f / cdet;
    o->conic[0] = cc * inv;
    o->conic[1] = -b * inv;
    o->conic[2] = a * inv;
    o->conic[3] = colour[3];
  }
  // render iff withinGuardBand && z < 0 (codelets.cpp:493)
  o->rendered = (within && clip.z < 0.0f) ? 1 : 0;
  if (!o->rendered) return;
  // converged lattice semantics: tile rectangle of the
  // Bounds2f::clip beam (ipu_geometry.hpp:133-155, codelets.cpp:251-293)
  float fx0 = std::floor(std::floor(minx) / c.tw);
  float fx1 = std::floor(std::ceil(maxx) / c.tw);
  float fy0 = std::floor(std::floor(miny) / c.th);
  float fy1 = std::floor(std::ceil(maxy) / c.th);
  const float gx1 = (float)(c.tiles_x - 1);
  const float gy0 = (float)c.by0, gy1 = (float)(c.by1 - 1);
  if (fx0 < 0.0f) fx0 = 0.0f;
  if (fx1 > gx1) fx1 = gx1;
  if (fy0 < gy0) fy0 = gy0;
  if (fy1 > gy1) fy1 = gy1;
  if (fx0 <= fx1 && fy0 <= fy1) {
    o->rect[0] = (int32_t)fx0;
    o->rect[1] = (int32_t)fy0 - c.by0;
    o->rect[2] = (int32_t)fx1;
    o->rect[3] = (int32_t)fy1 - c.by0;
  }
}

int nthreads_or_default(int n) {
#ifdef _OPENMP
  return n > 0 ? n : omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}

inline float conv255(float v) {
  // cv::min(image_f * 255.0f, 255.0f) (ipu_rasteriser.cpp:139)
  float x = v * 255.0f;
  x = (255.0f < x) ? 255.0f : x;
  return x;
}

inline uint8_t sat_u8(float x) {
  // convertTo(CV_8UC4): cvRound (half-to-even) then saturate
  if (x != x) return 0;
  float r = std::nearbyint(x);
  if (r < 0.0f) return 0;
  if (r > 255.0f) return 255;
  return (uint8_t)r;
}

}  // namespace

extern "C" {

void or_mat4_mul(const float* a, const float* b, float* out) {
  M4 A, B;
  std::memcpy(A.m, a, 64);
  std::memcpy(B.m, b, 64);
  const M4 R = m4_mul(A, B);
  std::memcpy(out, R.m, 64);
}

void or_mat4_mul_vec4(const float* m, const float* v, float* out) {
  M4 A;
  std::memcpy(A.m, m, 64);
  const V4 r = m4_mul_v4(A, V4{v[0], v[1], v[2], v[3]});
  out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}

// Portable expf: Cody-Waite reduction + degree-6 polynomial (Cephes-style
// coefficients), every step an exactly specified IEEE op (fmaf is fused on
// both sides).  The reference calls libm expf/exp(float) (codelets.cpp:400,
// ipu_geometry.hpp:319-321) whose last bit is platform specific; this is the
// shared specification both the oracle and the HIP kernels implement.
float or_expf(float x) {
  float xc = (x != x) ? 0.0f : x;
  xc = (xc < -104.0f) ? -104.0f : xc;
  xc = (xc > 89.0f) ? 89.0f : xc;
  const float k = std::nearbyint(xc * 1.44269502162933349609f);
  float r = std::fma(k, -0.693145751953125f, xc);
  r = std::fma(k, -1.428606765330187045e-06f, r);
  float p = 1.9875691500e-4f;
  p = std::fma(p, r, 1.3981999507e-3f);
  p = std::fma(p, r, 8.3334519073e-3f);
  p = std::fma(p, r, 4.1665795894e-2f);
  p = std::fma(p, r, 1.6666665459e-1f);
  p = std::fma(p, r, 5.0000001201e-1f);
  const float r2 = r * r;
  p = std::fma(p, r2, r);
  p = p + 1.0f;
  int ki = (int)k;
  if (ki < -125) {
    p = p * 5.42101086242752217004e-20f;  // 2^-64
    ki += 64;
  }
  if (ki > 127) {
    p = p * 2.0f;
    ki -= 1;
  }
  uint32_t bits = (uint32_t)(ki + 127) << 23;
  float scale;
  std::memcpy(&scale, &bits, 4);
  float res = p * scale;
  if (x < -103.972084045410f) res = 0.0f;
  if (x > 88.72283935546875f) res = INFINITY;
  if (x != x) res = x;
  return res;
}

void or_frame_scalars(const or_frame* f, float* tanfov, float* focal_x, float* focal_y,
                      float* guard_thr) {
  // codelets.cpp:444-448: tanfov = tan(0.5 * fxy[0]) in double, stored as float;
  // focal = (width, height) / (2.f * glm::tan(fxy[0] / 2.f)) in float.
  *tanfov = (float)std::tan(0.5 * (double)f->fov);
  const float tf = std::tan(f->fov / 2.0f);
  *focal_x = (float)f->width / (2.0f * tf);
  *focal_y = (float)f->height / (2.0f * tf);
  // tb.diagonal().length() * clipSize (codelets.cpp:470); ivec2::length (ipu_geometry.hpp:52-54)
  const int gw = f->guard_tile_w > 0 ? f->guard_tile_w : f->tile_w;
  const int gh = f->guard_tile_h > 0 ? f->guard_tile_h : f->tile_h;
  const float tx = (float)gw, ty = (float)gh;
  *guard_thr = std::sqrt(tx * tx + ty * ty) * f->guard_band;
}

int or_project(const float* g64, int64_t n, const or_frame* f, or_proj* out, int nthreads) {
  const FrameC c = make_frame(f);
  const int nt = nthreads_or_default(nthreads);
#pragma omp parallel for schedule(static, 4096) num_threads(nt)
  for (int64_t i = 0; i < n; ++i) project_one(g64 + 16 * i, c, f->scale_div, &out[i]);
  return 0;
}

int64_t or_bin(const or_proj* p, int64_t n, const or_frame* f, int64_t* tile_start,
               uint32_t* list, int64_t cap, int nthreads) {
  const FrameC c = make_frame(f);
  const int T = c.tiles_x * (c.by1 - c.by0);
  std::vector<int64_t> cnt(T + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    const or_proj& q = p[i];
    if (!q.rendered || q.rect[0] > q.rect[2]) continue;
    for (int ty = q.rect[1]; ty <= q.rect[3]; ++ty)
      for (int tx = q.rect[0]; tx <= q.rect[2]; ++tx) cnt[ty * c.tiles_x + tx]++;
  }
  tile_start[0] = 0;
  for (int t = 0; t < T; ++t) tile_start[t + 1] = tile_start[t] + cnt[t];
  const int64_t P = tile_start[T];
  if (P > cap) return -1;
  std::vector<int64_t> cur(tile_start, tile_start + T);
  // index order: a stable depth sort then breaks z ties by index
  for (int64_t i = 0; i < n; ++i) {
    const or_proj& q = p[i];
    if (!q.rendered || q.rect[0] > q.rect[2]) continue;
    for (int ty = q.rect[1]; ty <= q.rect[3]; ++ty)
      for (int tx = q.rect[0]; tx <= q.rect[2]; ++tx) list[cur[ty * c.tiles_x + tx]++] = (uint32_t)i;
  }
  const int nt = nthreads_or_default(nthreads);
  // per-tile depth sort, clip z ascending (codelets.cpp:295-356; stable order
  // instead of the reference's unstable off-by-one quicksort)
#pragma omp parallel for schedule(dynamic, 16) num_threads(nt)
  for (int t = 0; t < T; ++t) {
    std::stable_sort(list + tile_start[t], list + tile_start[t + 1],
                     [p](uint32_t a, uint32_t b) { return p[a].clip_z < p[b].clip_z; });
  }
  return P;
}

int or_blend(const float* g64, const or_proj* p, const or_frame* f, const int64_t* tile_start,
             const uint32_t* list, float* rgba, int nthreads) {
  const FrameC c = make_frame(f);
  const int bands_rows = c.by1 - c.by0;
  const int T = c.tiles_x * bands_rows;
  const int py0 = c.by0 * f->tile_h;
  const int nt = nthreads_or_default(nthreads);
#pragma omp parallel for schedule(dynamic, 4) num_threads(nt)
  for (int t = 0; t < T; ++t) {
    const int tx = t % c.tiles_x;
    const int ty = t / c.tiles_x + c.by0;
    const int64_t s = tile_start[t], e = tile_start[t + 1];
    const int x0 = tx * f->tile_w, y0 = ty * f->tile_h;
    // renderTile (codelets.cpp:362-420), pixels clipped to the image
    for (int y = y0; y < y0 + f->tile_h && y < f->height; ++y) {
      for (int x = x0; x < x0 + f->tile_w && x < f->width; ++x) {
        const float pfx = (float)x, pfy = (float)y;
        float T_ = 1.0f;
        float C[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int64_t k = s; k < e; ++k) {
          const uint32_t gi = list[k];
          const or_proj& q = p[gi];
          const float* col = g64 + 16 * (int64_t)gi + 4;  // gCont = g.colour
          const float* con = q.conic;
          if (con[3] == 0.0f) continue;
          const float dx = q.mean2d[0] - pfx;
          const float dy = q.mean2d[1] - pfy;
          const float power = -0.5f * (con[0] * dx * dx + con[2] * dy * dy) - con[1] * dx * dy;
          if (power > 0.0f) continue;
          const float v = con[3] * or_expf(power);
          const float alpha = (v < 0.99f) ? v : 0.99f;  // glm::min(0.99f, v)
          if (alpha < 1.0f / 255.0f) continue;
          const float test_T = T_ * (1.0f - alpha);
          if (test_T < 0.0001f) break;
          // colour += gCont * alpha * T
          C[0] = C[0] + (col[0] * alpha) * T_;
          C[1] = C[1] + (col[1] * alpha) * T_;
          C[2] = C[2] + (col[2] * alpha) * T_;
          C[3] = C[3] + (col[3] * alpha) * T_;
          T_ = test_T;
        }
        float* o = rgba + 4 * ((int64_t)(y - py0) * f->width + x);
        // setPixel adds into the zeroed tile framebuffer (codelets.cpp:178-188,610)
        o[0] = 0.0f + C[0];
        o[1] = 0.0f + C[1];
        o[2] = 0.0f + C[2];
        o[3] = 0.0f + C[3];
      }
    }
  }
  return 0;
}

void or_pack_bgr8(const float* rgba, int64_t n_pixels, uint8_t* bgr) {
  for (int64_t i = 0; i < n_pixels; ++i) {
    const float* s = rgba + 4 * i;
    uint8_t* d = bgr + 3 * i;
    d[0] = sat_u8(conv255(s[2]));  // RGBA2BGR
    d[1] = sat_u8(conv255(s[1]));
    d[2] = sat_u8(conv255(s[0]));
  }
}

int or_render(const float* g64, int64_t n, const or_frame* f, float* rgba, uint8_t* bgr,
              uint32_t* hist, or_stats* st, int nthreads) {
  const FrameC c = make_frame(f);
  const int T = c.tiles_x * (c.by1 - c.by0);
  std::vector<or_proj> p((size_t)n);
  or_project(g64, n, f, p.data(), nthreads);
  int64_t P = 0;
  for (int64_t i = 0; i < n; ++i) {
    const or_proj& q = p[i];
    if (q.rendered && q.rect[0] <= q.rect[2])
      P += (int64_t)(q.rect[2] - q.rect[0] + 1) * (q.rect[3] - q.rect[1] + 1);
  }
  std::vector<int64_t> ts(T + 1);
  std::vector<uint32_t> list((size_t)(P > 0 ? P : 1));
  if (or_bin(p.data(), n, f, ts.data(), list.data(), P, nthreads) < 0) return -1;
  const int rows = std::min(c.by1 * f->tile_h, f->height) - c.by0 * f->tile_h;
  const int64_t npx = (int64_t)rows * f->width;
  std::vector<float> tmp;
  float* out = rgba;
  if (!out) {
    tmp.resize((size_t)npx * 4);
    out = tmp.data();
  }
  or_blend(g64, p.data(), f, ts.data(), list.data(), out, nthreads);
  if (bgr) or_pack_bgr8(out, npx, bgr);
  int64_t maxl = 0;
  for (int t = 0; t < T; ++t) {
    const int64_t l = ts[t + 1] - ts[t];
    if (hist) hist[t] = (uint32_t)l;
    maxl = std::max(maxl, l);
  }
  if (st) {
    int64_t v = 0;
    for (int64_t i = 0; i < n; ++i) v += p[i].rendered;
    st->n_rendered = v;
    st->n_pairs = P;
    st->max_list = maxl;
    st->n_tiles = T;
    st->tiles_x = c.tiles_x;
    st->tiles_y = c.by1 - c.by0;
  }
  return 0;
}

uint32_t or_point_splat(const float* xyz, int64_t n, const float* view_rm, const float* proj_rm,
                        int32_t width, int32_t height, int32_t tile_w, int32_t tile_h,
                        uint8_t* image, uint32_t* hist, int nthreads) {
  // projectPoints + splatPoints + buildTileHistogram (cpu_rasteriser.cpp:9-92).
  // The reference's unsynchronised image += colour (cpu_rasteriser.cpp:55) is
  // restated as an atomic count followed by a saturating add of 25 per hit.
  const M4 mvp = m4_mul(m4_from_rowmajor(proj_rm), m4_from_rowmajor(view_rm));
  const int nt = nthreads_or_default(nthreads);
  std::vector<std::atomic<uint32_t>> hits((size_t)width * height);
  for (auto& h : hits) h.store(0, std::memory_order_relaxed);
  const int nta = width / tile_w;  // uint16 integer division (tile_config.hpp:38)
  if (hist) std::memset(hist, 0, sizeof(uint32_t) * (size_t)nta * (height / tile_h));
  std::atomic<uint32_t> count{0};
  std::vector<V4> clip((size_t)n);
#pragma omp parallel for schedule(static, 128) num_threads(nt)
  for (int64_t i = 0; i < n; ++i) {
    const V4 cs = m4_mul_v4(mvp, V4{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 1.0f});
    clip[i] = cs;
    float vx = cs.x, vy = cs.y;
    const float s = 0.5f / cs.w;
    vx = vx * s; vy = vy * s;
    vx = (vx + 0.5f) * (float)width + 0.0f;
    vy = (vy + 0.5f) * (float)height + 0.0f;
    auto to_u32 = [](float v) -> uint32_t {
      if (!(std::fabs(v) < 9.2e18f)) return 0u;
      return (uint32_t)(int64_t)v;
    };
    const uint32_t r = to_u32(vy), cc = to_u32(vx);
    if (r < (uint32_t)height && cc < (uint32_t)width) {
      hits[(size_t)r * width + cc].fetch_add(1, std::memory_order_relaxed);
      count.fetch_add(1, std::memory_order_relaxed);
      if (hist) {
        // fb.pixCoordToTile(r, c) (tile_config.hpp:43-54)
        const float tr = std::floor(std::nearbyint((float)r) / (float)tile_h);
        const float tc = std::floor(std::nearbyint((float)cc) / (float)tile_w);
        const int64_t tid = (int64_t)(tr * (float)nta + tc);
        if (tid >= 0 && tid < (int64_t)nta * (height / tile_h))
          __atomic_fetch_add(&hist[tid], 1u, __ATOMIC_RELAXED);
      }
    }
  }
#pragma omp parallel for schedule(static) num_threads(nt)
  for (int64_t px = 0; px < (int64_t)width * height; ++px) {
    const uint32_t h = hits[px].load(std::memory_order_relaxed);
    if (!h) continue;
    for (int ch = 0; ch < 3; ++ch) {
      uint32_t v = image[3 * px + ch] + 25u * h;
      image[3 * px + ch] = (uint8_t)(v > 255u ? 255u : v);
    }
  }
  return count.load();
}

}  // extern "C"

// ======================================================================= lattice
// the reference's multi-frame migration of the Gaussians over
// the 4-neighbour channel lattice, restated frame by frame: the GSplat codelet
// of every IPU tile (codelets.cpp:143-641: compute :605-639, readInput
// :507-586, renderInternal :437-505, renderTile :358-421, the quicksort
// :295-356), the initial distribution of the records over the tiles
// (ipu_rasteriser.cpp:164-214, 287-386) and the exchange of the out-channels
// into the neighbours' in-channels (edge_builder.cpp:15-84).  The choices
// where the reference reads memory it never wrote or converts out of range are
// listed in gs_oracle.h (or_lattice_create).
namespace {

enum LDir { kLeft = 0, kRight = 1, kUp = 2, kDown = 3, kNone = 4 };  // ipu_geometry.hpp:94-100
// channel: EdgeBuilder::addEdge allocates channelSize / 4 floats
// (edge_builder.cpp:18) with channelSize = 300 * 64 (ipu_rasteriser.cpp:
// 307-308); insert() walks it in 64-float slots: 75 records
constexpr int kChan = 75;
// extraStorageSize = 2 * channelSize floats of vertsIn (ipu_rasteriser.cpp:309,361-363)
constexpr int kExtra = 600;

struct LG3 { float f[16]; };  // Gaussian3D at the head of a 64-float slot (ipu_geometry.hpp:305-311)
struct LG2 { float colour[4]; float cov[3]; float mean[2]; float z; };  // Gaussian2D (:232-236)
struct LB { float x0, y0, x1, y1; };                                     // Bounds2f
struct LDirs { bool up, right, down, left; };

struct Lat {
  int W, H, tw, th, tx, ty, T;
  float across;  // TiledFramebuffer::numTilesAcross, a float (tile_config.hpp:135)
  int64_t n, gpt, rem;
  std::vector<LG3> vs;       // every tile's vertsIn slots
  std::vector<LG3> chan[2];  // out-channels [parity][tile][direction][slot]
  std::vector<LG2> zb;       // every tile's gaus2D z-buffer (persistent)
  std::vector<uint32_t> splatted;
  std::vector<float> rgba;   // row-major W x H
  uint64_t frames = 0, dropped = 0, send_failed = 0, overrun = 0;
  int64_t base(int t) const { return (int64_t)t * (gpt + kExtra); }
  int vs_n(int t) const { return (int)(gpt + kExtra + (t == T - 1 ? rem : 0)); }
  int z_n(int t) const { return t == T - 1 ? (int)(gpt + rem) : (int)(gpt + kExtra); }
};

// float -> unsigned of a negative / NaN / huge value is undefined in C++ (the
// reference does it for tiles above the first row and means left of or above
// the image); the emulator saturates
uint32_t lat_u32(float v) {
  if (!(v > 0.0f)) return 0u;
  if (v >= 4294967296.0f) return 0xFFFFFFFFu;
  return (uint32_t)v;
}

// TiledFramebuffer::getTileBounds (tile_config.hpp:57-71): float arithmetic
LB lat_bounds(const Lat& L, uint32_t tid) {
  const float div = std::floor((float)tid / L.across);
  const float mod = (float)tid - div * L.across;
  LB b;
  b.x0 = std::floor(mod * (float)L.tw);
  b.y0 = std::floor(div * (float)L.th);
  b.x1 = b.x0 + (float)L.tw;
  b.y1 = b.y0 + (float)L.th;
  return b;
}

// Bounds2f::centroid (ipu_geometry.hpp:109-111)
void lat_centroid(const LB& b, float& cx, float& cy) {
  cx = (b.x1 + b.x0) * 0.5f;
  cy = (b.y1 + b.y0) * 0.5f;
}

// TiledFramebuffer::getNearbyTile (tile_config.hpp:73-86): unsigned wrap for
// left / right, float arithmetic for up / down
uint32_t lat_nearby(const Lat& L, uint32_t tid, int from) {
  switch (from) {
    case kLeft: return tid - 1u;
    case kRight: return tid + 1u;
    case kUp: return lat_u32((float)tid - L.across);
    case kDown: return lat_u32((float)tid + L.across);
  }
  return tid;
}

// Bounds2f::contains (ipu_geometry.hpp:163-165)
bool lat_contains(const LB& b, float x, float y) {
  return std::ceil(x) >= b.x0 && std::floor(x) < b.x1 && std::ceil(y) >= b.y0 && std::floor(y) < b.y1;
}

// TiledFramebuffer::pixCoordToTile (tile_config.hpp:43-54)
float lat_pix_to_tile(const Lat& L, float row, float col) {
  const float r = std::nearbyint(row), c = std::nearbyint(col);
  const float tc = std::floor(c / (float)L.tw);
  const float tr = std::floor(r / (float)L.th);
  return tr * L.across + tc;
}

// manhattanDistance (tile_config.hpp:88-90) as float |.| (the centroids of even
// tile sizes are integers, where an int abs() would agree)
float lat_manhattan(float ax, float ay, float bx, float by) { return std::fabs(ax - bx) + std::fabs(ay - by); }

// getBestDirection (tile_config.hpp:92-110): y first
int lat_best_dir(float sx, float sy, float dx, float dy) {
  if (lat_manhattan(sx, sy, dx, dy) == 0.0f) return kNone;
  if (sy < dy) return kDown;
  if (sy > dy) return kUp;
  if (sx < dx) return kRight;
  if (sx > dx) return kLeft;
  return kNone;
}

// Bounds2f::clip's direction flags (ipu_geometry.hpp:133-139)
LDirs lat_clip(const LB& bb, const LB& tb) {
  LDirs d;
  d.left = std::floor(bb.x0) < tb.x0;
  d.up = std::floor(bb.y0) < tb.y0;
  d.right = std::ceil(bb.x1) >= tb.x1;
  d.down = std::ceil(bb.y1) >= tb.y1;
  return d;
}

// EdgeBuilder::constructLattice (edge_builder.cpp:35-84): the out-channel the
// exchange copies into in-channel `from` of tile t -- the neighbour's opposite
// out-channel, or the tile's own one at the image border (self loop)
void lat_source(const Lat& L, int t, int from, int& st, int& sd) {
  const LB b = lat_bounds(L, (uint32_t)t);  // checkImageBoundaries (tile_config.hpp:116-126)
  const bool bl = b.x0 < 1.0f, bu = b.y0 < 1.0f;
  const bool br = b.x1 > (float)(L.W - 1), bd = b.y1 > (float)(L.H - 1);
  st = t;
  sd = from;
  switch (from) {
    case kRight: if (!br) { st = t + 1; sd = kLeft; } break;
    case kLeft: if (!bl) { st = t - 1; sd = kRight; } break;
    case kUp: if (!bu) { st = t - L.tx; sd = kDown; } break;
    case kDown: if (!bd) { st = t + L.tx; sd = kUp; } break;
  }
}

// insert (codelets.cpp:41-59): a slot with the same gid -> done; else the first
// empty slot (gid == 0); false when there is none
bool lat_insert(LG3* buf, int n, const LG3& g) {
  int idx = n;
  for (int i = 0; i < n; ++i) {
    const float gid = buf[i].f[15];
    if (gid == g.f[15]) return true;
    if (gid == 0.0f && i < idx) idx = i;
  }
  if (idx >= n) return false;
  buf[idx] = g;
  return true;
}

// iterativeQuickSort / partition (codelets.cpp:303-344) on entries [l, h]
// (Lomuto, pivot = last, `<=` to the left; an explicit stack of (l, h))
void lat_quicksort(LG2* e, int l, int h) {
  std::vector<int> st;
  st.push_back(l);
  st.push_back(h);
  while (!st.empty()) {
    h = st.back();
    st.pop_back();
    l = st.back();
    st.pop_back();
    const float pivot = e[h].z;
    int i = l - 1;
    for (int j = l; j <= h - 1; ++j)
      if (e[j].z <= pivot) {
        ++i;
        std::swap(e[i], e[j]);
      }
    std::swap(e[i + 1], e[h]);
    const int pi = i + 1;
    if (pi - 1 > l) {
      st.push_back(l);
      st.push_back(pi - 1);
    }
    if (pi + 1 < h) {
      st.push_back(pi + 1);
      st.push_back(h);
    }
  }
}

struct LP {
  float vx, vy, z, cov[3];
  LB bb;
  bool within;
};

// the per-record math both readInput and renderInternal do (codelets.cpp:
// 460-470, 537-551, 576-578): the same functions as the single-frame path
void lat_project(const LG3& g, const FrameC& c, float scale_div, LP& p) {
  or_proj o;
  project_one(g.f, c, scale_div, &o);
  p.vx = o.mean2d[0];
  p.vy = o.mean2d[1];
  p.z = o.clip_z;
  for (int k = 0; k < 3; ++k) p.cov[k] = o.cov2d[k];
  const float r = o.radius;
  p.bb = LB{p.vx - r, p.vy - r, p.vx + r, p.vy + r};
  const float dx = p.bb.x1 - p.bb.x0, dy = p.bb.y1 - p.bb.y0;
  p.within = std::sqrt(dx * dx + dy * dy) < c.guard_thr;
}

struct LCount {
  uint64_t dropped = 0, send_failed = 0, overrun = 0;
};

// GSplat::compute of tile t (codelets.cpp:605-639)
void lat_tile(Lat& L, const FrameC& c, float scale_div, int t, LCount& cnt) {
  const int par = (int)(L.frames & 1);
  LG3* out = &L.chan[par][(size_t)t * 4 * kChan];
  for (int k = 0; k < 4 * kChan; ++k) out[k].f[15] = 0.0f;  // clearOutBuffers (:588-602)
  const LB tb = lat_bounds(L, (uint32_t)t);
  float tcx, tcy;
  lat_centroid(tb, tcx, tcy);
  LG3* vs = &L.vs[L.base(t)];
  const int nvs = L.vs_n(t);
  // sendOnce (:214-225)
  auto send_once = [&](const LG3& g, int dir) -> bool {
    if (dir == kNone) return false;
    const bool ok = lat_insert(out + dir * kChan, kChan, g);
    if (!ok) cnt.send_failed++;
    return ok;
  };
  auto dest_centroid = [&](const LP& p, float& dx, float& dy) {
    lat_centroid(lat_bounds(L, lat_u32(lat_pix_to_tile(L, p.vy, p.vx))), dx, dy);
  };
  // readInput of the four in-channels (:507-586), in the order of :630-633
  const int order[4] = {kRight, kLeft, kUp, kDown};
  for (const int from : order) {
    int st, sd;
    lat_source(L, t, from, st, sd);
    const LG3* in = &L.chan[par ^ 1][((size_t)st * 4 + sd) * kChan];
    float pcx, pcy;
    lat_centroid(lat_bounds(L, lat_nearby(L, (uint32_t)t, from)), pcx, pcy);
    for (int k = 0; k < kChan; ++k) {
      const LG3 g = in[k];
      if (g.f[15] <= 0.0f) continue;
      LP p;
      lat_project(g, c, scale_div, p);
      auto keep = [&]() {
        if (!lat_insert(vs, nvs, g)) cnt.dropped++;
      };
      if (lat_contains(tb, p.vx, p.vy)) {  // the anchor arrived
        keep();
        continue;
      }
      float dcx, dcy;
      dest_centroid(p, dcx, dcy);
      if (lat_manhattan(tcx, tcy, dcx, dcy) < lat_manhattan(pcx, pcy, dcx, dcy)) {  // in transit
        send_once(g, lat_best_dir(tcx, tcy, dcx, dcy));
        keep();
        continue;
      }
      if (p.within) {  // spreading away from the anchor: protocol (:251-293)
        const LDirs s = lat_clip(p.bb, tb);
        if (from == kRight && s.left) {
          bool ok = send_once(g, kLeft);
          if (s.down) ok = ok && send_once(g, kDown);
          if (s.up) ok = ok && send_once(g, kUp);
        } else if (from == kLeft && s.right) {
          bool ok = send_once(g, kRight);
          if (s.down) ok = ok && send_once(g, kDown);
          if (s.up) ok = ok && send_once(g, kUp);
        } else if (from == kUp && s.down) {
          send_once(g, kDown);
        } else if (from == kDown && s.up) {
          send_once(g, kUp);
        } else if (s.up || s.right || s.down || s.left) {
          bool ok = true;
          if (s.up && from != kUp) ok = ok && send_once(g, kUp);
          if (s.down && from != kDown) ok = ok && send_once(g, kDown);
        }
      }
      keep();
    }
  }
  // renderInternal (:437-505)
  LG2* zb = &L.zb[L.base(t)];
  const int nz = L.z_n(t);
  int to_render = 0;
  for (int i = 0; i < nvs; ++i) {
    const LG3 g = vs[i];
    if (g.f[15] <= 0.0f) continue;
    LP p;
    lat_project(g, c, scale_div, p);
    LDirs dirs{false, false, false, false};  // (uninitialised in the reference outside the guard band)
    if (p.within) dirs = lat_clip(p.bb, tb);
    if (lat_contains(tb, p.vx, p.vy)) {
      bool sent = true;  // send (:194-212)
      if (dirs.right) sent = sent && send_once(g, kRight);
      if (dirs.left) sent = sent && send_once(g, kLeft);
      if (dirs.up) sent = sent && send_once(g, kUp);
      if (dirs.down) sent = sent && send_once(g, kDown);
    } else {  // evict and send one hop toward the anchor tile
      float dcx, dcy;
      dest_centroid(p, dcx, dcy);
      const int dir = lat_best_dir(tcx, tcy, dcx, dcy);
      vs[i].f[15] = 0.0f;
      if (!send_once(g, dir)) vs[i] = g;  // guard against losing it
    }
    if (p.within && p.z < 0.0f) {
      if (to_render < nz) {
        LG2& e = zb[to_render];
        for (int k = 0; k < 4; ++k) e.colour[k] = g.f[4 + k];
        for (int k = 0; k < 3; ++k) e.cov[k] = p.cov[k];
        e.mean[0] = p.vx;
        e.mean[1] = p.vy;
        e.z = p.z;
      } else {
        cnt.overrun++;  // insertAt past the z-buffer fails (:33-39)
      }
      to_render++;
    }
  }
  // renderTile (:358-421): sortBuffer sorts [0, L] inclusive (the stale entry
  // L included, the largest z of the L + 1 dropped) unless L >= z_n - 1
  if (to_render >= 1 && to_render < nz - 1) lat_quicksort(zb, 0, to_render);
  for (int ly = 0; ly < L.th; ++ly) {
    for (int lx = 0; lx < L.tw; ++lx) {
      const float pfx = tb.x0 + (float)lx, pfy = tb.y0 + (float)ly;
      float T_ = 1.0f;
      float C[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      for (int gi = 0; gi < to_render; ++gi) {
        LG2 e;
        if (gi < nz) e = zb[gi];
        else std::memset(&e, 0, sizeof(e));  // past the z-buffer: read as empty
        // ComputeConicOpacity (ipu_geometry.hpp:278-286)
        const float det = e.cov[0] * e.cov[2] - e.cov[1] * e.cov[1];
        float k0 = 0.0f, k1 = 0.0f, k2 = 0.0f, op = 0.0f;
        if (!(det == 0.0f)) {
          const float inv = 1.0f / det;
          k0 = e.cov[2] * inv;
          k1 = -e.cov[1] * inv;
          k2 = e.cov[0] * inv;
          op = e.colour[3];
        }
        if (op == 0.0f) continue;
        const float dx = e.mean[0] - pfx, dy = e.mean[1] - pfy;
        const float power = -0.5f * (k0 * dx * dx + k2 * dy * dy) - k1 * dx * dy;
        if (power > 0.0f) continue;
        const float v = op * or_expf(power);
        const float alpha = (v < 0.99f) ? v : 0.99f;
        if (alpha < 1.0f / 255.0f) continue;
        const float test_T = T_ * (1.0f - alpha);
        if (test_T < 0.0001f) break;
        for (int k = 0; k < 4; ++k) C[k] = C[k] + (e.colour[k] * alpha) * T_;
        T_ = test_T;
      }
      float* o = &L.rgba[4 * ((size_t)(tb.y0 + (float)ly) * L.W + (size_t)(tb.x0 + (float)lx))];
      for (int k = 0; k < 4; ++k) o[k] = 0.0f + C[k];  // colourFb black, then setPixel
    }
  }
  if (to_render > 0) L.splatted[t] = (uint32_t)to_render;
}

}  // namespace

struct or_lattice : Lat {};

extern "C" {

or_lattice* or_lattice_create(const float* g64, int64_t n, const or_frame* f) {
  if (!g64 || !f || n < 1 || f->tile_w <= 0 || f->tile_h <= 0 || f->width % f->tile_w || f->height % f->tile_h)
    return nullptr;
  or_lattice* L = new or_lattice();
  L->W = f->width;
  L->H = f->height;
  L->tw = f->tile_w;
  L->th = f->tile_h;
  L->tx = f->width / f->tile_w;
  L->ty = f->height / f->tile_h;
  L->T = L->tx * L->ty;
  L->across = (float)L->tx;
  L->n = n;
  // calculateMapping (ipu_rasteriser.cpp:164-193) of the 64-float records:
  // grainsPerTile = ceil(64 n / (numTiles * 64)) in float, fullTiles = floor(n / gpt)
  const float q = (float)((uint64_t)n * 64u) / ((float)L->T * 64.0f);
  L->gpt = (int64_t)std::ceil(q);
  const int64_t full = n / L->gpt;
  L->rem = n - full * L->gpt;
  const size_t slots = (size_t)L->base(L->T - 1) + L->vs_n(L->T - 1);
  L->vs.assign(slots, LG3{});
  L->zb.assign(slots, LG2{});
  for (int p = 0; p < 2; ++p) L->chan[p].assign((size_t)L->T * 4 * kChan, LG3{});
  L->splatted.assign((size_t)L->T, 0u);
  L->rgba.assign((size_t)L->W * L->H * 4, 0.0f);
  // applyTileMapping (:199-214): record j on tile j / gpt
  for (int64_t j = 0; j < n; ++j) {
    const int64_t t = j / L->gpt;
    std::memcpy(L->vs[(size_t)(L->base((int)t) + (j - t * L->gpt))].f, g64 + 16 * j, 64);
  }
  return L;
}

int or_lattice_step(or_lattice* L, const or_frame* f, int nthreads) {
  if (!L || !f) return -1;
  const FrameC c = make_frame(f);
  const int nt = nthreads_or_default(nthreads);
  uint64_t d = 0, s = 0, o = 0;
#pragma omp parallel for schedule(dynamic, 8) num_threads(nt) reduction(+ : d, s, o)
  for (int t = 0; t < L->T; ++t) {
    LCount cnt;
    lat_tile(*L, c, f->scale_div, t, cnt);
    d += cnt.dropped;
    s += cnt.send_failed;
    o += cnt.overrun;
  }
  L->dropped = d;
  L->send_failed = s;
  L->overrun = o;
  L->frames++;  // the exchange: this frame's out-channels are the next one's in-channels
  return 0;
}

int64_t or_lattice_total_slots(const or_lattice* L) { return L ? (int64_t)L->vs.size() : 0; }

void or_lattice_read(const or_lattice* L, float* rgba, uint32_t* hist, float* slot_gids, uint64_t* counters) {
  if (!L) return;
  if (rgba) std::memcpy(rgba, L->rgba.data(), L->rgba.size() * 4);
  if (hist) std::memcpy(hist, L->splatted.data(), L->splatted.size() * 4);
  if (slot_gids)
    for (size_t i = 0; i < L->vs.size(); ++i) slot_gids[i] = L->vs[i].f[15];
  if (counters) {
    counters[0] = L->frames;
    counters[1] = L->dropped;
    counters[2] = L->send_failed;
    counters[3] = L->overrun;
    counters[4] = (uint64_t)L->gpt;
    counters[5] = (uint64_t)L->rem;
  }
}

void or_lattice_destroy(or_lattice* L) { delete L; }

}  // extern "C"

// OpenMP team placement probe (bench.py's CPU baseline records the cores its
// threads really ran on, not the calling thread's affinity mask)
int or_omp_team_cpus(int nthreads, int* cpus, int cap, double spin_ms) {
  const int nt = nthreads_or_default(nthreads);
  int team = 0;
#pragma omp parallel num_threads(nt)
  {
    const double t0 = omp_get_wtime();
    volatile double x = 0.0;
    while ((omp_get_wtime() - t0) * 1e3 < spin_ms) x = x + 1.0;
    const int id = omp_get_thread_num();
    if (id < cap) cpus[id] = sched_getcpu();
#pragma omp single
    team = omp_get_num_threads();
  }
  return team;
}

// Opt-in SH colour (3DGS convention, computeColorFromSH of the INRIA
// rasteriser restated; constants are its SH_C0..SH_C3).  Every operation in
// the order written; -ffp-contract=off.
void or_sh_colours(const float* g64, int64_t n, const float* f_dc, const float* f_rest, int degree,
                   const float campos[3], float* out_g64) {
  const float C0 = 0.28209479177387814f, C1 = 0.4886025119029199f;
  const float C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f, -1.0925484305920792f,
                       0.5462742152960396f};
  const float C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f, 0.3731763325901154f,
                       -0.4570457994644658f, 1.445305721320277f, -0.5900435899266435f};
  for (int64_t i = 0; i < n; ++i) {
    const float* g = g64 + i * 16;
    float* o = out_g64 + i * 16;
    for (int k = 0; k < 16; ++k) o[k] = g[k];
    const float dx = g[0] - campos[0], dy = g[1] - campos[1], dz = g[2] - campos[2];
    const float len = std::sqrt((dx * dx + dy * dy) + dz * dz);
    const float x = dx / len, y = dy / len, z = -dz / len;  // the PLY frame's z
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    for (int c = 0; c < 3; ++c) {
      const float* sh = f_rest ? f_rest + i * 45 + c * 15 - 1 : nullptr;  // sh[k], k = 1..15
      float r = C0 * f_dc[i * 3 + c];
      if (degree > 0) {
        r = r - C1 * y * sh[1] + C1 * z * sh[2] - C1 * x * sh[3];
        if (degree > 1) {
          r = r + C2[0] * xy * sh[4] + C2[1] * yz * sh[5] + C2[2] * (2.0f * zz - xx - yy) * sh[6] +
              C2[3] * xz * sh[7] + C2[4] * (xx - yy) * sh[8];
          if (degree > 2)
            r = r + C3[0] * y * (3.0f * xx - yy) * sh[9] + C3[1] * xy * z * sh[10] +
                C3[2] * y * (4.0f * zz - xx - yy) * sh[11] + C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[12] +
                C3[4] * x * (4.0f * zz - xx - yy) * sh[13] + C3[5] * z * (xx - yy) * sh[14] +
                C3[6] * x * (xx - 3.0f * yy) * sh[15];
        }
      }
      r = r + 0.5f;
      o[4 + c] = (r < 0.0f) ? 0.0f : r;  // glm::max(colour, vec3(0)) (splat.cpp:136-147)
    }
  }
}

void or_camera_position(const float* v, float* campos) {
  double a[3][3], t[3];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) a[i][j] = v[i * 4 + j];
    t[i] = v[i * 4 + 3];
  }
  // adjugate rows / determinant
  const double c00 = a[1][1] * a[2][2] - a[1][2] * a[2][1];
  const double c01 = a[1][2] * a[2][0] - a[1][0] * a[2][2];
  const double c02 = a[1][0] * a[2][1] - a[1][1] * a[2][0];
  const double det = (a[0][0] * c00 + a[0][1] * c01) + a[0][2] * c02;
  const double inv[3][3] = {
      {c00, a[0][2] * a[2][1] - a[0][1] * a[2][2], a[0][1] * a[1][2] - a[0][2] * a[1][1]},
      {c01, a[0][0] * a[2][2] - a[0][2] * a[2][0], a[0][2] * a[1][0] - a[0][0] * a[1][2]},
      {c02, a[0][1] * a[2][0] - a[0][0] * a[2][1], a[0][0] * a[1][1] - a[0][1] * a[1][0]}};
  for (int i = 0; i < 3; ++i) campos[i] = (float)(-((inv[i][0] * t[0] + inv[i][1] * t[1]) + inv[i][2] * t[2]) / det);
}
