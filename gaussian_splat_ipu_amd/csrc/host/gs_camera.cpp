// gs_camera.cpp -- camera / matrix helpers of the render server (host side).
//
// The reference builds its matrices with glm (external/glm, empty submodule in
// the reference snapshot).  These functions restate the glm 0.9.9 routines the
// reference calls, column-major m[c*4 + r]:
//   glm::lookAt        src/splat/camera.cpp:14, codelets/tests/codelets.cpp:53-69
//   glm::frustum       src/splat/geometry.cpp:23
//   glm::rotate/translate  src/main/splat.cpp:312-314
//   mat4*mat4, mat4*vec4   codelets.cpp:443,460; tests/test.cpp:21-34
// Pinned by the reference's known-answer tests (tests/test_camera_kat.py).
#include <cmath>
#include <cstring>

#include "../../../include/gsplat.h"
#include "gs_host.hpp"

namespace gsh {

void mat4_mul(const float* a, const float* b, float* out) {
  // glm: Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3]
  float r[16];
  for (int c = 0; c < 4; ++c)
    for (int row = 0; row < 4; ++row) {
      float s = a[0 * 4 + row] * b[c * 4 + 0];
      s = s + a[1 * 4 + row] * b[c * 4 + 1];
      s = s + a[2 * 4 + row] * b[c * 4 + 2];
      s = s + a[3 * 4 + row] * b[c * 4 + 3];
      r[c * 4 + row] = s;
    }
  std::memcpy(out, r, sizeof(r));
}

void mat4_mul_vec4(const float* m, const float* v, float* out) {
  // glm: (m0*x + m1*y) + (m2*z + m3*w)
  float r[4];
  for (int row = 0; row < 4; ++row) {
    const float p = m[0 * 4 + row] * v[0] + m[1 * 4 + row] * v[1];
    const float q = m[2 * 4 + row] * v[2] + m[3 * 4 + row] * v[3];
    r[row] = p + q;
  }
  std::memcpy(out, r, sizeof(r));
}

void mat4_transpose(const float* m, float* out) {
  float r[16];
  for (int c = 0; c < 4; ++c)
    for (int row = 0; row < 4; ++row) r[c * 4 + row] = m[row * 4 + c];
  std::memcpy(out, r, sizeof(r));
}

static float dot3(const float* a, const float* b) {
  // glm compute_dot<vec3>: tmp = a*b; (tmp.x + tmp.y) + tmp.z
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}

static void normalize3(const float* v, float* out) {
  // glm::normalize(vec3) = v * inversesqrt(dot(v, v)); inversesqrt = 1 / sqrt(x)
  const float inv = 1.0f / std::sqrt(dot3(v, v));
  out[0] = v[0] * inv;
  out[1] = v[1] * inv;
  out[2] = v[2] * inv;
}

static void cross3(const float* x, const float* y, float* out) {
  const float r0 = x[1] * y[2] - y[1] * x[2];
  const float r1 = x[2] * y[0] - y[2] * x[0];
  const float r2 = x[0] * y[1] - y[0] * x[1];
  out[0] = r0; out[1] = r1; out[2] = r2;
}

static void identity(float* m) {
  std::memset(m, 0, 16 * sizeof(float));
  m[0] = m[5] = m[10] = m[15] = 1.0f;
}

void look_at(const float* eye, const float* center, const float* up, float* out) {
  // glm::lookAtRH (GLM_FORCE_LEFT_HANDED not set)
  const float d[3] = {center[0] - eye[0], center[1] - eye[1], center[2] - eye[2]};
  float f[3], s[3], u[3], fs[3];
  normalize3(d, f);
  cross3(f, up, fs);
  normalize3(fs, s);
  cross3(s, f, u);
  float m[16];
  identity(m);
  m[0 * 4 + 0] = s[0];
  m[1 * 4 + 0] = s[1];
  m[2 * 4 + 0] = s[2];
  m[0 * 4 + 1] = u[0];
  m[1 * 4 + 1] = u[1];
  m[2 * 4 + 1] = u[2];
  m[0 * 4 + 2] = -f[0];
  m[1 * 4 + 2] = -f[1];
  m[2 * 4 + 2] = -f[2];
  m[3 * 4 + 0] = -dot3(s, eye);
  m[3 * 4 + 1] = -dot3(u, eye);
  m[3 * 4 + 2] = dot3(f, eye);
  std::memcpy(out, m, sizeof(m));
}

void frustum(float l, float r, float b, float t, float n, float f, float* out) {
  // glm::frustumRH_NO
  float m[16];
  std::memset(m, 0, sizeof(m));
  m[0 * 4 + 0] = (2.0f * n) / (r - l);
  m[1 * 4 + 1] = (2.0f * n) / (t - b);
  m[2 * 4 + 0] = (r + l) / (r - l);
  m[2 * 4 + 1] = (t + b) / (t - b);
  m[2 * 4 + 2] = -(f + n) / (f - n);
  m[2 * 4 + 3] = -1.0f;
  m[3 * 4 + 2] = -(2.0f * f * n) / (f - n);
  std::memcpy(out, m, sizeof(m));
}

static float length3(const float* v) { return std::sqrt(dot3(v, v)); }

void fit_frustum(const float* bb_min, const float* bb_max, float fov, float aspect, float* out) {
  // splat::fitFrustumToBoundingBox (src/splat/geometry.cpp:9-24)
  const float diag[3] = {bb_max[0] - bb_min[0], bb_max[1] - bb_min[1], bb_max[2] - bb_min[2]};
  const float radius = length3(diag) * 0.5f;
  const float near_plane = radius / std::tan(fov);
  const float far_plane = near_plane + 20.0f * radius;
  const float half_w = radius * aspect;
  const float half_h = radius;
  frustum(-half_w, half_w, -half_h, half_h, near_plane, far_plane, out);
}

void look_at_bbox(const float* bb_min, const float* bb_max, const float* up, float scale,
                  float* out) {
  // splat::lookAtBoundingBox (src/splat/camera.cpp:10-15)
  float centre[3], diag[3];
  for (int i = 0; i < 3; ++i) {
    centre[i] = (bb_max[i] + bb_min[i]) * 0.5f;  // Bounds3f::centroid
    diag[i] = bb_max[i] - bb_min[i];
  }
  const float radius = length3(diag) * 0.5f;
  const float eye[3] = {centre[0] - 0.0f, centre[1] - 0.0f, centre[2] - scale * radius};
  look_at(eye, centre, up, out);
}

void rotate(const float* m, float angle, const float* v, float* out) {
  // glm::rotate(mat4, angle, axis)
  const float c = std::cos(angle);
  const float s = std::sin(angle);
  float axis[3];
  normalize3(v, axis);
  const float temp[3] = {(1.0f - c) * axis[0], (1.0f - c) * axis[1], (1.0f - c) * axis[2]};
  float R[3][3];
  R[0][0] = c + temp[0] * axis[0];
  R[0][1] = temp[0] * axis[1] + s * axis[2];
  R[0][2] = temp[0] * axis[2] - s * axis[1];
  R[1][0] = temp[1] * axis[0] - s * axis[2];
  R[1][1] = c + temp[1] * axis[1];
  R[1][2] = temp[1] * axis[2] + s * axis[0];
  R[2][0] = temp[2] * axis[0] + s * axis[1];
  R[2][1] = temp[2] * axis[1] - s * axis[0];
  R[2][2] = c + temp[2] * axis[2];
  float r[16];
  for (int col = 0; col < 3; ++col)
    for (int row = 0; row < 4; ++row) {
      float acc = m[0 * 4 + row] * R[col][0];
      acc = acc + m[1 * 4 + row] * R[col][1];
      acc = acc + m[2 * 4 + row] * R[col][2];
      r[col * 4 + row] = acc;
    }
  for (int row = 0; row < 4; ++row) r[3 * 4 + row] = m[3 * 4 + row];
  std::memcpy(out, r, sizeof(r));
}

void translate(const float* m, const float* v, float* out) {
  // glm::translate: Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]
  float r[16];
  std::memcpy(r, m, sizeof(r));
  for (int row = 0; row < 4; ++row) {
    float acc = m[0 * 4 + row] * v[0];
    acc = acc + m[1 * 4 + row] * v[1];
    acc = acc + m[2 * 4 + row] * v[2];
    acc = acc + m[3 * 4 + row];
    r[3 * 4 + row] = acc;
  }
  std::memcpy(out, r, sizeof(r));
}

void mvp_start(float* out) {
  // splat.cpp:235-241
  identity(out);
  out[0 * 4 + 0] = -1.0f;
  out[1 * 4 + 1] = -0.09709989f;
  out[1 * 4 + 2] = -0.99527466f;
  out[2 * 4 + 1] = -0.99527466f;
  out[2 * 4 + 2] = 0.09709989f;
  out[3 * 4 + 2] = -5.1539507f;
}

void headless(const float* bb6, uint32_t width, uint32_t height, float fov, float* view_rm,
              float* proj_rm) {
  // splat.cpp:105-107: aspect = cols / (float)rows
  const float aspect = (float)width / (float)height;
  // splat.cpp:186: modelView = lookAtBoundingBox(bb, vec3(0, 1, 1), 1)
  const float up[3] = {0.0f, 1.0f, 1.0f};
  float mv[16];
  look_at_bbox(bb6, bb6 + 3, up, 1.0f, mv);
  // splat.cpp:189-192: bbInCamera(modelView * (bb.min, 1), modelView * (bb.max, 1))
  const float pmin[4] = {bb6[0], bb6[1], bb6[2], 1.0f};
  const float pmax[4] = {bb6[3], bb6[4], bb6[5], 1.0f};
  float cmin[4], cmax[4];
  mat4_mul_vec4(mv, pmin, cmin);
  mat4_mul_vec4(mv, pmax, cmax);
  float proj[16];
  fit_frustum(cmin, cmax, fov, aspect, proj);  // splat.cpp:195
  float view[16];
  mvp_start(view);  // splat.cpp:244: dynamicView = mvpStart
  // IpuSplatter::updateModelView/updateProjection store the transpose (row-major)
  mat4_transpose(view, view_rm);
  mat4_transpose(proj, proj_rm);
}

}  // namespace gsh

extern "C" {

int gs_mat4_mul(const float* a, const float* b, float* out) {
  if (!a || !b || !out) return GS_EINVAL;
  gsh::mat4_mul(a, b, out);
  return GS_OK;
}
int gs_mat4_mul_vec4(const float* m, const float* v, float* out) {
  if (!m || !v || !out) return GS_EINVAL;
  gsh::mat4_mul_vec4(m, v, out);
  return GS_OK;
}
int gs_mat4_transpose(const float* m, float* out) {
  if (!m || !out) return GS_EINVAL;
  gsh::mat4_transpose(m, out);
  return GS_OK;
}
int gs_cam_look_at(const float* eye, const float* center, const float* up, float* out) {
  if (!eye || !center || !up || !out) return GS_EINVAL;
  gsh::look_at(eye, center, up, out);
  return GS_OK;
}
int gs_cam_frustum(float l, float r, float b, float t, float n, float f, float* out) {
  if (!out) return GS_EINVAL;
  gsh::frustum(l, r, b, t, n, f, out);
  return GS_OK;
}
int gs_cam_fit_frustum(const float* bb_min, const float* bb_max, float fov, float aspect,
                       float* out) {
  if (!bb_min || !bb_max || !out) return GS_EINVAL;
  gsh::fit_frustum(bb_min, bb_max, fov, aspect, out);
  return GS_OK;
}
int gs_cam_look_at_bbox(const float* bb_min, const float* bb_max, const float* up, float scale,
                        float* out) {
  if (!bb_min || !bb_max || !up || !out) return GS_EINVAL;
  gsh::look_at_bbox(bb_min, bb_max, up, scale, out);
  return GS_OK;
}
int gs_cam_rotate(const float* m, float angle_rad, const float* axis, float* out) {
  if (!m || !axis || !out) return GS_EINVAL;
  gsh::rotate(m, angle_rad, axis, out);
  return GS_OK;
}
int gs_cam_translate(const float* m, const float* v, float* out) {
  if (!m || !v || !out) return GS_EINVAL;
  gsh::translate(m, v, out);
  return GS_OK;
}
int gs_cam_mvp_start(float* out) {
  if (!out) return GS_EINVAL;
  gsh::mvp_start(out);
  return GS_OK;
}
int gs_cam_headless(const float* bb6, uint32_t width, uint32_t height, float fov, float* view_rm,
                    float* proj_rm) {
  if (!bb6 || !view_rm || !proj_rm || width == 0 || height == 0) return GS_EINVAL;
  gsh::headless(bb6, width, height, fov, view_rm, proj_rm);
  return GS_OK;
}

}  // extern "C"
