// gs_host.hpp -- internal declarations of the host-side data path (PLY ingest,
// scene preparation, synthetic scenes, camera).  Not part of the C ABI.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/gsplat.h"

// Opaque PLY handle of the C ABI: the vertex element as named float columns
// (splat::Ply, include/splat/file_io.hpp:14-25, generalised to keep f_rest_*).
struct gs_ply {
  int64_t n = 0;
  std::vector<std::string> order;  // property order as in the file
  std::unordered_map<std::string, std::vector<float>> props;

  const std::vector<float>* get(const std::string& k) const {
    auto it = props.find(k);
    return it == props.end() ? nullptr : &it->second;
  }
  std::vector<float>& add(const std::string& k) {
    auto it = props.find(k);
    if (it != props.end()) return it->second;
    order.push_back(k);
    auto& v = props[k];
    v.resize((size_t)n);
    return v;
  }
};

namespace gsh {

void set_error(const std::string& msg);
const char* last_error();

void mat4_mul(const float* a, const float* b, float* out);
void mat4_mul_vec4(const float* m, const float* v, float* out);
void mat4_transpose(const float* m, float* out);
void look_at(const float* eye, const float* center, const float* up, float* out);
void frustum(float l, float r, float b, float t, float n, float f, float* out);
void fit_frustum(const float* bb_min, const float* bb_max, float fov, float aspect, float* out);
void look_at_bbox(const float* bb_min, const float* bb_max, const float* up, float scale,
                  float* out);
void rotate(const float* m, float angle, const float* v, float* out);
void translate(const float* m, const float* v, float* out);
void mvp_start(float* out);
void headless(const float* bb6, uint32_t width, uint32_t height, float fov, float* view_rm,
              float* proj_rm);

}  // namespace gsh
