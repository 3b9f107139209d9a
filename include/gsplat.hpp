// gsplat.hpp -- header-only C++ mirror of splat::IpuSplatter over the C ABI.
//
// Drop-in for include/splat/ipu_rasteriser.hpp:20-55 in Nmjfry/gaussian_splat_ipu:
// the same member names and argument meaning, C++ exceptions on failure (the
// reference throws std::runtime_error), no Poplar / GraphManager.  Matrices are
// passed as 16 floats in glm's column-major storage (glm::value_ptr(m)); the
// class transposes them to the row-major wire format exactly as
// IpuSplatter::updateModelView/updateProjection do (ipu_rasteriser.cpp:86-102).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "gsplat.h"

namespace splat {

struct GsError : std::runtime_error {
  int status;
  GsError(int s, const std::string& what) : std::runtime_error(what), status(s) {}
};

inline void gs_check(int rc, const char* what) {
  if (rc != GS_OK) throw GsError(rc, std::string(what) + ": " + gs_last_error());
}

// Framebuffer geometry (TiledFramebuffer(w, h, tw, th); the build uses a ceil
// tile grid).
struct GpuFramebuffer {
  uint32_t width = 1280, height = 720, tileWidth = 32, tileHeight = 20;
};

class GpuSplatter {
 public:
  // IpuSplatter(const Gaussians&, TiledFramebuffer&, bool noAMP)
  GpuSplatter(const std::vector<gs_gaussian3d>& gaussians, const GpuFramebuffer& fb,
              int device = -1, uint32_t bandIndex = 0, uint32_t bandCount = 1,
              uint32_t flags = 0 /* GS_FLAG_* */)
      : fb_(fb) {
    gs_config cfg;
    gs_check(gs_config_init(&cfg), "gs_config_init");
    cfg.width = fb.width;
    cfg.height = fb.height;
    cfg.tile_width = fb.tileWidth;
    cfg.tile_height = fb.tileHeight;
    cfg.device = device;
    cfg.band_index = bandIndex;
    cfg.band_count = bandCount;
    cfg.flags = flags;
    gs_check(gs_create(gaussians.data(), gaussians.size(), &cfg, &r_), "gs_create");
  }
  ~GpuSplatter() { gs_destroy(r_); }
  GpuSplatter(const GpuSplatter&) = delete;
  GpuSplatter& operator=(const GpuSplatter&) = delete;

  // updateModelView(const glm::mat4&): pass glm::value_ptr(mv)
  void updateModelView(const float* colMajor16) {
    float rm[16];
    gs_check(gs_mat4_transpose(colMajor16, rm), "transpose");
    gs_check(gs_set_view(r_, rm), "gs_set_view");
  }
  void updateProjection(const float* colMajor16) {
    float rm[16];
    gs_check(gs_mat4_transpose(colMajor16, rm), "transpose");
    gs_check(gs_set_projection(r_, rm), "gs_set_projection");
  }
  // updateFocalLengths(fov, lambda1 / 10)
  void updateFocalLengths(float fx, float fy) { gs_check(gs_set_focal(r_, fx, fy), "gs_set_focal"); }

  // GraphManager::execute(splatter): one blocking frame
  void execute() { gs_check(gs_render(r_), "gs_render"); }

  // frames in flight (no reference counterpart): enqueue on the renderer's
  // stream / wait for it; the stream (a hipStream_t) for ordering caller work
  void executeAsync() { gs_check(gs_render_async(r_), "gs_render_async"); }
  void sync() { gs_check(gs_sync(r_), "gs_sync"); }
  void* stream() {
    void* s = nullptr;
    gs_check(gs_get_stream(r_, &s), "gs_get_stream");
    return s;
  }
  // later frames write their padded BGR8 band at dst (device memory; nullptr:
  // the renderer's own buffer), e.g. a slot of an all-gather buffer
  void setBgr8Target(void* dst, size_t bytes) {
    gs_check(gs_set_bgr8_target(r_, dst, bytes), "gs_set_bgr8_target");
  }

  // getFrameBuffer(cv::Mat&): band rows x width x 3, 8-bit BGR, row-major
  void getFrameBuffer(std::vector<uint8_t>& bgr) {
    const gs_frame_stats st = stats();
    bgr.resize((size_t)st.band_rows * fb_.width * 3);
    gs_check(gs_read_bgr8(r_, bgr.data(), bgr.size()), "gs_read_bgr8");
  }
  // getIPUHistogram(std::vector<u32>&): thread-safe snapshot
  void getIPUHistogram(std::vector<uint32_t>& counts) {
    counts.resize(stats().n_tiles);
    gs_check(gs_read_tile_histogram(r_, counts.data(), counts.size()), "gs_read_tile_histogram");
  }

  gs_frame_stats stats() {
    gs_frame_stats st;
    gs_check(gs_get_stats(r_, &st), "gs_get_stats");
    return st;
  }
  const GpuFramebuffer& framebuffer() const { return fb_; }
  gs_renderer* handle() { return r_; }

 private:
  GpuFramebuffer fb_;
  gs_renderer* r_ = nullptr;
};

}  // namespace splat
