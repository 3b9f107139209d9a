// gs_points.cpp -- the render server's `--device cpu` path:
// the reference's CPU point splatter, projectPoints + splatPoints +
// buildTileHistogram (src/splat/cpu_rasteriser.cpp:9-92).  It is a separate
// device of the render server (splat.cpp:250-256), not a fallback of the
// Gaussian frame path: gs_render has no CPU path.
//
// Semantics kept from the reference:
// - mvp = projection * modelView, clip = mvp * (p, 1) with glm's order of
//   operations (cpu_rasteriser.cpp:12,16);
// - window = clipSpaceToViewport(clip) (viewport.hpp:21-26); r = (u32)y,
//   c = (u32)x (cpu_rasteriser.cpp:50-51); a point inside the image adds
//   `value` (25) to its pixel's three channels, saturating like cv::Vec3b +=
//   (:55), and counts as splatted (:57-58);
// - the histogram counts the points per tile of TiledFramebuffer(tw, th):
//   pixCoordToTile(r, c) = floor(nearbyint(r) / th) * (W / tw) +
//   floor(nearbyint(c) / tw), W / tw an integer division
//   (tile_config.hpp:38-54, cpu_rasteriser.cpp:80-90).
// Deviations: the reference's image += from 32 threads is unsynchronised
// (a race); here hits are counted atomically and added once.  The
// float -> u32 conversion of an out-of-range coordinate (undefined in C++) is
// pinned: |v| >= 9.2e18 or NaN -> 0, else (u32)(i64)v (x86's wrap-around).
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "gs_host.hpp"

namespace {

uint32_t to_u32(float v) {
  if (!(std::fabs(v) < 9.2e18f)) return 0u;
  return (uint32_t)(int64_t)v;
}

template <typename F>
void parallel_for(int64_t n, int nthreads, F&& f) {
  if (nthreads <= 1 || n < 4096) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const int64_t chunk = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int64_t a = t * chunk, b = std::min<int64_t>(n, a + chunk);
    if (a >= b) break;
    ts.emplace_back([&f, a, b] { f(a, b); });
  }
  for (auto& t : ts) t.join();
}

}  // namespace

extern "C" int gs_cpu_point_splat(const float* xyz, size_t n, const float* view_rm, const float* proj_rm,
                                  uint32_t width, uint32_t height, uint32_t tile_w, uint32_t tile_h,
                                  uint8_t value, uint8_t* bgr, uint32_t* tile_hist, uint32_t* splatted,
                                  int nthreads) {
  if ((n && !xyz) || !view_rm || !proj_rm || !bgr || width == 0 || height == 0 || tile_w == 0 ||
      tile_h == 0) {
    gsh::set_error("gs_cpu_point_splat: invalid argument");
    return GS_EINVAL;
  }
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  float view[16], proj[16], mvp[16];
  gsh::mat4_transpose(view_rm, view);
  gsh::mat4_transpose(proj_rm, proj);
  gsh::mat4_mul(proj, view, mvp);  // cpu_rasteriser.cpp:12
  const uint32_t nta = width / tile_w, ntd = height / tile_h;  // tile_config.hpp:38-39
  if (tile_hist) std::memset(tile_hist, 0, sizeof(uint32_t) * (size_t)nta * ntd);
  std::vector<uint32_t> hits((size_t)width * height, 0u);
  std::atomic<uint64_t> count{0};
  const float W = (float)width, H = (float)height;
  parallel_for((int64_t)n, nthreads, [&](int64_t a, int64_t b) {
    uint64_t local = 0;
    for (int64_t i = a; i < b; ++i) {
      const float p[4] = {xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 1.0f};
      float c[4];
      gsh::mat4_mul_vec4(mvp, p, c);
      // Viewport::clipSpaceToViewport (viewport.hpp:21-26), viewport (0, 0, W, H)
      const float s = 0.5f / c[3];
      float vx = c[0] * s, vy = c[1] * s;
      vx = (vx + 0.5f) * W + 0.0f;
      vy = (vy + 0.5f) * H + 0.0f;
      const uint32_t r = to_u32(vy), cc = to_u32(vx);
      if (r < height && cc < width) {
        __atomic_fetch_add(&hits[(size_t)r * width + cc], 1u, __ATOMIC_RELAXED);
        ++local;
        if (tile_hist) {
          const float tr = std::floor(std::nearbyint((float)r) / (float)tile_h);
          const float tc = std::floor(std::nearbyint((float)cc) / (float)tile_w);
          const int64_t tid = (int64_t)(tr * (float)nta + tc);
          if (tid >= 0 && tid < (int64_t)nta * ntd) __atomic_fetch_add(&tile_hist[tid], 1u, __ATOMIC_RELAXED);
        }
      }
    }
    count.fetch_add(local, std::memory_order_relaxed);
  });
  parallel_for((int64_t)width * height, nthreads, [&](int64_t a, int64_t b) {
    for (int64_t px = a; px < b; ++px) {
      const uint32_t h = hits[px];
      if (!h) continue;
      for (int ch = 0; ch < 3; ++ch) {
        const uint64_t v = bgr[3 * px + ch] + (uint64_t)value * h;
        bgr[3 * px + ch] = (uint8_t)(v > 255u ? 255u : v);
      }
    }
  });
  if (splatted) *splatted = (uint32_t)count.load();
  return GS_OK;
}
