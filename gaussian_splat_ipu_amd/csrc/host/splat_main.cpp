// splat_main.cpp -- the render server on the C ABI (SURVEY §8 f1 + f3;
// reference: src/main/splat.cpp:24-329).
//
//   splat --input scene.ply [--device cpu|gpu] [--log-level info] [--ui-port 0]
//         [--gpus N] [--width 1280 --height 720 --tile-width 32 --tile-height 20]
//         [--frames 1] [--scale-div 0.1] [--out test.png] [--lattice]
//
// Same flags and flow as the reference: load the PLY, centre + negate z,
// build the Gaussians, set up the camera (lookAtBoundingBox, frustum fitted to
// the eye-space bounds, first view mvpStart), then the frame loop:
//   --device cpu  the reference's CPU point splatter (gs_cpu_point_splat,
//                 cpu_rasteriser.cpp:9-92), the reference's default device;
//   --device gpu  the Gaussian frame path on the MI355X (gs_render; "ipu" is
//                 accepted as an alias), --gpus N: N devices as one row-band
//                 group (one all-gather per frame inside gs_render);
//                 --lattice: every frame is one step of the emulated IPU
//                 lattice (GS_FLAG_LATTICE), the reference's own transient
//                 frames, instead of the converged single-frame binning.
// Without --ui-port the loop runs --frames frames (the reference: exactly one,
// splat.cpp:322) and logs "Splat time: {} points/sec: {}" (:318).  With
// --ui-port (built with REMOTE_UI=1) it serves one remote-UI client
// (remote_ui.hpp): after every frame the histogram and a preview go out on an
// AsyncTask thread, the UI state is consumed, the projection is refitted to
// the state's fov and the view rebuilt from its rotations and X/Y/Z
// (splat.cpp:280-315), until the client sends "stop".  test.png is the last
// rendered frame (splat.cpp:326).
#include <zlib.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/gsplat.h"
#include "../../../include/gsplat.hpp"
#if GSPLAT_REMOTE_UI
#include "remote_ui.hpp"
#endif

namespace {

struct Args {
  std::string input, device = "cpu", log_level = "info", out = "test.png", ui_host = "127.0.0.1";
  int ui_port = 0, frames = 1, gpus = 0;
  bool lattice = false;
  uint32_t width = 1280, height = 720, tw = 32, th = 20;
  float scale_div = -1.0f;  // default: lambda1 / 10 = 0.1 (InterfaceServer.hpp:238, splat.cpp:262)
};

void usage() {
  std::printf(
      "splat --input <file.ply|file.xyz> [--device cpu|gpu] [--log-level info] [--ui-port 0]\n"
      "      [--ui-host 127.0.0.1 (the address the UI server listens on; 0.0.0.0 = every interface)]\n"
      "      [--gpus N] [--width 1280] [--height 720] [--tile-width 32] [--tile-height 20]\n"
      "      [--frames 1] [--scale-div 0.1] [--out test.png] [--lattice]\n");
}

bool parse(int argc, char** argv, Args& a) {
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto val = [&](void) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", k.c_str());
        std::exit(EXIT_FAILURE);
      }
      return argv[++i];
    };
    if (k == "--help") {
      usage();
      std::exit(EXIT_SUCCESS);
    } else if (k == "--input" || k == "-o") {
      a.input = val();
    } else if (k == "--device") {
      a.device = val();
    } else if (k == "--log-level") {
      a.log_level = val();
    } else if (k == "--ui-port") {
      a.ui_port = std::atoi(val());
    } else if (k == "--ui-host") {
      a.ui_host = val();
    } else if (k == "--gpus") {
      a.gpus = std::atoi(val());
    } else if (k == "--width") {
      a.width = (uint32_t)std::atoi(val());
    } else if (k == "--height") {
      a.height = (uint32_t)std::atoi(val());
    } else if (k == "--tile-width") {
      a.tw = (uint32_t)std::atoi(val());
    } else if (k == "--tile-height") {
      a.th = (uint32_t)std::atoi(val());
    } else if (k == "--frames") {
      a.frames = std::atoi(val());
    } else if (k == "--scale-div") {
      a.scale_div = (float)std::atof(val());
    } else if (k == "--out") {
      a.out = val();
    } else if (k == "--lattice") {
      a.lattice = true;
    } else if (k == "--no-amp") {
      // accepted for compatibility (splat.cpp:34-35), no effect
    } else {
      std::fprintf(stderr, "unknown option %s\n", k.c_str());
      return false;
    }
  }
  if (a.input.empty()) {
    std::fprintf(stderr, "the option '--input' is required but missing\n");
    return false;
  }
  return true;
}

bool log_on(const Args& a, const char* level) {
  static const char* order[] = {"trace", "debug", "info", "warn", "err", "critical", "off"};
  int want = 2, have = 2;
  for (int i = 0; i < 7; ++i) {
    if (a.log_level == order[i]) want = i;
    if (std::strcmp(level, order[i]) == 0) have = i;
  }
  return have >= want && want < 6;
}

void put_u32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back((uint8_t)(x >> 24));
  v.push_back((uint8_t)(x >> 16));
  v.push_back((uint8_t)(x >> 8));
  v.push_back((uint8_t)x);
}

void chunk(std::vector<uint8_t>& png, const char* type, const std::vector<uint8_t>& data) {
  put_u32(png, (uint32_t)data.size());
  std::vector<uint8_t> td(type, type + 4);
  td.insert(td.end(), data.begin(), data.end());
  png.insert(png.end(), td.begin(), td.end());
  put_u32(png, (uint32_t)crc32(0L, td.data(), (uInt)td.size()));
}

// cv::imwrite("test.png", bgr) equivalent: 8-bit RGB PNG
bool write_png(const std::string& path, const uint8_t* bgr, uint32_t w, uint32_t h) {
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (w * 3 + 1));
  for (uint32_t y = 0; y < h; ++y) {
    raw.push_back(0);
    for (uint32_t x = 0; x < w; ++x) {
      const uint8_t* p = bgr + ((size_t)y * w + x) * 3;
      raw.push_back(p[2]);
      raw.push_back(p[1]);
      raw.push_back(p[0]);
    }
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return false;
  z.resize(zlen);
  std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put_u32(ihdr, w);
  put_u32(ihdr, h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
  chunk(png, "IHDR", ihdr);
  chunk(png, "IDAT", z);
  chunk(png, "IEND", {});
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(png.data(), 1, png.size(), f) == png.size();
  std::fclose(f);
  return ok;
}

float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }  // glm::radians

struct Mat4 {
  float m[16];  // glm column-major
};

Mat4 transposed(const Mat4& a) {
  Mat4 r;
  splat::gs_check(gs_mat4_transpose(a.m, r.m), "transpose");
  return r;
}

// The render-server's GPU device: one renderer, or a row-band group over
// --gpus devices, created on first use (a --device cpu run needs no GPU).
class GpuDevice {
 public:
  GpuDevice(const std::vector<gs_gaussian3d>& g, const Args& a) {
    gs_config cfg;
    splat::gs_check(gs_config_init(&cfg), "gs_config_init");
    cfg.width = a.width;
    cfg.height = a.height;
    cfg.tile_width = a.tw;
    cfg.tile_height = a.th;
    if (a.gpus > 0) {
      cfg.num_gpus = (uint32_t)a.gpus;
      for (int k = 0; k < a.gpus && k < GS_MAX_GPUS; ++k) cfg.device_ids[k] = k;
    }
    if (a.lattice) cfg.flags |= GS_FLAG_LATTICE;
    splat::gs_check(gs_create(g.data(), g.size(), &cfg, &r_), "gs_create");
  }
  ~GpuDevice() { gs_destroy(r_); }
  GpuDevice(const GpuDevice&) = delete;
  GpuDevice& operator=(const GpuDevice&) = delete;

  // splat.cpp:259-264: updateModelView, updateProjection, updateFocalLengths,
  // execute, getFrameBuffer; getIPUHistogram (:222)
  void frame(const Mat4& view, const Mat4& proj, float fov, float scale_div, std::vector<uint8_t>& bgr,
             std::vector<uint32_t>& hist) {
    splat::gs_check(gs_set_view(r_, transposed(view).m), "gs_set_view");
    splat::gs_check(gs_set_projection(r_, transposed(proj).m), "gs_set_projection");
    splat::gs_check(gs_set_focal(r_, fov, scale_div), "gs_set_focal");
    splat::gs_check(gs_render(r_), "gs_render");
    splat::gs_check(gs_read_bgr8(r_, bgr.data(), bgr.size()), "gs_read_bgr8");
    gs_frame_stats st;
    splat::gs_check(gs_get_stats(r_, &st), "gs_get_stats");
    hist.assign(st.n_tiles, 0u);
    splat::gs_check(gs_read_tile_histogram(r_, hist.data(), hist.size()), "gs_read_tile_histogram");
    n_rendered = st.n_rendered;
    n_pairs = st.n_pairs;
  }
  uint64_t n_rendered = 0, n_pairs = 0;

 private:
  gs_renderer* r_ = nullptr;
};

}  // namespace

int main(int argc, char** argv) {
  Args a;
  if (!parse(argc, argv, a)) {
    usage();
    return EXIT_FAILURE;
  }
#if !GSPLAT_REMOTE_UI
  if (a.ui_port != 0) {
    std::fprintf(stderr, "Exiting after: this splat was built without the remote UI (make REMOTE_UI=1).\n");
    return EXIT_FAILURE;
  }
#endif
  try {
    gs_ply* ply = nullptr;
    splat::gs_check(gs_ply_load(a.input.c_str(), &ply), "load");
    const int64_t n = gs_ply_count(ply);
    std::vector<gs_gaussian3d> g((size_t)n);
    float bb[6];
    splat::gs_check(gs_scene_prepare(ply, g.data(), g.size(), bb), "scene preparation");
    gs_ply_free(ply);
    if (log_on(a, "info")) {
      std::printf("[info] Total point count: %lld\n", (long long)n);
      std::printf("[info] Point bounds (centred, z negated): (%g, %g, %g) -> (%g, %g, %g)\n", bb[0], bb[1],
                  bb[2], bb[3], bb[4], bb[5]);
    }
    std::vector<float> xyz((size_t)n * 3);  // the points of the CPU path (pts[i].p)
    for (int64_t i = 0; i < n; ++i)
      for (int k = 0; k < 3; ++k) xyz[(size_t)i * 3 + k] = g[(size_t)i].mean[k];

    const float aspect = a.width / (float)a.height;  // splat.cpp:107
    // splat.cpp:186-195: modelView, eye-space bounds, fitted projection
    Mat4 modelView, projection, dynamicView;
    const float up[3] = {0.f, 1.f, 1.f};
    splat::gs_check(gs_cam_look_at_bbox(bb, bb + 3, up, 1.f, modelView.m), "lookAtBoundingBox");
    float bbCamMin[4], bbCamMax[4];
    {
      const float pmin[4] = {bb[0], bb[1], bb[2], 1.f}, pmax[4] = {bb[3], bb[4], bb[5], 1.f};
      gs_mat4_mul_vec4(modelView.m, pmin, bbCamMin);
      gs_mat4_mul_vec4(modelView.m, pmax, bbCamMax);
    }
#if GSPLAT_REMOTE_UI
    using State = gsui::InterfaceServer::State;
#else
    struct State {
      float envRotationDegrees = 0.f, envRotationDegrees2 = 0.f, X = 640.f, Y = 360.f, Z = 1.f, lambda1 = 1.f,
            fov = 90.f;
      std::string device = "cpu";
      bool stop = false;
    };
#endif
    State state;
    state.fov = radians(40.f);  // splat.cpp:175
    state.device = a.device;
    if (a.scale_div > 0.f) state.lambda1 = a.scale_div * 10.f;
#if GSPLAT_REMOTE_UI
    std::unique_ptr<gsui::InterfaceServer> ui;
    if (a.ui_port) {
      ui.reset(new gsui::InterfaceServer(a.ui_port, a.ui_host.c_str()));
      if (!ui->start(state)) throw std::runtime_error("remote UI server could not start");
      ui->updateFov(state.fov);
    }
#endif
    splat::gs_check(gs_cam_fit_frustum(bbCamMin, bbCamMax, state.fov, aspect, projection.m), "fitFrustum");
    splat::gs_check(gs_cam_mvp_start(dynamicView.m), "mvpStart");  // splat.cpp:235-244

    std::unique_ptr<GpuDevice> gpu;
    const size_t px = (size_t)a.width * a.height;
    std::vector<uint8_t> image(px * 3, 0), imageBuffered(px * 3, 0);
    std::vector<uint32_t> hist, histBuffered;
#if GSPLAT_REMOTE_UI
    gsui::AsyncTask hostProcessing;
#endif
    double secondsElapsed = 0.0;
    int frame = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      std::fill(image.begin(), image.end(), (uint8_t)0);  // *imagePtr = 0 (splat.cpp:247)
      uint32_t count = 0;
      const float scaleDiv = state.lambda1 / 10.f;
      if (state.device == "cpu") {
        hist.assign((size_t)(a.width / a.tw) * (a.height / a.th), 0u);
        splat::gs_check(gs_cpu_point_splat(xyz.data(), (size_t)n, transposed(dynamicView).m, transposed(projection).m,
                                           a.width, a.height, a.tw, a.th, 25, image.data(), hist.data(), &count, 0),
                        "splatPoints");
      } else if (state.device == "gpu" || state.device == "ipu") {
        if (!gpu) gpu.reset(new GpuDevice(g, a));
        gpu->frame(dynamicView, projection, state.fov, scaleDiv, image, hist);
        count = (uint32_t)gpu->n_rendered;
      } else if (log_on(a, "warn")) {
        std::printf("[warn] unknown device '%s': nothing rendered\n", state.device.c_str());
      }
      const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      secondsElapsed += secs;
      ++frame;
#if GSPLAT_REMOTE_UI
      if (ui) {
        if (secondsElapsed > 3.0 && log_on(a, "info"))
          std::printf("[info] Splat time: %g points/sec: %g\n", secs, (double)n / secs);
        // splat.cpp:280-315
        hostProcessing.waitForCompletion();
        std::swap(image, imageBuffered);
        std::swap(hist, histBuffered);
        hostProcessing.run([&] {
          ui->sendHistogram(histBuffered);
          ui->sendPreviewImage(imageBuffered.data(), (int)a.width, (int)a.height);
        });
        state = ui->consumeState();
        splat::gs_check(gs_cam_fit_frustum(bbCamMin, bbCamMax, state.fov, aspect, projection.m), "fitFrustum");
        if (secondsElapsed >= 3.0) {
          if (log_on(a, "info"))
            std::printf("[info] envRotationDegrees: %f envRotationDegrees2: %f lambda1: %f fov: %f\n",
                        state.envRotationDegrees, state.envRotationDegrees2, state.lambda1, state.fov);
          secondsElapsed = 0.0;
        }
        Mat4 id, t;
        for (int i = 0; i < 16; ++i) id.m[i] = (i % 5 == 0) ? 1.f : 0.f;
        const float ax[3] = {1.f, 0.f, 0.f}, ay[3] = {0.f, 1.f, 0.f};
        splat::gs_check(gs_cam_rotate(id.m, radians(state.envRotationDegrees), ax, t.m), "rotate");
        splat::gs_check(gs_mat4_mul(modelView.m, t.m, dynamicView.m), "modelView * rotate");
        splat::gs_check(gs_cam_rotate(dynamicView.m, radians(state.envRotationDegrees2), ay, t.m), "rotate");
        const float tr[3] = {state.X / 50.f, state.Y / 50.f, -state.Z / 20.f + 20.f};
        splat::gs_check(gs_cam_translate(t.m, tr, dynamicView.m), "translate");
        if (state.stop) break;
        continue;
      }
#endif
      if (log_on(a, "info")) {
        std::printf("[info] Splat time: %g points/sec: %g\n", secs, (double)n / secs);
        std::printf("[info] Splatted point count: %u\n", count);
      }
      if (frame >= a.frames) break;
    }
#if GSPLAT_REMOTE_UI
    hostProcessing.waitForCompletion();
    if (ui) std::swap(image, imageBuffered);  // the last rendered frame
#endif
    if (!write_png(a.out, image.data(), a.width, a.height)) {
      std::fprintf(stderr, "could not write %s\n", a.out.c_str());
      return EXIT_FAILURE;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[info] Exiting after: %s.\n", e.what());
    return EXIT_FAILURE;
  }
  return EXIT_SUCCESS;
}
