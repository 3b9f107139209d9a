// splat_main.cpp -- the render server's headless frame loop on the C ABI
// (reference: src/main/splat.cpp:24-329).
//
//   splat --input scene.ply [--device gpu] [--log-level info] [--ui-port 0]
//         [--width 1280 --height 720 --tile-width 32 --tile-height 20]
//         [--frames 1] [--scale-div 0.1] [--out test.png]
//
// Same flags and flow as the reference: load the PLY, centre + negate z,
// build the Gaussians, set up the headless camera, render, log
// "Splat time: {} points/sec: {}" per frame (splat.cpp:272,318) and write
// test.png (splat.cpp:326).  --device gpu replaces --device ipu; the
// reference's --device cpu point splatter and the remote UI (--ui-port) are
// not part of this build and are rejected with a clear message.
#include <zlib.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/gsplat.h"
#include "../../../include/gsplat.hpp"

namespace {

struct Args {
  std::string input, device = "gpu", log_level = "info", out = "test.png";
  int ui_port = 0, frames = 1;
  uint32_t width = 1280, height = 720, tw = 32, th = 20;
  float scale_div = 0.1f;  // lambda1 / 10 (InterfaceServer.hpp:238, splat.cpp:262)
};

void usage() {
  std::printf(
      "splat --input <file.ply|file.xyz> [--device gpu] [--log-level info] [--ui-port 0]\n"
      "      [--width 1280] [--height 720] [--tile-width 32] [--tile-height 20]\n"
      "      [--frames 1] [--scale-div 0.1] [--out test.png]\n");
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

}  // namespace

int main(int argc, char** argv) {
  Args a;
  if (!parse(argc, argv, a)) {
    usage();
    return EXIT_FAILURE;
  }
  if (a.ui_port != 0) {
    std::fprintf(stderr, "Exiting after: remote UI (--ui-port) is not part of this build.\n");
    return EXIT_FAILURE;
  }
  if (a.device != "gpu") {
    std::fprintf(stderr, "Exiting after: --device %s is not supported (use --device gpu).\n",
                 a.device.c_str());
    return EXIT_FAILURE;
  }
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
      std::printf("[info] Point bounds (centred, z negated): (%g, %g, %g) -> (%g, %g, %g)\n", bb[0],
                  bb[1], bb[2], bb[3], bb[4], bb[5]);
    }
    splat::GpuFramebuffer fb{a.width, a.height, a.tw, a.th};
    splat::GpuSplatter splatter(g, fb);
    float view_rm[16], proj_rm[16];
    const float fov = 40.0f * 0.01745329251994329576923690768489f;  // glm::radians(40.f)
    splat::gs_check(gs_cam_headless(bb, a.width, a.height, fov, view_rm, proj_rm), "camera");
    splat::gs_check(gs_set_view(splatter.handle(), view_rm), "view");
    splat::gs_check(gs_set_projection(splatter.handle(), proj_rm), "projection");
    splatter.updateFocalLengths(fov, a.scale_div);
    std::vector<uint8_t> bgr;
    for (int f = 0; f < a.frames; ++f) {
      const auto t0 = std::chrono::steady_clock::now();
      splatter.execute();
      splatter.getFrameBuffer(bgr);
      const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (log_on(a, "info")) {
        const gs_frame_stats st = splatter.stats();
        std::printf("[info] Splat time: %g points/sec: %g\n", secs, (double)n / secs);
        std::printf("[info] Splatted point count: %llu (tile pairs %llu)\n",
                    (unsigned long long)st.n_rendered, (unsigned long long)st.n_pairs);
      }
    }
    if (!write_png(a.out, bgr.data(), a.width, a.height)) {
      std::fprintf(stderr, "could not write %s\n", a.out.c_str());
      return EXIT_FAILURE;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[info] Exiting after: %s.\n", e.what());
    return EXIT_FAILURE;
  }
  return EXIT_SUCCESS;
}
