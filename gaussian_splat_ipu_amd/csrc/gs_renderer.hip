// gs_renderer.hip -- host side of the C ABI (include/gsplat.h): the MI355X
// replacement of splat::IpuSplatter (src/splat/ipu_rasteriser.cpp).
//
// Owns one device's copy of the scene (SoA, uploaded once like the reference's
// "write_verts" program, ipu_rasteriser.cpp:401-418), the per-frame workspace
// and the outputs, and enqueues the five stages of the frame on one HIP
// stream.  No exceptions cross the ABI; failures return a gs_status and set the
// thread-local message of gs_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gsplat.h"
#include "gs_internal.hpp"
#include "gs_kernels.hpp"
#include "host/gs_host.hpp"

using gsh::set_error;

namespace {
// scene allocation: the 64-B records (SoA), the permutation both ways, then
// the band cull's 16-B records (16-B aligned)
size_t cull_offset(size_t nn) { return (nn * (64 + 8) + 15) / 16 * 16; }
// + the band cull's records (16 B) + mean xyz with the opacity (16 B)
size_t scene_bytes(size_t nn) { return cull_offset(nn) + nn * 32; }
}  // namespace

#ifndef GS_X_BAND
#define GS_X_BAND 0
#endif
#ifndef GS_X_DIRECT_OFF
#define GS_X_DIRECT_OFF 0
#endif

namespace gsr {

int hip_fail(hipError_t e, const char* what) {
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return GS_EOOM;
  return GS_EDEVICE;
}

int select_device(gs_renderer* r) {
  GS_HIP(hipSetDevice(r->device));
  return GS_OK;
}

// gs_test_set (include/gsplat.h): the test hooks gs_create reads
std::atomic<int64_t> g_test_chunk_size{0}, g_test_bin_agg{-1}, g_test_poison{0}, g_test_cov_cache{-1},
    g_test_bin_direct{-1};

// gs_test_set("debug_poison", 1): every device buffer is filled with 0xA5
// bytes when it is allocated (before any initialisation the renderer does
// itself), so a kernel that reads memory no earlier stage of the frame wrote
// gives a different frame than in a fresh process (tests/test_gpu_poison.py).
void poison(void* p, size_t bytes, const char* name) {
  (void)name;
  if (!p || !bytes || g_test_poison.load() == 0) return;
  (void)hipMemset(p, 0xA5, bytes);
}

void free_pairs(gs_renderer* r) {
  if (r->d_pairs) (void)hipFree(r->d_pairs);
  r->d_pairs = nullptr;
}

// Device order of the Gaussians: 3D Morton order of the means (21 bits per
// axis over their bounding box; non-finite coordinates count as the box
// minimum), ties by input index.  Neighbours in this order are neighbours on
// screen, so a binning chunk's entries of one tile are contiguous and a tile's
// records share cache lines.  The order is an internal layout: keys carry the
// input index, so the depth order (ties by input index) is unchanged.
std::vector<uint32_t> morton_order(const gs_gaussian3d* g, size_t n, bool keep) {
  std::vector<uint32_t> perm(n);
  for (size_t i = 0; i < n; ++i) perm[i] = (uint32_t)i;
  if (keep || n < 2) return perm;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (size_t i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a) {
      const float v = g[i].mean[a];
      if (std::isfinite(v)) {
        lo[a] = std::min(lo[a], v);
        hi[a] = std::max(hi[a], v);
      }
    }
  auto spread = [](uint64_t v) {  // 21 bits -> every third bit
    v &= 0x1FFFFFull;
    v = (v | (v << 32)) & 0x1F00000000FFFFull;
    v = (v | (v << 16)) & 0x1F0000FF0000FFull;
    v = (v | (v << 8)) & 0x100F00F00F00F00Full;
    v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
    v = (v | (v << 2)) & 0x1249249249249249ull;
    return v;
  };
  std::vector<std::pair<uint64_t, uint32_t>> key(n);
  for (size_t i = 0; i < n; ++i) {
    uint64_t c = 0;
    for (int a = 0; a < 3; ++a) {
      const float v = g[i].mean[a];
      double t = 0.0;
      if (std::isfinite(v) && hi[a] > lo[a]) t = ((double)v - lo[a]) / ((double)hi[a] - lo[a]);
      const uint64_t q = (uint64_t)std::min(2097151.0, std::max(0.0, t * 2097151.0));
      c |= spread(q) << a;
    }
    key[i] = {c, (uint32_t)i};
  }
  std::sort(key.begin(), key.end());
  for (size_t i = 0; i < n; ++i) perm[i] = key[i].second;
  return perm;
}

int alloc_pairs(gs_renderer* r, uint64_t cap) {
  free_pairs(r);
  // + one u32 per 2048-key work item a big list can have, and the big-list
  // sample sort's bucket tables (one bucket per ~1024 keys, gs_kernels.hip kBktAvg)
  const size_t n_items = (size_t)(cap / 2048) + (size_t)r->n_tiles + 1;
  const size_t n_bk = (size_t)(cap / 1024) + (size_t)r->n_tiles + 1;
  const size_t bytes = (size_t)cap * (8 + 8 + 4) + n_bk * 8 + n_items * 4 + n_bk * 12 +
                       ((size_t)r->n_tiles + 1) * 4;
  GS_HIP(hipMalloc(&r->d_pairs, bytes));
  poison(r->d_pairs, bytes, "pairs");
  r->pair_cap = cap;
  char* p = (char*)r->d_pairs;
  r->buf.pairs = (unsigned long long*)p;
  r->buf.pairs_alt = (unsigned long long*)(p + (size_t)cap * 8);
  p += (size_t)cap * 16;
  r->buf.bk_spl = (unsigned long long*)p;
  p += n_bk * 8;
  r->buf.list = (uint32_t*)p;
  p += (size_t)cap * 4;
  r->buf.big_item = (uint32_t*)p;
  p += n_items * 4;
  r->buf.bk_start = (uint32_t*)p;
  r->buf.bk_cnt = r->buf.bk_start + n_bk;
  r->buf.bk_list = r->buf.bk_cnt + n_bk;
  r->buf.bk_off = r->buf.bk_list + n_bk;
  return GS_OK;
}

// probe builds: the ring of this renderer's frames appended to
// GSPLAT_PROBE_FILE (tools/probe_timeline.py): "GSPR", the device, the
// frames recorded (the last kProbeFrames, oldest first), the kernel count,
// then [frames][kProbeKernels][start, end] u64 (100 MHz wall clock, reduced
// over the slots; start ~0 / end 0 = the kernel did not run)
void dump_probe(gs_renderer* r) {
  const char* path = std::getenv("GSPLAT_PROBE_FILE");
  const int nf = std::min(r->probe_n, gsk::kProbeFrames);
  if (!path || nf <= 0) return;
  const size_t per_frame = (size_t)gsk::kProbeKernels * gsk::kProbeSlots * 2;
  std::vector<unsigned long long> h((size_t)gsk::kProbeFrames * per_frame);
  if (hipMemcpy(h.data(), r->d_probe, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  std::vector<unsigned long long> out((size_t)nf * gsk::kProbeKernels * 2);
  for (int j = 0; j < nf; ++j) {
    const int f = (r->probe_n - nf + j) % gsk::kProbeFrames;
    for (int k = 0; k < gsk::kProbeKernels; ++k) {
      unsigned long long s = ~0ull, e = 0ull;
      const unsigned long long* p = h.data() + (size_t)f * per_frame + (size_t)k * gsk::kProbeSlots * 2;
      for (int q = 0; q < gsk::kProbeSlots; ++q) {
        s = std::min(s, p[2 * q]);
        e = std::max(e, p[2 * q + 1]);
      }
      out[((size_t)j * gsk::kProbeKernels + k) * 2] = s;
      out[((size_t)j * gsk::kProbeKernels + k) * 2 + 1] = e;
    }
  }
  if (FILE* f = std::fopen(path, "ab")) {
    const int32_t hdr[4] = {0x52505347, r->device, nf, gsk::kProbeKernels};
    std::fwrite(hdr, 4, 4, f);
    std::fwrite(out.data(), 8, out.size(), f);
    std::fclose(f);
  }
}

#if GS_LANES
// lane-count builds: the blend counters of this renderer's frames appended to
// GSPLAT_LANES_FILE (tools/blend_lanes.py): 8 u64
void dump_lanes(gs_renderer* r) {
  const char* path = std::getenv("GSPLAT_LANES_FILE");
  unsigned long long h[8] = {};
  if (!path || hipMemcpy(h, r->buf.lanes, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return;
  if (FILE* f = std::fopen(path, "ab")) {
    std::fwrite(h, 8, 8, f);
    std::fclose(f);
  }
}
#endif

void release(gs_renderer* r) {
  if (!r) return;
  (void)hipSetDevice(r->device);
  if (r->stream) (void)hipStreamSynchronize(r->stream);
  if (r->d_scene && r->owns_scene) (void)hipFree(r->d_scene);
  if (r->d_probe) dump_probe(r);
#if GS_LANES
  if (r->buf.lanes) {
    dump_lanes(r);
    (void)hipFree(r->buf.lanes);
  }
#endif
  for (void* p : {r->d_gauss, r->d_zero, r->d_tiles, r->d_out, r->d_chunk, r->d_lazy, r->d_lat, r->d_bcount, r->d_agg, r->d_dir, r->d_cov,
                  r->d_probe})
    if (p) (void)hipFree(p);
  if (r->d_sh && r->owns_sh) (void)hipFree(r->d_sh);
  free_pairs(r);
  if (r->h_counters) (void)hipHostFree(r->h_counters);
  for (auto& s : r->ring)
    for (auto& e : s.ev)
      if (e) (void)hipEventDestroy(e);
  if (r->own_stream) (void)hipStreamDestroy(r->own_stream);
}

// bands: the chunk count grows with the band's share of the tiles up to this
// (gs_colscan_kernel walks a tile's chunk rows: past 256 of them it reads
// them twice, in batches of 8)
constexpr size_t kMaxBandChunks = 1024;
// the aggregated binning up to this many tiles per frame (or band)
constexpr int kAggMaxTiles = 16384;

gsk::FrameParams make_params(const gs_renderer* r) {
  gsk::FrameParams fp{};
  // mvp = projmatrix * viewmatrix, both from the row-major wire format
  // (codelets.cpp:625-628, 443): glm::transpose(glm::make_mat4(p)).
  float view[16], proj[16];
  gsh::mat4_transpose(r->view_rm, view);
  gsh::mat4_transpose(r->proj_rm, proj);
  gsh::mat4_mul(proj, view, fp.mvp);
  // codelets.cpp:444-448
  fp.tanfov = (float)std::tan(0.5 * (double)r->fov);
  const float tf = std::tan(r->fov / 2.0f);
  fp.focal_x = (float)r->cfg.width / (2.0f * tf);
  fp.focal_y = (float)r->cfg.height / (2.0f * tf);
  const uint32_t gw = r->cfg.guard_tile_width ? r->cfg.guard_tile_width : r->cfg.tile_width;
  const uint32_t gh = r->cfg.guard_tile_height ? r->cfg.guard_tile_height : r->cfg.tile_height;
  const float gx = (float)gw, gy = (float)gh;
  fp.guard_thr = std::sqrt(gx * gx + gy * gy) * r->cfg.guard_band;  // codelets.cpp:470
  fp.scale_div = r->scale_div;
  fp.W = (float)r->cfg.width;
  fp.H = (float)r->cfg.height;
  fp.tw = (float)r->cfg.tile_width;
  fp.th = (float)r->cfg.tile_height;
  fp.width = (int)r->cfg.width;
  fp.height = (int)r->cfg.height;
  fp.tile_w = (int)r->cfg.tile_width;
  fp.tile_h = (int)r->cfg.tile_height;
  fp.tiles_x = r->tiles_x;
  fp.band_ty0 = r->band_ty0;
  fp.band_stride = r->band_stride;
  fp.band_nrows = r->band_nrows;
  fp.tiles_y = r->tiles_y;
  fp.band_rows = r->band_rows;
  fp.band_cull = ((r->cfg.flags & GS_FLAG_BAND_CULL) && r->band_nrows < r->tiles_y) ? 1 : 0;
  fp.n = (int)r->n;
  fp.n_tiles = r->n_tiles;
  // blend: one wave per 16 pixel quads -- an 8x8 or 16x4 pixel block when the
  // tile is a multiple of it, else a run of quads
  const uint32_t tw = r->cfg.tile_width, th = r->cfg.tile_height;
  fp.blend_bqw = (tw % 8 == 0 && th % 8 == 0) ? 4 : ((tw % 16 == 0 && th % 4 == 0) ? 8 : 0);
  fp.chunks_per_tile = fp.blend_bqw == 4   ? (int)((tw / 8) * (th / 8))
                       : fp.blend_bqw == 8 ? (int)((tw / 16) * (th / 4))
                                           : (int)((((tw + 1) / 2) * ((th + 1) / 2) + 15) / 16);
  fp.blend_lpt = r->band_nrows < r->tiles_y ? 1 : 0;
  // the tile sort inside the blend's workgroups (16x16 tiles: one workgroup
  // per tile) for row bands: 8 bands of config 4, 38.2 -> 37.2 us per frame;
  // whole frames keep the sort launch (config 3: 7 980 against 7 800
  // frames/s, the sort launch overlapping the other frames' blends better;
  // config 5 1 440 against 1 453).
  // The aggregated emit runs as 2048 workgroups walking the 256-Gaussian
  // blocks (one resident round: 8 per CU) rather than one per block: a band's
  // culled blocks cost a loop iteration, not a workgroup.
  fp.emit_grid = 2048;
  fp.blend_sort = (fp.blend_bqw == 4 && fp.chunks_per_tile == 4 && r->band_nrows < r->tiles_y) ? 1 : 0;
  fp.pair_cap = r->pair_cap;
  fp.write_rgba = (r->cfg.flags & GS_FLAG_NO_RGBA32F) ? 0 : 1;
  fp.bgr_pitch = (int)r->cfg.width * 3;
  fp.bin_global = r->bin_global;
  fp.chunk_size = r->chunk_size;
  fp.n_chunks = r->n_chunks;
  if (r->chunk_adaptive && r->n_chunks > 0 && r->n_tiles > 0 &&
      (size_t)r->n_tiles * (size_t)r->n_chunks < r->chunk_entries) {
    // a band: as many chunks as the table holds for its tiles, of >= 4096
    // Gaussians (smaller ones made the 1M-Gaussian bands slower: 8 bands,
    // 40.5 -> 48-51 us per frame; at 8 M, 8 bands, 287 -> 253 us)
    const size_t nc = std::min<size_t>(r->chunk_entries / (size_t)r->n_tiles, kMaxBandChunks);
    const size_t cs = std::min<size_t>(65535, std::max<size_t>(4096, (r->n + nc - 1) / nc));
    fp.chunk_size = (int)cs;
    fp.n_chunks = (int)((r->n + cs - 1) / cs);
  }
  fp.emit_wide = (size_t)r->n_tiles * 4 <= gsk::kBinLdsMax ? 1 : 0;
  // aggregated binning: row bands (8 bands of config 4: 39.7 -> 37.2 us per
  // frame; of config 5: 294 -> 259 us); whole frames keep the chunked
  // binning (config 3: 8 087 against 8 057 frames/s; config 5's 32 400
  // tiles: 1 447 against 1 444, its projection 156 against 224 us from the
  // clustered scene's hot-tile atomics)
  fp.bin_agg = (r->bin_agg && !r->lattice && r->band_nrows < r->tiles_y && r->n_tiles <= kAggMaxTiles) ? 1 : 0;
  fp.pair_cull = (r->pair_cull && !r->bin_global && ((r->n_chunks > 0 && fp.emit_wide) || fp.bin_agg)) ? 1 : 0;
  fp.mean_w1 = r->scene_w1 ? 1 : 0;
  fp.cov_cache = r->d_cov ? 1 : 0;
  // both rectangles in one 8-B word per Gaussian when every bound fits 8 bits
  fp.rect8 = (fp.pair_cull && r->tiles_x <= 256 && r->band_nrows <= 256) ? 1 : 0;
  // the big-list launch only when the last frame the device completed had
  // big lists (a hint read from the mapped counters: either choice sorts
  // every list, the other launch handles them otherwise)
  fp.big_separate = (r->h_counters && ((volatile const uint32_t*)r->h_counters)[0] > 0) ? 1 : 0;
  // lazy big lists: sort only the lists' nearest keys before the blend
  fp.lazy = (fp.big_separate && r->d_lazy && fp.blend_bqw == 4 && fp.chunks_per_tile == 4 && !r->bin_global &&
             r->n_chunks > 0) ? 1 : 0;
  fp.big_pass = 0;
  fp.blend_cont = 0;
  // two pixels per blend lane on whole frames without lazy big lists
  // (config 3: 8 235 -> 8 454 frames/s, three interleaved repeats, although
  // the blend alone, one frame in flight, takes 87 instead of 77 us: half
  // the waves, each with two pixel chains, leave CUs to the other frames and
  // stage each tile's records twice instead of four times).  Lazy frames
  // (config 5) keep one pixel per lane: the continuation resumes those waves.
  // blend_wave_px2 maps a wave onto a 16x8 half of a 16x16 tile: other
  // shapes with four 8x8 blocks (32x8, 8x32) keep one pixel per lane.
  const bool tile16 = tw == 16 && th == 16;
  fp.blend_px2 = (tile16 && !fp.blend_sort && !fp.lazy) ? 1 : 0;
  // two-pixel lanes walk a tile's list in half the waves, so a heavy tile's
  // walk is twice as long: its waves start first (the sort queues' order,
  // longest lists first) -- config 3 blend 86.4 -> 79.4 us alone, 8 451 ->
  // 8 524 frames/s, three interleaved repeats
  if (fp.blend_px2) fp.blend_lpt = 1;
  // ... and read their slot's tile and list segment in one load, written by
  // the sort launch (which sorts every list when big_separate is off)
  fp.blend_seg = (fp.blend_px2 && !fp.big_separate) ? 1 : 0;
  fp.bin_direct = 0;
  fp.fast_exp = (r->cfg.flags & GS_FLAG_FAST_EXP) ? 1 : 0;
  fp.sh_degree = r->d_sh ? r->sh_degree : -1;
  camera_position(r->view_rm, fp.campos);
  {
    auto log2_exact = [](double v, int& sh) -> bool {  // v == 2^sh, sh in [-126, 126]
      int e = 0;
      const double m = std::frexp(v, &e);  // v = m * 2^e, m in [0.5, 1)
      sh = e - 1;
      return v > 0.0 && m == 0.5 && sh >= -126 && sh <= 126;
    };
    int stw = 0, sth = 0, sst = 0, ssd = 0;
    fp.pow2 = (log2_exact(fp.tile_w, stw) && log2_exact(fp.tile_h, sth) && log2_exact(fp.band_stride, sst) &&
               log2_exact(fp.scale_div, ssd)) ? 1 : 0;
    fp.sh_tw = stw;
    fp.sh_th = sth;
    fp.sh_stride = sst;
    fp.inv_tw = std::ldexp(1.0f, -stw);
    fp.inv_th = std::ldexp(1.0f, -sth);
    fp.inv_sd = std::ldexp(1.0f, -ssd);
  }
  return fp;
}

void camera_position(const float* v, float* campos) {
  // view (row-major wire) = [A t; 0 1]: the camera sits at -A^-1 t
  double a[3][3], t[3];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) a[i][j] = v[i * 4 + j];
    t[i] = v[i * 4 + 3];
  }
  const double c00 = a[1][1] * a[2][2] - a[1][2] * a[2][1];
  const double c01 = a[1][2] * a[2][0] - a[1][0] * a[2][2];
  const double c02 = a[1][0] * a[2][1] - a[1][1] * a[2][0];
  const double det = (a[0][0] * c00 + a[0][1] * c01) + a[0][2] * c02;
  double inv[3][3];
  inv[0][0] = c00;
  inv[1][0] = c01;
  inv[2][0] = c02;
  inv[0][1] = a[0][2] * a[2][1] - a[0][1] * a[2][2];
  inv[1][1] = a[0][0] * a[2][2] - a[0][2] * a[2][0];
  inv[2][1] = a[0][1] * a[2][0] - a[0][0] * a[2][1];
  inv[0][2] = a[0][1] * a[1][2] - a[0][2] * a[1][1];
  inv[1][2] = a[0][2] * a[1][0] - a[0][0] * a[1][2];
  inv[2][2] = a[0][0] * a[1][1] - a[0][1] * a[1][0];
  for (int i = 0; i < 3; ++i)
    campos[i] = (float)(-((inv[i][0] * t[0] + inv[i][1] * t[1]) + inv[i][2] * t[2]) / det);
}

int set_sh(gs_renderer* r, const float* f_dc, const float* f_rest, size_t n, int degree, const gs_renderer* share) {
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  // a frame in flight may still read the coefficients: done before they change
  if (r->frame_pending) GS_HIP(hipStreamSynchronize(r->stream));
  auto drop = [&] {
    if (r->d_sh && r->owns_sh) (void)hipFree(r->d_sh);
    r->d_sh = nullptr;
    r->owns_sh = false;
    r->buf.sh = nullptr;
    r->sh_degree = -1;
  };
  if (degree < 0) {
    drop();
    return GS_OK;
  }
  if (degree > 3 || n != r->n || !f_dc || (degree > 0 && !f_rest)) {
    set_error("gs_set_sh: need degree 0..3, n equal to the scene's Gaussians, f_dc and (degree > 0) f_rest");
    return GS_EINVAL;
  }
  if (share && share != r && share->device == r->device && share->n == r->n && share->d_sh &&
      share->sh_degree == degree && share->d_scene == r->d_scene) {
    drop();
    r->d_sh = share->d_sh;  // the same coefficients in the same device order
    r->buf.sh = (const float*)r->d_sh;
    r->sh_degree = degree;
    return GS_OK;
  }
  const size_t nn = std::max<size_t>(n, 1);
  const int K = (degree + 1) * (degree + 1);
  // [K x 3][n], device order: only the planes the degree reads
  // (sh_colour reads coefficient k < (degree + 1)^2)
  std::vector<float> h((size_t)K * 3 * nn, 0.0f);
  for (size_t i = 0; i < n; ++i) {
    const size_t o = r->perm[i];  // device index i holds input Gaussian o
    for (int c = 0; c < 3; ++c) {
      h[(size_t)(0 * 3 + c) * nn + i] = f_dc[o * 3 + c];
      for (int k = 1; k < K; ++k) h[(size_t)(k * 3 + c) * nn + i] = f_rest[o * 45 + (size_t)c * 15 + (k - 1)];
    }
  }
  // the new copy first: if it fails, the renderer (and any renderer sharing
  // its old copy) keeps the old coefficients
  void* d_new = nullptr;
  GS_HIP(hipMalloc(&d_new, h.size() * 4));
  const hipError_t e = hipMemcpy(d_new, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(d_new);
    return hip_fail(e, "gs_set_sh: hipMemcpy");
  }
  drop();
  r->d_sh = d_new;
  r->owns_sh = true;
  r->buf.sh = (const float*)r->d_sh;
  r->sh_degree = degree;
  return GS_OK;
}

int profile_harvest(gs_renderer* r, ProfileSlot& s) {
  if (!s.pending) return GS_OK;
  GS_HIP(hipEventSynchronize(s.ev[gsk::GS_STAGE_EVENTS - 1]));
  for (int k = 0; k < kStages; ++k) {
    float ms = 0.0f;
    GS_HIP(hipEventElapsedTime(&ms, s.ev[k], s.ev[k + 1]));
    r->k_ms[kStageKernel[k]] += ms;
    r->k_launches[kStageKernel[k]] += 1;
  }
  s.pending = false;
  return GS_OK;
}

// GS_FLAG_LATTICE: one step of the emulated lattice (compute set + exchange,
// ipu_rasteriser.cpp:393-399); its kernel time is reported as the blend stage
int enqueue_lattice(gs_renderer* r, const gsk::FrameParams& fp, ProfileSlot* slot) {
  hipStream_t s = r->stream;
  gsk::LatticeParams lp{};
  std::memcpy(lp.mvp, fp.mvp, sizeof(lp.mvp));
  lp.tanfov = fp.tanfov;
  lp.focal_x = fp.focal_x;
  lp.focal_y = fp.focal_y;
  lp.guard_thr = fp.guard_thr;
  lp.scale_div = fp.scale_div;
  lp.W = fp.W;
  lp.H = fp.H;
  lp.tw = fp.tw;
  lp.th = fp.th;
  lp.across = (float)r->tiles_x;
  lp.width = fp.width;
  lp.height = fp.height;
  lp.tile_w = fp.tile_w;
  lp.tile_h = fp.tile_h;
  lp.tiles_x = r->tiles_x;
  lp.n_tiles = r->tiles_x * r->tiles_y;
  lp.gpt = r->lat_gpt;
  lp.rem = r->lat_rem;
  lp.parity = (int)(r->lat_frames & 1);
  lp.write_rgba = fp.write_rgba;
  lp.bgr_pitch = fp.bgr_pitch;
  gsk::LatticeBufs lb = r->lat;
  lb.rgba = r->buf.rgba;
  lb.bgr = r->buf.bgr;
  lb.host_counters = r->buf.host_counters;
  if (slot)
    for (int k = 0; k < gsk::GS_STAGE_EVENTS - 2; ++k) GS_HIP(hipEventRecord(slot->ev[k], s));
  gsk::launch_lattice(lp, lb, s);
  if (slot) {
    GS_HIP(hipEventRecord(slot->ev[gsk::GS_STAGE_EVENTS - 2], s));
    GS_HIP(hipEventRecord(slot->ev[gsk::GS_STAGE_EVENTS - 1], s));
    slot->pending = true;
  }
  GS_HIP(hipGetLastError());
  r->lat_frames++;
  r->frame_pending = true;
  return GS_OK;
}

// FrameParams::cov_cache: the scene's 3D covariances for fp's fxy[1], computed
// on the renderer's stream before the projection that first needs them (the
// frames in flight on this stream are ordered behind it)
int ensure_cov(gs_renderer* r, const gsk::FrameParams& fp, hipStream_t s) {
  if (!fp.cov_cache || (r->cov_valid && r->cov_sd == fp.scale_div)) return GS_OK;
  gsk::launch_cov3d(fp, r->buf, s);
  GS_HIP(hipGetLastError());
  r->cov_sd = fp.scale_div;
  r->cov_valid = true;
  return GS_OK;
}

// Direct band binning (FrameParams::bin_direct).  A row band whose camera,
// projection, focal lengths and band have not changed since a frame binned
// by the scan and emit has completed bins the same lists again: each tile's
// pairs then go straight to that frame's segment of the pair buffer
// (tile_start, left by the scan), placed by the projection itself, and the
// scan and emit launches leave the band's chain.  The first frame of a view
// (and any frame enqueued before one of its view has completed) takes the
// scan and emit.  A direct frame whose pairs do not fit their segments (only
// the test hook's forced frames can) drops the pairs past them and reports
// GS_EOVERFLOW like a pair-buffer overflow; the next frame takes the scan.
// Test hook (gs_test_set "bin_direct"): 0 off, > 0 forced on (the first
// frame too, into whatever layout tile_start holds) until an overflow.
void choose_direct(const gs_renderer* r, gsk::FrameParams& fp) {
  fp.bin_direct = 0;
  const int64_t hook = GS_X_DIRECT_OFF ? 0 : g_test_bin_direct.load();  // (measurement builds: off)
  if (hook == 0 || !fp.blend_sort || fp.lazy || r->bin_global || r->n_tiles <= 0 || !r->buf.dir_word ||
      !r->h_counters || gsk::project_kind(fp, r->buf) != 2)  // (2: the row band's projection)
    return;
  const volatile uint32_t* h = (const volatile uint32_t*)r->h_counters;
  const uint32_t hseq = h[15];  // the last completed frame
  const bool known = r->layout_seq != 0 && (int32_t)(r->layout_seq - r->cam_first_seq) >= 0 && hseq != 0 &&
                     (int32_t)(hseq - r->layout_seq) >= 0;
  if (hook > 0 ? !r->direct_veto : known) {
    fp.bin_direct = 1;
    fp.big_separate = 0;  // (the blend's workgroups radix-sort a list > kSortLdsCap themselves)
  }
}

int enqueue_frame(gs_renderer* r) {
  // several frames may be in flight on the stream; the host mirrors always
  // hold the last one's counters after gs_sync
  gsk::FrameParams fp = make_params(r);
  if (r->d_probe) fp.probe_frame = r->probe_n++;
  {  // the frame's number, and the first of its view (choose_direct)
    fp.frame_seq = r->seq_next++;
    if (r->seq_next == 0) r->seq_next = 1;
    float key[40] = {0};
    std::memcpy(key, r->view_rm, 16 * sizeof(float));
    std::memcpy(key + 16, r->proj_rm, 16 * sizeof(float));
    key[32] = r->fov;
    key[33] = r->scale_div;
    const int32_t bk[4] = {r->band_ty0, r->band_nrows, r->band_stride, r->n_tiles};
    std::memcpy(key + 34, bk, sizeof(bk));
    if (!r->cam_key_set || std::memcmp(key, r->cam_key, sizeof(key)) != 0) {
      std::memcpy(r->cam_key, key, sizeof(key));
      r->cam_key_set = true;
      r->cam_first_seq = fp.frame_seq;
    }
    choose_direct(r, fp);
    if (!fp.bin_direct) {  // (this frame's scan lays out the pair buffer)
      r->layout_seq = fp.frame_seq;
      r->direct_veto = false;
    }
  }
  r->last_fp = fp;
  r->have_fp = true;
  r->band_moved = false;
  // this frame's band (gs_set_band_rows may have moved it since the last one)
  r->stats.n_tiles = (uint32_t)r->n_tiles;
  r->stats.tiles_y = (uint32_t)r->band_nrows;
  r->stats.band_stride = (uint32_t)r->band_stride;
  r->stats.band_y0 = (uint32_t)r->band_py0;
  r->stats.band_rows = (uint32_t)r->band_rows;
  hipStream_t s = r->stream;
  // BGR8 destination of this frame (gs_set_bgr8_target)
  r->buf.bgr = r->bgr_target ? r->bgr_target : r->own_bgr;
  r->last_bgr = r->buf.bgr;
  ProfileSlot* slot = nullptr;
  if (r->profile && r->frame_seq++ % r->profile_every == 0) {
    slot = &r->ring[r->ring_head];
    r->ring_head = (r->ring_head + 1) % kProfileRing;
    int rc = profile_harvest(r, *slot);
    if (rc != GS_OK) return rc;
  }
  if (r->lattice) return enqueue_lattice(r, fp, slot);
  // counters + tile_count: the chunked path rewrites all of them (colscan,
  // scan); the global-atomic path accumulates tile_count and needs zeros
  if (r->bin_global || r->n_chunks == 0 || r->n_tiles == 0)
    GS_HIP(hipMemsetAsync(r->d_zero, 0, r->zero_bytes, s));
  if (int rc = ensure_cov(r, fp, s); rc != GS_OK) return rc;
  if (slot) GS_HIP(hipEventRecord(slot->ev[0], s));
  gsk::launch_project(fp, r->buf, s);
  if (slot) GS_HIP(hipEventRecord(slot->ev[1], s));
  // (GS_X_BAND == 5, measurement builds only, wrong frames: a band renderer
  // launches the aggregated scan and emit for its first 4 frames only; later
  // frames blend those lists again -- what the two launches cost the chain)
  const bool x_skip = GS_X_BAND == 5 && fp.bin_agg && fp.band_cull && ++r->x_frames > 4;
  if (!x_skip) gsk::launch_scan(fp, r->buf, s);
  if (slot) GS_HIP(hipEventRecord(slot->ev[2], s));
  if (!x_skip) gsk::launch_emit(fp, r->buf, s);
  if (slot) GS_HIP(hipEventRecord(slot->ev[3], s));
  gsk::launch_sort(fp, r->buf, s);
  if (slot) GS_HIP(hipEventRecord(slot->ev[4], s));
  gsk::FrameParams fb = fp;
  fb.count_records = (slot && r->buf.blend_count) ? 1 : 0;  // profiled frames count the blend's records
  r->last_counted = fb.count_records != 0;
  gsk::launch_blend(fb, r->buf, s);
  if (slot) GS_HIP(hipEventRecord(slot->ev[5], s));
  gsk::launch_blend_cont(fb, r->buf, s);
  if (slot) {
    GS_HIP(hipEventRecord(slot->ev[6], s));
    slot->pending = true;
  }
  GS_HIP(hipGetLastError());
  // the chunked scan writes the counters and list lengths into the mapped host
  // mirror itself; the other paths copy them (adjacent: one small D2H copy)
  if (r->bin_global || r->n_chunks == 0 || r->n_tiles == 0) {
    GS_HIP(hipMemcpyAsync(r->h_counters, r->d_zero, (16 + (size_t)r->n_tiles) * 4,
                          hipMemcpyDeviceToHost, s));
    // (the chunked scan writes the group footer itself)
    if (r->buf.footer)
      GS_HIP(hipMemcpyAsync(r->buf.footer, r->d_zero, (16 + (size_t)r->n_tiles) * 4,
                            hipMemcpyDeviceToDevice, s));
  }
  r->frame_pending = true;
  return GS_OK;
}

// gs_frame_stats.paths of the renderer's last enqueued frame
uint32_t frame_paths(const gs_renderer* r) {
  if (!r->have_fp) return 0u;
  const int kind = gsk::project_kind(r->last_fp, r->buf);
  return (r->last_fp.bin_agg ? GS_PATH_BIN_AGG : 0u) | (r->last_fp.blend_sort ? GS_PATH_BLEND_SORT : 0u) |
         (r->last_fp.blend_px2 ? GS_PATH_BLEND_PX2 : 0u) | (r->last_fp.lazy ? GS_PATH_LAZY : 0u) |
         (r->last_fp.big_separate ? GS_PATH_BIG_LISTS : 0u) | (kind == 2 ? GS_PATH_PROJ_BAND : 0u) |
         (kind == 0 ? GS_PATH_PROJ_ANY : 0u) | (kind == 3 ? GS_PATH_BIN_DIRECT : 0u);
}

int finish_frame(gs_renderer* r) {
  if (!r->frame_pending) return GS_OK;
  GS_HIP(hipStreamSynchronize(r->stream));
  r->frame_pending = false;
  const int nt0 = r->have_fp ? r->last_fp.n_tiles : r->n_tiles;
  // the aggregated binning keeps the frame's histogram on the device (a
  // per-frame copy into mapped memory from one workgroup cost the scan more
  // than the rest of its work): one copy here, at sync.  A group member's
  // histogram travels in its footer instead.
  if (r->have_fp && r->last_fp.bin_agg && !r->buf.footer && nt0 > 0)
    GS_HIP(hipMemcpy(r->h_counters + 16, r->buf.tile_ref, (size_t)nt0 * 4, hipMemcpyDeviceToHost));
  const uint32_t* c = r->h_counters;
  const uint64_t P = (uint64_t)c[5] | ((uint64_t)c[6] << 32);
  // the chunked scan also sums the reference (unculled) list lengths
  const bool chunked = !r->bin_global && r->n_chunks > 0 && r->n_tiles > 0;
  const uint64_t P_ref = chunked ? ((uint64_t)c[10] | ((uint64_t)c[11] << 32)) : P;
  r->stats.n_gaussians = r->n;
  r->stats.n_rendered = c[2];
  r->stats.n_pairs = P_ref;
  r->stats.n_pairs_binned = P;
  // the longest reference list (the binned lists can be shorter), over the
  // tiles of the frame (its band, even if the band has moved since)
  const int nt = r->have_fp ? r->last_fp.n_tiles : r->n_tiles;
  uint32_t mx = 0;
  for (int t = 0; t < nt; ++t) mx = std::max(mx, c[16 + t]);
  r->stats.max_list = mx;
  r->stats.pair_capacity = r->pair_cap;
  r->stats.n_big_tiles = c[0];
  r->stats.paths = frame_paths(r);
  r->stats.blend_records = r->stats.blend_cont_records = r->stats.cont_keys = 0;
  r->stats.cont_lists = r->stats.cont_max = r->stats.prefix_overflows = r->stats.cont_full_sorts = 0;
  r->stats.big_pairs = r->stats.big_prefix_keys = r->stats.big_window_keys = 0;
  if (r->last_counted && r->bcount_words) {
    // profiled frame: the list records the blend read.  The waves of a tile
    // each stage a prefix of the same list (the tile's records come from HBM
    // once, the other waves' reads hit L2), so a tile counts its longest prefix.
    // (the frame's tiles: the band may have moved since it was enqueued)
    const int nt_f = r->last_fp.n_tiles;
    const size_t cpt = (size_t)r->last_fp.chunks_per_tile;
    const size_t nw = std::min(r->bcount_words / 2, (size_t)nt_f * cpt);
    std::vector<uint32_t> bc(2 * nw);
    GS_HIP(hipMemcpy(bc.data(), r->buf.blend_count, nw * 4, hipMemcpyDeviceToHost));
    GS_HIP(hipMemcpy(bc.data() + nw, r->buf.blend_count + r->bcount_words / 2, nw * 4, hipMemcpyDeviceToHost));
    for (size_t t = 0; t + cpt <= nw; t += cpt) {
      uint32_t m0 = 0, m1 = 0;
      for (size_t k = t; k < t + cpt; ++k) {
        m0 = std::max(m0, bc[k]);
        m1 = std::max(m1, bc[nw + k]);
      }
      r->stats.blend_records += m0;
      // (the continuation ran the waves of the c[0] big lists only)
      if (r->last_fp.lazy && t < (size_t)c[0] * cpt) r->stats.blend_cont_records += m1;
    }
    if (c[0] > 0 && nt_f > 0) {
      // the big lists' binned pairs (bench.py's sort bytes)
      std::vector<uint32_t> ts((size_t)nt_f + 1), bt(c[0]);
      GS_HIP(hipMemcpy(ts.data(), r->buf.tile_start, ts.size() * 4, hipMemcpyDeviceToHost));
      GS_HIP(hipMemcpy(bt.data(), r->buf.big_tiles, (size_t)c[0] * 4, hipMemcpyDeviceToHost));
      for (uint32_t j = 0; j < c[0]; ++j)
        if (bt[j] < (uint32_t)nt_f) r->stats.big_pairs += ts[bt[j] + 1] - ts[bt[j]];
    }
    if (r->last_fp.lazy && c[0] > 0) {
      // the continuation's lists and their filtered key counts
      std::vector<uint32_t> fl(c[0]), cl(c[0]), bl(c[0]), f2(c[0]), w2(c[0]);
      GS_HIP(hipMemcpy(w2.data(), r->buf.big_cnt2, (size_t)c[0] * 4, hipMemcpyDeviceToHost));
      GS_HIP(hipMemcpy(fl.data(), r->buf.big_flag, (size_t)c[0] * 4, hipMemcpyDeviceToHost));
      GS_HIP(hipMemcpy(f2.data(), r->buf.big_flag2, (size_t)c[0] * 4, hipMemcpyDeviceToHost));
      GS_HIP(hipMemcpy(cl.data(), r->buf.cont_len, (size_t)c[0] * 4, hipMemcpyDeviceToHost));
      GS_HIP(hipMemcpy(bl.data(), r->buf.big_len, (size_t)c[0] * 4, hipMemcpyDeviceToHost));
      for (uint32_t j = 0; j < c[0]; ++j) {
        r->stats.big_prefix_keys += bl[j];
        r->stats.big_window_keys += w2[j];
      }
      for (uint32_t j = 0; j < c[0]; ++j)
        if (fl[j]) {
          r->stats.prefix_overflows += bl[j] == 0u ? 1u : 0u;
          r->stats.cont_full_sorts += f2[j] != 0u ? 1u : 0u;
          r->stats.cont_lists += 1;
          r->stats.cont_keys += cl[j];
          r->stats.cont_max = std::max(r->stats.cont_max, cl[j]);
        }
    }
  }
  // the scan of EVERY frame ORs its overflow into the sticky word (several
  // frames may have run since the last sync; counters[3] is only the last one's)
  volatile uint32_t* sticky = r->h_counters + 16 + r->t_cap;
  const bool ovf = c[3] != 0 || *sticky != 0;
  *sticky = 0;
  if (ovf) {
    r->layout_seq = 0;  // (the next frame takes the scan: choose_direct)
    r->direct_veto = true;
    set_error("pair list overflow: a frame since the last sync binned more pairs than the capacity " +
              std::to_string(r->pair_cap) + " (last frame: " + std::to_string(P) + " pairs)");
    return GS_EOVERFLOW;
  }
  {
    std::lock_guard<std::mutex> lk(r->hist_mu);
    r->hist_snapshot.assign(r->h_counters + 16, r->h_counters + 16 + nt);
    r->hist_moved = r->band_moved;  // (a frame enqueued before a move: still refused, as the frame readbacks)
  }
  r->have_frame = true;
  return GS_OK;
}

// GS_FLAG_LATTICE: the emulator's device state, with the reference's initial
// distribution of the records over the tiles: calculateMapping /
// applyTileMapping of the 64-float records (ipu_rasteriser.cpp:164-214,
// 287-298) put record j on tile j / gpt, gpt = ceil(64 n / (tiles * 64)) in
// float; every tile has gpt + 600 vertsIn slots (:307-309, 361-363), the last
// one also the rem records past fullTiles * gpt.  Never-written memory
// (padding, extra storage, channels, z-buffers) starts as zeros.
int lattice_init(gs_renderer* r, const gs_gaussian3d* g, size_t n) {
  const int T = r->tiles_x * r->tiles_y;
  const float q = (float)((uint64_t)n * 64u) / ((float)T * 64.0f);
  const int64_t gpt = (int64_t)std::ceil(q);
  const int64_t rem = (int64_t)n - ((int64_t)n / gpt) * gpt;
  if (gpt + rem + gsk::kLatExtra > gsk::kLatMaxSlots) {
    set_error("gs_create: lattice mode holds at most " + std::to_string(gsk::kLatMaxSlots) +
              " vertsIn slots per tile (" + std::to_string(gpt) + " records per tile + 600)");
    return GS_EINVAL;
  }
  const size_t slots = (size_t)T * (size_t)(gpt + gsk::kLatExtra) + (size_t)rem;
  const size_t chan = (size_t)2 * T * 4 * gsk::kLatChan * 4;  // float4
  const size_t bytes = slots * 64 + chan * 16 + slots * 48 * 2 + (size_t)T * 4 * 5;
  GS_HIP(hipMalloc(&r->d_lat, bytes));
  GS_HIP(hipMemset(r->d_lat, 0, bytes));
  char* p = (char*)r->d_lat;
  r->lat.slots = (float4*)p;
  p += slots * 64;
  r->lat.chan = (float4*)p;
  p += chan * 16;
  r->lat.zbuf = (float4*)p;
  p += slots * 48;
  r->lat.zscratch = (float4*)p;
  p += slots * 48;
  r->lat.splatted = (uint32_t*)p;
  r->lat.tile_stat = r->lat.splatted + T;
  std::vector<float> img(slots * 16, 0.0f);
  for (size_t j = 0; j < n; ++j) {
    const size_t t = j / (size_t)gpt;
    std::memcpy(&img[(t * (size_t)(gpt + gsk::kLatExtra) + (j - t * (size_t)gpt)) * 16], &g[j], 64);
  }
  GS_HIP(hipMemcpy(r->lat.slots, img.data(), slots * 64, hipMemcpyHostToDevice));
  r->lat_gpt = (int)gpt;
  r->lat_rem = (int)rem;
  r->lat_slots = slots;
  r->lattice = true;
  return GS_OK;
}

int create(const gs_gaussian3d* g, size_t n, const gs_config* cfg, const gs_renderer* share,
           gs_renderer** out) {
  if (!out || !cfg || (n > 0 && !g)) {
    set_error("gs_create: null argument");
    return GS_EINVAL;
  }
  *out = nullptr;
  if (cfg->width == 0 || cfg->height == 0 || cfg->tile_width == 0 || cfg->tile_height == 0 ||
      cfg->width > 65535 * 16 || cfg->tile_width * cfg->tile_height > (1u << 20) ||
      cfg->band_count == 0 || cfg->band_index >= cfg->band_count || n >= 0x7FFFFFFFull) {
    set_error("gs_create: invalid configuration");
    return GS_EINVAL;
  }
  const bool lattice = (cfg->flags & GS_FLAG_LATTICE) != 0;
  if (lattice && (cfg->width % cfg->tile_width || cfg->height % cfg->tile_height || cfg->band_count != 1 ||
                  cfg->band_row_end > cfg->band_row_begin || (cfg->flags & GS_FLAG_BAND_INTERLEAVED) || n == 0 ||
                  n >= (1u << 24))) {
    set_error("gs_create: GS_FLAG_LATTICE needs a whole tile grid (width % tile_width == 0, height % "
              "tile_height == 0), one band and 1 <= n < 2^24");
    return GS_EINVAL;
  }
  gs_renderer* r = new gs_renderer();
  r->cfg = *cfg;
  if (lattice) {  // the guard band of the lattice is the tile's own diagonal (codelets.cpp:470)
    r->cfg.guard_tile_width = 0;
    r->cfg.guard_tile_height = 0;
  }
  r->n = n;
  r->profile = (cfg->flags & GS_FLAG_PROFILE) != 0;
  r->pair_cull = (cfg->flags & GS_FLAG_NO_PAIR_CULL) == 0;
  int dev = cfg->device;
  if (dev < 0) {
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) {
      delete r;
      return hip_fail(e, "hipGetDevice");
    }
  }
  r->device = dev;
  auto fail = [&](int rc) {
    release(r);
    delete r;
    return rc;
  };
  if (hipSetDevice(dev) != hipSuccess) return fail(hip_fail(hipSetDevice(dev), "hipSetDevice"));
  // identity camera until set
  for (int i = 0; i < 16; ++i) r->view_rm[i] = r->proj_rm[i] = (i % 5 == 0) ? 1.0f : 0.0f;

  // tile grid (ceil: partial tiles are masked) and the row band
  r->tiles_x = (int)((cfg->width + cfg->tile_width - 1) / cfg->tile_width);
  r->tiles_y = (int)((cfg->height + cfg->tile_height - 1) / cfg->tile_height);
  if (r->tiles_x > 65535 || r->tiles_y > 65535) {
    set_error("gs_create: tile grid too large");
    return fail(GS_EINVAL);
  }
  int rpb = (r->tiles_y + (int)cfg->band_count - 1) / (int)cfg->band_count;
  const int th_px = (int)cfg->tile_height;
  const bool explicit_band = cfg->band_row_end > cfg->band_row_begin;
  if (explicit_band && (cfg->band_row_end > (uint32_t)r->tiles_y || (cfg->flags & GS_FLAG_BAND_INTERLEAVED))) {
    set_error("gs_create: explicit band rows outside the tile grid (or combined with interleaving)");
    return fail(GS_EINVAL);
  }
  if (explicit_band) {
    // caller-chosen contiguous band (work-balanced row split)
    r->band_ty0 = (int)cfg->band_row_begin;
    r->band_stride = 1;
    r->band_nrows = (int)(cfg->band_row_end - cfg->band_row_begin);
    r->band_py0 = r->band_ty0 * th_px;
    r->band_rows = std::max(0, std::min((int)cfg->height, (int)cfg->band_row_end * th_px) - r->band_py0);
    rpb = std::max(r->band_nrows, (int)cfg->band_pad_rows);
  } else if (cfg->flags & GS_FLAG_BAND_INTERLEAVED) {
    // rows band_index, band_index + band_count, ...; output = those tile rows
    // back to back (whole tiles; rows past the image stay 0)
    const int bc = (int)cfg->band_count, bi = (int)cfg->band_index;
    r->band_ty0 = std::min(r->tiles_y, bi);
    r->band_stride = bc;
    r->band_nrows = r->tiles_y > bi ? (r->tiles_y - bi + bc - 1) / bc : 0;
    r->band_py0 = r->band_ty0 * th_px;
    r->band_rows = r->band_nrows * th_px;
  } else {
    r->band_ty0 = std::min(r->tiles_y, (int)cfg->band_index * rpb);
    const int ty1 = std::min(r->tiles_y, r->band_ty0 + rpb);
    r->band_stride = 1;
    r->band_nrows = ty1 - r->band_ty0;
    r->band_py0 = r->band_ty0 * th_px;
    r->band_rows = std::max(0, std::min((int)cfg->height, ty1 * th_px) - r->band_py0);
  }
  r->band_rows_padded = rpb * th_px;
  r->rows_cap = rpb;
  r->n_tiles = r->tiles_x * r->band_nrows;
  r->t_cap = r->n_tiles;
  r->stats.n_tiles = (uint32_t)r->n_tiles;
  r->stats.tiles_x = (uint32_t)r->tiles_x;
  r->stats.tiles_y = (uint32_t)r->band_nrows;
  r->stats.band_stride = (uint32_t)r->band_stride;
  r->stats.band_y0 = (uint32_t)r->band_py0;
  r->stats.band_rows = (uint32_t)r->band_rows;

  hipError_t e;
  if ((e = hipStreamCreateWithFlags(&r->own_stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(hip_fail(e, "hipStreamCreate"));
  r->stream = r->own_stream;

  // scene: SoA of the 64-B records, in device order (3D Morton order of the
  // means unless GS_FLAG_INPUT_ORDER), plus the permutation both ways.  A
  // renderer of a group shares the first one's copy on the same device.
  const size_t nn = std::max<size_t>(n, 1);
  if (share && share->device == dev && share->n == n && share->d_scene) {
    r->perm = share->perm;
    r->d_scene = share->d_scene;
    r->owns_scene = false;
    r->scene_w1 = share->scene_w1;
  } else {
    r->perm = morton_order(g, n, (cfg->flags & GS_FLAG_INPUT_ORDER) != 0);
    if ((e = hipMalloc(&r->d_scene, scene_bytes(nn))) != hipSuccess)
      return fail(hip_fail(e, "hipMalloc(scene)"));
    {
      // staged in pinned host memory (one DMA at full PCIe rate)
      float* soa = nullptr;
      if ((e = hipHostMalloc((void**)&soa, scene_bytes(nn), hipHostMallocDefault)) != hipSuccess)
        return fail(hip_fail(e, "hipHostMalloc(scene staging)"));
      std::memset(soa, 0, scene_bytes(nn));
      uint32_t* pi = (uint32_t*)(soa + nn * 16);
      bool w1 = true;
      for (size_t i = 0; i < n; ++i) {
        const uint32_t o = r->perm[i];
        const float* s = reinterpret_cast<const float*>(&g[o]);
        for (int k = 0; k < 4; ++k) {
          soa[(0 * nn + i) * 4 + k] = s[0 + k];
          soa[(1 * nn + i) * 4 + k] = s[4 + k];
          soa[(2 * nn + i) * 4 + k] = s[8 + k];
          soa[(3 * nn + i) * 4 + k] = s[12 + k];
        }
        pi[i] = o;
        pi[nn + o] = (uint32_t)i;
        // the band cull's record: the mean and the largest log-scale -- all
        // band_culled_fast reads -- in 16 B instead of the mean's and the
        // scales' 32 (a mean with w != 1 is never culled: +inf; an empty slot
        // goes to the full path as before: NaN)
        float* cr = soa + cull_offset(nn) / 4 + 4 * i;
        cr[0] = s[0];
        cr[1] = s[1];
        cr[2] = s[2];
        cr[3] = (s[15] <= 0.0f) ? std::numeric_limits<float>::quiet_NaN()
                : (s[3] != 1.0f ? std::numeric_limits<float>::infinity()
                                : std::fmax(std::fmax(s[12], s[13]), s[14]));
        // the projection's 16-B read when every w is 1 (clip = mvp (xyz, 1))
        float* mo = soa + cull_offset(nn) / 4 + 4 * nn + 4 * i;
        mo[0] = s[0];
        mo[1] = s[1];
        mo[2] = s[2];
        mo[3] = s[7];  // opacity
        w1 = w1 && s[3] == 1.0f;
      }
      r->scene_w1 = w1;
      e = hipMemcpy(r->d_scene, soa, scene_bytes(nn), hipMemcpyHostToDevice);
      (void)hipHostFree(soa);
      if (e != hipSuccess) return fail(hip_fail(e, "hipMemcpy(scene)"));
    }
  }
  const float4* sc = (const float4*)r->d_scene;
  r->buf.mean = sc;
  r->buf.colour = sc + nn;
  r->buf.rot = sc + 2 * nn;
  r->buf.scale_gid = sc + 3 * nn;
  r->buf.perm = (const uint32_t*)(sc + 4 * nn);
  r->buf.cull = (const float4*)((const char*)r->d_scene + cull_offset(nn));
  r->buf.mean_op = r->buf.cull + nn;
  r->buf.inv_perm = r->buf.perm + nn;

  // per Gaussian: 48 B of record (frames: the 32-B record the blend reads and,
  // with gs_set_sh, the 16-B view-dependent colour; the readback: the 48-B
  // record), its 8-B readback tail, 8-B tile rectangle and its alpha-box cut
  // (rect8: 4 B each), 4-B depth key; plus V per project workgroup
  const size_t nblk = (nn + 255) / 256;
  if ((e = hipMalloc(&r->d_gauss, nn * (48 + 8 + 8 + 8 + 4) + nblk * 4)) != hipSuccess)
    return fail(hip_fail(e, "hipMalloc(per-Gaussian)"));
  poison(r->d_gauss, nn * (48 + 8 + 8 + 8 + 4) + nblk * 4, "gauss");
  r->buf.rec = (float4*)r->d_gauss;
  r->buf.rec_tail = (float2*)((char*)r->d_gauss + nn * 48);
  r->buf.col_out = (float4*)((char*)r->d_gauss + nn * 32);  // (frames: the record region past the 32-B records)
  r->buf.rect = (uint2*)((char*)r->d_gauss + nn * 56);
  r->buf.crect = (uint2*)((char*)r->d_gauss + nn * 64);
  r->buf.depth_key = (uint32_t*)((char*)r->d_gauss + nn * 72);
  r->buf.block_rendered = (uint32_t*)((char*)r->d_gauss + nn * 76);
  // the 3D covariance cache: 9 float planes (SoA), 36 B per Gaussian; an empty
  // slot is marked by a negative Sigma[2][2] (gs_cov3d_kernel).  An
  // optimisation only: the lattice emulator never reads it, and when the
  // allocation fails the projection keeps computing the covariances from the
  // rotation and the scales (cov_cache = 0) instead of refusing the scene.
  // (test hook: gs_test_set("cov_cache", 0) takes the fallback)
  if (!lattice && g_test_cov_cache.load() != 0) {
    if ((e = hipMalloc(&r->d_cov, nn * 36)) == hipSuccess) {
      poison(r->d_cov, nn * 36, "cov");
      r->buf.cov3 = (float*)r->d_cov;
    } else {
      (void)hipGetLastError();  // (clear the sticky error of the failed allocation)
      r->d_cov = nullptr;
      r->buf.cov3 = nullptr;
    }
  }

  const size_t T = (size_t)std::max(r->n_tiles, 1);
  r->zero_bytes = ((16 + T) * 4 + 15) / 16 * 16;
  if ((e = hipMalloc(&r->d_zero, r->zero_bytes)) != hipSuccess) return fail(hip_fail(e, "hipMalloc(zero)"));
  poison(r->d_zero, r->zero_bytes, "zero");
  r->buf.counters = (uint32_t*)r->d_zero;
  r->buf.tile_count = (uint32_t*)r->d_zero + 16;
  const size_t n_agg = (T + 63) / 64;
  const size_t tiles_bytes = (T + 1 + 4 * T) * 4 + n_agg * 32 + 16 + T * 8 + 8 + T * 4 + T * 4 + 16 + T * 16;
  if ((e = hipMalloc(&r->d_tiles, tiles_bytes)) != hipSuccess) return fail(hip_fail(e, "hipMalloc(tiles)"));
  poison(r->d_tiles, tiles_bytes, "tiles");
  r->buf.tile_start = (uint32_t*)r->d_tiles;
  // (an empty layout until a scan writes one: a forced direct frame before
  // any scan drops every pair and reports the overflow)
  if ((e = hipMemset(r->buf.tile_start, 0, (T + 1) * 4)) != hipSuccess) return fail(hip_fail(e, "hipMemset(tiles)"));
  r->buf.tile_cursor = r->buf.tile_start + T + 1;
  r->buf.big_tiles = r->buf.tile_cursor + T;
  r->buf.medium_tiles = r->buf.big_tiles + T;
  r->buf.small_tiles = r->buf.medium_tiles + T;
  r->buf.tile_agg = (uint4*)(((uintptr_t)(r->buf.small_tiles + T) + 15) & ~(uintptr_t)15);
  // the aggregated binning's per-tile counters: zero between frames (the
  // scan resets them)
  r->buf.tile_cnt64 = (unsigned long long*)(((uintptr_t)(r->buf.tile_agg + 2 * n_agg) + 7) & ~(uintptr_t)7);
  r->buf.tile_ref = (uint32_t*)(r->buf.tile_cnt64 + T);
  r->buf.tile_fb = r->buf.tile_ref + T;
  r->buf.blend_seg = (uint4*)(((uintptr_t)(r->buf.tile_fb + T) + 15) & ~(uintptr_t)15);
  if ((e = hipMemset(r->d_tiles, 0, (T + 1 + 4 * T) * 4)) != hipSuccess)
    return fail(hip_fail(e, "hipMemset(tiles)"));
  if ((e = hipMemset(r->buf.tile_cnt64, 0, T * 8)) != hipSuccess) return fail(hip_fail(e, "hipMemset(tile counters)"));
  if ((e = hipMemset(r->buf.tile_fb, 0, T * 4)) != hipSuccess) return fail(hip_fail(e, "hipMemset(tile counters)"));

  // binning mode: chunked LDS histograms unless the band's tile grid is too
  // large for one CU's LDS (or the caller asks for the global-atomic path)
  r->bin_global = ((cfg->flags & GS_FLAG_BIN_GLOBAL) || !gsk::bin_lds_fits(r->n_tiles)) ? 1 : 0;
  if (!r->bin_global && n > 0 && r->n_tiles > 0) {
    size_t cs = std::max<size_t>(4096, (n + 255) / 256);
    cs = std::min<size_t>(cs, 65535);
    // chunks of <= 65535 Gaussians (16-bit LDS counters): scenes beyond
    // ~16.7 M take more than 256 chunks, which gs_colscan_kernel handles with a
    // second read of the extra rows.  Test hook (gs_test_set): the chunk
    // size, to reach many chunks at a small N.
    const int64_t fixed_cs = g_test_chunk_size.load();
    if (fixed_cs > 0) cs = (size_t)std::max<int64_t>(64, std::min<int64_t>(65535, fixed_cs));
    {
      if ((e = gsk::init_kernel_attributes()) != hipSuccess) return fail(hip_fail(e, "hipFuncSetAttribute"));
      r->chunk_size = (int)cs;
      r->n_chunks = (int)((n + cs - 1) / cs);
      // the chunk table holds the whole frame's chunks x tiles: a band (fewer
      // tiles) cuts the scene into proportionally more, smaller chunks
      // (make_params), so the densest chunk -- the binning's critical path --
      // shrinks with the band instead of staying a whole-frame chunk
      r->chunk_entries = (size_t)r->n_chunks * (size_t)std::max(r->n_tiles, r->tiles_x * r->tiles_y);
      r->chunk_adaptive = fixed_cs <= 0;
      // the aggregated binning for grids of up to kAggMaxTiles tiles (frames
      // at 1080p, any row band of a 4K frame split over >= 2 GPUs), the
      // chunked count / column scan / emit beyond (config 5's 4K frame on one
      // GPU: its clustered workgroups fill few tiles, whose LDS atomics cost
      // the projection more than the chunked passes take).  Test hook
      // (gs_test_set "bin_agg" 0): row bands bin with the chunked passes too.
      r->bin_agg = g_test_bin_agg.load() != 0 && fixed_cs <= 0;
      if (r->bin_agg) {  // per projection block: its tile box and its offsets in each tile
        const size_t nb = (nn + 255) / 256;
        const size_t agg_bytes = nb * 16 + nb * (size_t)gsk::kAggCap * 4;
        if ((e = hipMalloc(&r->d_agg, agg_bytes)) != hipSuccess) return fail(hip_fail(e, "hipMalloc(agg boxes)"));
        poison(r->d_agg, agg_bytes, "agg");
        r->buf.agg_box = (uint4*)r->d_agg;
        r->buf.agg_off = (uint32_t*)((char*)r->d_agg + nb * 16);
        // the direct binning's ticket and overflow words (zero between frames)
        if ((e = hipMalloc(&r->d_dir, 16)) != hipSuccess) return fail(hip_fail(e, "hipMalloc(direct words)"));
        if ((e = hipMemset(r->d_dir, 0, 16)) != hipSuccess) return fail(hip_fail(e, "hipMemset(direct words)"));
        r->buf.dir_word = (uint32_t*)r->d_dir;
      }
      if ((e = hipMalloc(&r->d_chunk, r->chunk_entries * 4)) != hipSuccess)
        return fail(hip_fail(e, "hipMalloc(chunk offsets)"));
      poison(r->d_chunk, r->chunk_entries * 4, "chunk");
      r->buf.chunk_off = (uint32_t*)r->d_chunk;
    }
  }
  r->stats.bin_global = (uint32_t)r->bin_global;

  // lazy big lists (gs_kernels.hip, kLazyPrefix): with the chunked binning
  // and 16x16 tiles (four 8x8 blend waves per tile); per tile 9 u32 + the
  // saved state of 4 waves (6 x 64 floats each) + their boxes + 6 u32
  if (!r->bin_global && r->n_chunks > 0 && cfg->tile_width == 16 && cfg->tile_height == 16) {
    const size_t TT = (size_t)r->t_cap;
    const size_t lazy_bytes = TT * (9 * 4 + 4 * 6 * 64 * 4 + 4 * 8 + 4 + 5 * 4) + 8;
    if ((e = hipMalloc(&r->d_lazy, lazy_bytes)) != hipSuccess)
      return fail(hip_fail(e, "hipMalloc(lazy big lists)"));
    poison(r->d_lazy, lazy_bytes, "lazy");
    uint32_t* u = (uint32_t*)r->d_lazy;
    r->buf.tile_big = u;
    r->buf.big_len = u + TT;
    r->buf.big_thr = u + 2 * TT;
    r->buf.big_cnt = u + 3 * TT;
    r->buf.big_flag = u + 4 * TT;
    r->buf.cont_flag = u + 5 * TT;  // 4 per slot: [5 T, 9 T)
    r->buf.cont_state = (float*)(u + 9 * TT);
    r->buf.cont_box = (uint2*)(((uintptr_t)(r->buf.cont_state + TT * 4 * 6 * 64) + 7) & ~(uintptr_t)7);
    r->buf.cont_len = (uint32_t*)(r->buf.cont_box + TT * 4);
    r->buf.big_thr2 = r->buf.cont_len + TT;
    r->buf.big_cnt2 = r->buf.cont_len + 2 * TT;
    r->buf.big_flag2 = r->buf.cont_len + 3 * TT;
    r->buf.cont_full = r->buf.cont_len + 4 * TT;
    r->buf.cont_thr = r->buf.cont_len + 5 * TT;
    if ((e = hipMemset(r->d_lazy, 0, TT * 9 * 4)) != hipSuccess) return fail(hip_fail(e, "hipMemset(lazy)"));
  }

  uint64_t cap = cfg->pair_capacity;
  if (cap == 0) cap = std::max<uint64_t>(1u << 20, 8ull * n);
  cap = std::min<uint64_t>(cap, 0xFFFFFFF0ull);
  int rc = alloc_pairs(r, cap);
  if (rc != GS_OK) return fail(rc);

  const size_t px = (size_t)cfg->width * std::max(r->band_rows_padded, 1);
  r->bgr_bytes = px * 3;
  if ((e = hipMalloc(&r->d_out, px * 16 + (r->bgr_bytes + 15) / 16 * 16)) != hipSuccess)
    return fail(hip_fail(e, "hipMalloc(framebuffer)"));
  poison(r->d_out, px * 16 + (r->bgr_bytes + 15) / 16 * 16, "out");
  r->buf.rgba = (float4*)r->d_out;
  r->buf.bgr = (uint8_t*)r->d_out + px * 16;
  r->own_bgr = r->last_bgr = r->buf.bgr;
  if ((e = hipMemset(r->d_out, 0, px * 16 + r->bgr_bytes)) != hipSuccess)
    return fail(hip_fail(e, "hipMemset(framebuffer)"));

  // + one sticky overflow word after the list lengths (h_counters[16 + T])
  if ((e = hipHostMalloc((void**)&r->h_counters, r->zero_bytes + 16,
                         hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return fail(hip_fail(e, "hipHostMalloc"));
  std::memset(r->h_counters, 0, r->zero_bytes + 16);
  if ((e = hipHostGetDevicePointer((void**)&r->buf.host_counters, r->h_counters, 0)) != hipSuccess)
    return fail(hip_fail(e, "hipHostGetDevicePointer"));
  r->buf.host_sticky = r->buf.host_counters + 16 + T;
  r->hist_snapshot.assign((size_t)r->n_tiles, 0u);
  if (lattice) {
    const int rc2 = lattice_init(r, g, n);
    if (rc2 != GS_OK) return fail(rc2);
  }
  if (r->profile && !lattice) {
    // the blend's staged-record counts of profiled frames: one word per blend
    // wave of the prefix pass, one per wave of the continuation
    const uint32_t tw = cfg->tile_width, th = cfg->tile_height;
    const size_t cpt = (tw % 8 == 0 && th % 8 == 0)    ? (size_t)(tw / 8) * (th / 8)
                       : (tw % 16 == 0 && th % 4 == 0) ? (size_t)(tw / 16) * (th / 4)
                                                       : (size_t)((((tw + 1) / 2) * ((th + 1) / 2) + 15) / 16);
    r->bcount_words = 2 * (size_t)r->t_cap * cpt;
    if ((e = hipMalloc(&r->d_bcount, r->bcount_words * 4)) != hipSuccess)
      return fail(hip_fail(e, "hipMalloc(blend counts)"));
    if ((e = hipMemset(r->d_bcount, 0, r->bcount_words * 4)) != hipSuccess)
      return fail(hip_fail(e, "hipMemset(blend counts)"));
    r->buf.blend_count = (uint32_t*)r->d_bcount;
    r->buf.blend_count_cont = r->buf.blend_count + r->bcount_words / 2;
  }
  if (r->profile) {
    for (auto& s : r->ring)
      for (auto& ev : s.ev)
        if ((e = hipEventCreate(&ev)) != hipSuccess) return fail(hip_fail(e, "hipEventCreate"));
  }
  if (GS_PROBE && std::getenv("GSPLAT_PROBE_FILE") && !lattice) {
    // the probe ring: starts at ~0 (atomicMin), ends at 0 (atomicMax)
    std::vector<unsigned long long> init((size_t)gsk::kProbeFrames * gsk::kProbeKernels * gsk::kProbeSlots * 2);
    for (size_t k = 0; k < init.size(); k += 2) init[k] = ~0ull;
    if ((e = hipMalloc(&r->d_probe, init.size() * 8)) != hipSuccess) return fail(hip_fail(e, "hipMalloc(probe)"));
    if ((e = hipMemcpy(r->d_probe, init.data(), init.size() * 8, hipMemcpyHostToDevice)) != hipSuccess)
      return fail(hip_fail(e, "hipMemcpy(probe)"));
    r->buf.probe = (unsigned long long*)r->d_probe;
  }
#if GS_LANES
  if (std::getenv("GSPLAT_LANES_FILE") && !lattice) {
    if ((e = hipMalloc(&r->buf.lanes, 64)) != hipSuccess) return fail(hip_fail(e, "hipMalloc(lanes)"));
    if ((e = hipMemset(r->buf.lanes, 0, 64)) != hipSuccess) return fail(hip_fail(e, "hipMemset(lanes)"));
  }
#endif
  *out = r;
  return GS_OK;
}


void destroy(gs_renderer* r) {
  if (!r) return;
  release(r);
  delete r;
}

int set_band_rows(gs_renderer* r, int ty0, int ty1, int pad_rows) {
  if (ty0 < 0 || ty1 > r->tiles_y || ty1 <= ty0 || pad_rows < ty1 - ty0 || pad_rows > r->rows_cap ||
      (ty1 - ty0) * r->tiles_x > r->t_cap) {
    set_error("set_band_rows: band outside the renderer's tile rows");
    return GS_EINVAL;
  }
  const int th_px = (int)r->cfg.tile_height;
  r->band_ty0 = ty0;
  r->band_stride = 1;
  r->band_nrows = ty1 - ty0;
  r->band_py0 = ty0 * th_px;
  r->band_rows = std::max(0, std::min((int)r->cfg.height, ty1 * th_px) - r->band_py0);
  r->band_rows_padded = pad_rows * th_px;
  r->n_tiles = r->tiles_x * r->band_nrows;
  r->bgr_bytes = (size_t)r->cfg.width * r->band_rows_padded * 3;
  // (the stats keep the last frame's band until the next frame is enqueued)
  return GS_OK;
}

int grow_pairs(gs_renderer* r, bool force) {
  const uint64_t need = r->stats.n_pairs_binned + r->stats.n_pairs_binned / 4 + 1024;
  if (need > 0xFFFFFFF0ull) {
    set_error("gs_render: pair count exceeds 2^32");
    return GS_EOVERFLOW;
  }
  if (!force && r->pair_cap >= need) return GS_OK;
  const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>(need, 2 * r->pair_cap), 0xFFFFFFF0ull);
  GS_HIP(hipStreamSynchronize(r->stream));
  return alloc_pairs(r, cap);
}

int refuse_moved(const gs_renderer* r, const char* what) {
  if (!r->band_moved) return GS_OK;
  set_error(std::string(what) + ": the band moved (gs_set_band_rows) after the last frame; render a frame first");
  return GS_EINVAL;
}

int read_rgba32f(gs_renderer* r, float* dst, size_t n_floats, int layout) {
  if (refuse_moved(r, "gs_read_rgba32f") != GS_OK) return GS_EINVAL;
  if (r->cfg.flags & GS_FLAG_NO_RGBA32F) {
    set_error("gs_read_rgba32f: renderer created with GS_FLAG_NO_RGBA32F");
    return GS_EINVAL;
  }
  const size_t W = r->cfg.width;
  const size_t rows = (size_t)r->band_rows;
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  if ((rc = finish_frame(r)) != GS_OK) return rc;
  if (layout == GS_LAYOUT_ROW_MAJOR) {
    if (n_floats < rows * W * 4) {
      set_error("gs_read_rgba32f: destination too small");
      return GS_EINVAL;
    }
    GS_HIP(hipMemcpy(dst, r->buf.rgba, rows * W * 16, hipMemcpyDeviceToHost));
    return GS_OK;
  }
  if (layout != GS_LAYOUT_REF_TILE_MAJOR) return GS_EINVAL;
  const size_t tw = r->cfg.tile_width, th = r->cfg.tile_height;
  const size_t need = (size_t)r->n_tiles * tw * th * 4;
  if (n_floats < need) {
    set_error("gs_read_rgba32f: destination too small");
    return GS_EINVAL;
  }
  std::vector<float> rm(rows * W * 4);
  GS_HIP(hipMemcpy(rm.data(), r->buf.rgba, rm.size() * 4, hipMemcpyDeviceToHost));
  retile(rm.data(), rows, W, tw, th, r->tiles_x, r->n_tiles, dst);
  return GS_OK;
}

// the IPU layout (ipu_rasteriser.cpp:164-214 + codelets.cpp:174-176)
void retile(const float* rm, size_t rows, size_t W, size_t tw, size_t th, int tiles_x, int n_tiles,
            float* dst) {
  std::memset(dst, 0, (size_t)n_tiles * tw * th * 16);
  for (int t = 0; t < n_tiles; ++t) {
    const size_t tx = t % tiles_x, ty = t / tiles_x;
    for (size_t ly = 0; ly < th; ++ly) {
      const size_t y = ty * th + ly;
      if (y >= rows) break;
      for (size_t lx = 0; lx < tw; ++lx) {
        const size_t x = tx * tw + lx;
        if (x >= W) break;
        std::memcpy(dst + ((size_t)t * tw * th + lx + ly * tw) * 4, &rm[(y * W + x) * 4], 16);
      }
    }
  }
}

int read_bins(gs_renderer* r, uint64_t* tile_start, size_t n_start, uint32_t* list, size_t n_list) {
  if (r->lattice) {
    set_error("gs_read_bins: a lattice renderer has no converged tile lists (gs_read_lattice_slots)");
    return GS_EINVAL;
  }
  if (refuse_moved(r, "gs_read_bins") != GS_OK) return GS_EINVAL;
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  if ((rc = finish_frame(r)) != GS_OK) return rc;
  if (!r->have_frame || !r->have_fp) {
    set_error("gs_read_bins: no frame rendered yet");
    return GS_EINVAL;
  }
  const size_t T = (size_t)r->n_tiles;
  if (n_start < T + 1 || n_list < r->stats.n_pairs) {
    set_error("gs_read_bins: destination too small");
    return GS_EINVAL;
  }
  if (r->last_fp.pair_cull) {
    // The frame binned each Gaussian only into the tiles its alpha box meets.
    // Bin the reference lists of THAT frame again (its FrameParams, pair cull
    // off): project, scan, emit and sort only -- no blend, so the framebuffer,
    // the BGR8 target, the stats and the histogram snapshot are untouched.
    gsk::FrameParams fp = r->last_fp;
    fp.pair_cull = 0;
    fp.rect8 = 0;
    fp.blend_sort = 0;  // (no blend here: the sort launch sorts the lists)
    fp.bin_direct = 0;  // (the scan and emit place the reference lists)
    gsk::Buffers bb = r->buf;
    bb.footer = nullptr;        // (a group's all-gather slot belongs to the frame)
    bb.group_sticky = nullptr;  // (this re-binning's overflow is handled here, not by the group)
    for (int attempt = 0; attempt < 8; ++attempt) {
      fp.pair_cap = r->pair_cap;
      bb.pairs = r->buf.pairs;
      bb.pairs_alt = r->buf.pairs_alt;
      bb.list = r->buf.list;
      bb.big_item = r->buf.big_item;
      bb.bk_spl = r->buf.bk_spl;
      bb.bk_start = r->buf.bk_start;
      bb.bk_cnt = r->buf.bk_cnt;
      bb.bk_list = r->buf.bk_list;
      bb.bk_off = r->buf.bk_off;
      fp.big_separate = 0;  // the tile sort radix-sorts big lists itself
      fp.lazy = 0;
      if (r->bin_global || r->n_chunks == 0 || r->n_tiles == 0)
        GS_HIP(hipMemsetAsync(r->d_zero, 0, r->zero_bytes, r->stream));
      if ((rc = ensure_cov(r, fp, r->stream)) != GS_OK) return rc;
      gsk::launch_project(fp, bb, r->stream);
      gsk::launch_scan(fp, bb, r->stream);
      gsk::launch_emit(fp, bb, r->stream);
      gsk::launch_sort(fp, bb, r->stream);
      GS_HIP(hipGetLastError());
      if (r->bin_global || r->n_chunks == 0 || r->n_tiles == 0)
        GS_HIP(hipMemcpyAsync(r->h_counters, r->d_zero, (16 + T) * 4, hipMemcpyDeviceToHost, r->stream));
      GS_HIP(hipStreamSynchronize(r->stream));
      volatile uint32_t* sticky = r->h_counters + 16 + r->t_cap;
      *sticky = 0;
      const uint32_t* c = r->h_counters;
      const uint64_t P = (uint64_t)c[5] | ((uint64_t)c[6] << 32);
      if (!c[3]) break;
      const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>(P + P / 4 + 1024, 2 * r->pair_cap), 0xFFFFFFF0ull);
      if (P > 0xFFFFFFF0ull || attempt == 7) {
        set_error("gs_read_bins: reference lists exceed the pair capacity");
        return GS_EOVERFLOW;
      }
      if ((rc = alloc_pairs(r, cap)) != GS_OK) return rc;
    }
  }
  std::vector<uint32_t> ts(T + 1);
  GS_HIP(hipMemcpy(ts.data(), r->buf.tile_start, (T + 1) * 4, hipMemcpyDeviceToHost));
  for (size_t i = 0; i <= T; ++i) tile_start[i] = ts[i];
  if (r->stats.n_pairs) {
    GS_HIP(hipMemcpy(list, r->buf.list, r->stats.n_pairs * 4, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < r->stats.n_pairs; ++k)  // device -> input indices
      list[k] = list[k] < r->n ? r->perm[list[k]] : list[k];
  }
  return GS_OK;
}

int read_projected(gs_renderer* r, float* dst, size_t n_floats) {
  if (n_floats < r->n * 12) {
    set_error("gs_read_projected: destination too small");
    return GS_EINVAL;
  }
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  if ((rc = finish_frame(r)) != GS_OK) return rc;
  if (!r->have_fp) {
    set_error("gs_read_projected: no frame rendered yet");
    return GS_EINVAL;
  }
  std::vector<float> rec(r->n * 12), tail(r->n * 2);
  std::vector<uint32_t> rect(r->n * 2);
  if (r->n) {
    // project the last frame's camera again (its FrameParams) with the
    // readback tail of the record (radius, clip z), which frames skip, and
    // without the band cull (same values otherwise).  Only the per-Gaussian
    // scratch of the finished frame is rewritten.
    gsk::FrameParams fp = r->last_fp;
    fp.band_cull = 0;
    fp.bin_global = 0;  // (no tile_count atomics)
    fp.bin_agg = 0;     // (nor the aggregated binning's: this pass has no scan to reset them)
    fp.bin_direct = 0;
    fp.full_record = 1;
    fp.rect8 = 0;  // (the readback takes the 16-bit reference rectangle)
    fp.mean_w1 = 0;  // (and the 48-B record with the colour)
    if ((rc = ensure_cov(r, fp, r->stream)) != GS_OK) return rc;
    gsk::launch_project(fp, r->buf, r->stream);
    GS_HIP(hipGetLastError());
    GS_HIP(hipStreamSynchronize(r->stream));
    GS_HIP(hipMemcpy(rec.data(), r->buf.rec, r->n * 48, hipMemcpyDeviceToHost));
    GS_HIP(hipMemcpy(tail.data(), r->buf.rec_tail, r->n * 8, hipMemcpyDeviceToHost));
    GS_HIP(hipMemcpy(rect.data(), r->buf.rect, r->n * 8, hipMemcpyDeviceToHost));
  }
  for (size_t i = 0; i < r->n; ++i) {
    const float* q = &rec[i * 12];
    float* o = dst + (size_t)r->perm[i] * 12;  // in input order
    o[0] = q[0];  // mean2d
    o[1] = q[1];
    o[2] = q[2];  // conic (k0, k1, k2, opacity)
    o[3] = q[4];
    o[4] = q[3];
    o[5] = q[9];
    o[6] = tail[i * 2 + 1];  // clip z
    o[7] = tail[i * 2];      // radius
    const uint32_t rx = rect[i * 2], ry = rect[i * 2 + 1];
    o[8] = (float)(rx & 0xFFFF);
    o[9] = (float)(ry & 0xFFFF);
    o[10] = (float)(rx >> 16);
    o[11] = (float)(ry >> 16);
  }
  return GS_OK;
}

}  // namespace gsr

using namespace gsr;

extern "C" {

int gs_abi_version(void) { return GSPLAT_ABI_VERSION; }

int gs_test_set(const char* key, int64_t value) {
  if (!key) return GS_EINVAL;
  const std::string k(key);
  if (k == "bin_chunk_size" && value >= 0) {
    gsr::g_test_chunk_size.store(value);
  } else if (k == "bin_agg" && (value == -1 || value == 0)) {
    gsr::g_test_bin_agg.store(value);
  } else if (k == "debug_poison" && (value == 0 || value == 1)) {
    gsr::g_test_poison.store(value);
  } else if (k == "cov_cache" && (value == -1 || value == 0)) {
    gsr::g_test_cov_cache.store(value);
  } else if (k == "bin_direct" && (value == -1 || value == 0 || value == 1)) {
    gsr::g_test_bin_direct.store(value);  // -1: default; 0: off; 1: forced on until an overflow
  } else {
    gsh::set_error("gs_test_set: unknown key or value");
    return GS_EINVAL;
  }
  return GS_OK;
}

const char* gs_last_error(void) { return gsh::last_error(); }

int gs_device_count(int* count) {
  if (!count) return GS_EINVAL;
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  *count = c;
  return GS_OK;
}

int gs_config_init(gs_config* cfg) {
  if (!cfg) return GS_EINVAL;
  std::memset(cfg, 0, sizeof(*cfg));
  // tile_config.hpp:5-15: 1280x720, 40x36 tiles of 32x20; codelets.cpp:622
  cfg->width = 1280;
  cfg->height = 720;
  cfg->tile_width = 32;
  cfg->tile_height = 20;
  cfg->guard_band = 15.0f;
  cfg->device = -1;
  cfg->band_index = 0;
  cfg->band_count = 1;
  for (int k = 0; k < GS_MAX_GPUS; ++k) cfg->device_ids[k] = k;
  return GS_OK;
}

int gs_create(const gs_gaussian3d* g, size_t n, const gs_config* cfg, gs_renderer** out) {
  if (cfg && cfg->num_gpus > 0) return gsg::create(g, n, cfg, nullptr, 0, 1, out);
  return gsr::create(g, n, cfg, nullptr, out);
}

int gs_create_rank(const gs_gaussian3d* g, size_t n, const gs_config* cfg, const gs_comm_id* id,
                   int rank, int world, gs_renderer** out) {
  if (!id) {
    set_error("gs_create_rank: null communicator id");
    return GS_EINVAL;
  }
  return gsg::create(g, n, cfg, id, rank, world, out);
}

void gs_destroy(gs_renderer* r) {
  if (!r) return;
  if (r->grp) {
    gsg::destroy(r->grp);
    delete r;
    return;
  }
  gsr::destroy(r);
}

int gs_set_view(gs_renderer* r, const float rowmajor[16]) {
  if (!r || !rowmajor) return GS_EINVAL;
  if (r->grp) return gsg::set_view(r->grp, rowmajor);
  std::memcpy(r->view_rm, rowmajor, sizeof(r->view_rm));
  return GS_OK;
}

int gs_set_projection(gs_renderer* r, const float rowmajor[16]) {
  if (!r || !rowmajor) return GS_EINVAL;
  if (r->grp) return gsg::set_projection(r->grp, rowmajor);
  std::memcpy(r->proj_rm, rowmajor, sizeof(r->proj_rm));
  return GS_OK;
}

int gs_set_focal(gs_renderer* r, float fov_rad, float scale_divisor) {
  if (!r) return GS_EINVAL;
  if (r->grp) return gsg::set_focal(r->grp, fov_rad, scale_divisor);
  r->fov = fov_rad;
  r->scale_div = scale_divisor;
  return GS_OK;
}

int gs_set_sh(gs_renderer* r, const float* f_dc, const float* f_rest, size_t n, int degree) {
  if (!r) return GS_EINVAL;
  if (r->grp) return gsg::set_sh(r->grp, f_dc, f_rest, n, degree);
  if (r->lattice) {
    set_error("gs_set_sh: the lattice emulator keeps the reference's DC colours");
    return GS_EINVAL;
  }
  return gsr::set_sh(r, f_dc, f_rest, n, degree);
}

int gs_set_band_rows(gs_renderer* r, uint32_t row_begin, uint32_t row_end, uint32_t pad_rows) {
  if (!r) return GS_EINVAL;
  if (r->grp || r->lattice) {
    set_error("gs_set_band_rows: a single-GPU frame renderer only (a group moves its own bands)");
    return GS_EINVAL;
  }
  if (r->band_stride != 1) {
    set_error("gs_set_band_rows: interleaved bands are fixed at creation");
    return GS_EINVAL;
  }
  if (row_end > (uint32_t)r->tiles_y || row_begin >= row_end) {
    set_error("gs_set_band_rows: rows outside the tile grid");
    return GS_EINVAL;
  }
  // No wait: a frame in flight keeps the rows it was enqueued with (its
  // parameters went with its launches), and its overflow stays in the sticky
  // word for the next gs_sync.  Its readbacks are refused from here on (they
  // would read it with the new band's geometry) until the next frame.
  const int pad = std::max<int>((int)(row_end - row_begin), (int)pad_rows);
  const int rc = gsr::set_band_rows(r, (int)row_begin, (int)row_end, pad);
  if (rc == GS_OK && r->have_fp) {
    r->band_moved = true;
    std::lock_guard<std::mutex> lk(r->hist_mu);
    r->hist_moved = true;  // (the snapshot is the old band's until the next frame completes)
  }
  return rc;
}

int gs_set_stream(gs_renderer* r, void* hip_stream) {
  if (!r) return GS_EINVAL;
  if (r->grp) {
    set_error("gs_set_stream: a row-band group runs its frames on its own streams");
    return GS_EINVAL;
  }
  if (r->frame_pending) {
    set_error("gs_set_stream: a frame is in flight");
    return GS_EINVAL;
  }
  r->stream = hip_stream ? (hipStream_t)hip_stream : r->own_stream;
  return GS_OK;
}

int gs_get_stream(gs_renderer* r, void** hip_stream) {
  if (!r || !hip_stream) return GS_EINVAL;
  if (r->grp) return gsg::get_stream(r->grp, hip_stream);
  *hip_stream = (void*)r->stream;
  return GS_OK;
}

int gs_render_async(gs_renderer* r) {
  if (!r) return GS_EINVAL;
  if (r->grp) return gsg::render_async(r->grp);
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  return enqueue_frame(r);
}

int gs_sync(gs_renderer* r) {
  if (!r) return GS_EINVAL;
  if (r->grp) return gsg::sync(r->grp);
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  return finish_frame(r);
}

int gs_render(gs_renderer* r) {
  if (!r) return GS_EINVAL;
  if (r->grp) return gsg::render(r->grp);
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  for (int attempt = 0; attempt < 8; ++attempt) {
    rc = enqueue_frame(r);
    if (rc != GS_OK) return rc;
    rc = finish_frame(r);
    if (rc != GS_EOVERFLOW) return rc;
    // grow the pair capacity (the reference silently drops on overflow)
    if ((rc = grow_pairs(r, true)) != GS_OK) return rc;
  }
  set_error("gs_render: capacity growth did not converge");
  return GS_EOVERFLOW;
}

int gs_read_bgr8(gs_renderer* r, uint8_t* dst, size_t bytes) {
  if (!r || !dst) return GS_EINVAL;
  if (r->grp) return gsg::read_bgr8(r->grp, dst, bytes);
  if (refuse_moved(r, "gs_read_bgr8") != GS_OK) return GS_EINVAL;
  const size_t need = (size_t)r->band_rows * r->cfg.width * 3;
  if (bytes < need) {
    set_error("gs_read_bgr8: destination too small");
    return GS_EINVAL;
  }
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  if ((rc = finish_frame(r)) != GS_OK) return rc;
  GS_HIP(hipMemcpy(dst, r->last_bgr, need, hipMemcpyDeviceToHost));
  return GS_OK;
}

int gs_read_rgba32f(gs_renderer* r, float* dst, size_t n_floats, int layout) {
  if (!r || !dst) return GS_EINVAL;
  if (r->grp) return gsg::read_rgba32f(r->grp, dst, n_floats, layout);
  return gsr::read_rgba32f(r, dst, n_floats, layout);
}

int gs_read_tile_histogram(gs_renderer* r, uint32_t* dst, size_t n) {
  if (!r || !dst) return GS_EINVAL;
  if (r->grp) return gsg::read_tile_histogram(r->grp, dst, n);
  std::lock_guard<std::mutex> lk(r->hist_mu);
  if (r->hist_moved) {
    set_error("gs_read_tile_histogram: the band moved (gs_set_band_rows) after the last frame; render a frame first");
    return GS_EINVAL;
  }
  if (n < r->hist_snapshot.size()) {
    set_error("gs_read_tile_histogram: destination too small");
    return GS_EINVAL;
  }
  std::copy(r->hist_snapshot.begin(), r->hist_snapshot.end(), dst);
  return GS_OK;
}

int gs_get_stats(gs_renderer* r, gs_frame_stats* st) {
  if (!r || !st) return GS_EINVAL;
  if (r->grp) return gsg::get_stats(r->grp, st);
  *st = r->stats;
  st->pair_capacity = r->pair_cap;
  return GS_OK;
}

int gs_read_bins(gs_renderer* r, uint64_t* tile_start, size_t n_start, uint32_t* list,
                 size_t n_list) {
  if (!r || !tile_start || (!list && n_list)) return GS_EINVAL;
  if (r->grp) return gsg::read_bins(r->grp, tile_start, n_start, list, n_list);
  return gsr::read_bins(r, tile_start, n_start, list, n_list);
}

int gs_read_projected(gs_renderer* r, float* dst, size_t n_floats) {
  if (!r || !dst) return GS_EINVAL;
  if (r->grp) return gsg::read_projected(r->grp, dst, n_floats);
  return gsr::read_projected(r, dst, n_floats);
}

int gs_bgr8_device(gs_renderer* r, void** dev_ptr, size_t* bytes) {
  if (!r || !dev_ptr || !bytes) return GS_EINVAL;
  if (r->grp) {
    set_error("gs_bgr8_device: a row-band group gathers its frame itself (gs_read_bgr8)");
    return GS_EINVAL;
  }
  *dev_ptr = r->own_bgr;
  *bytes = r->bgr_bytes;
  return GS_OK;
}

int gs_copy_bgr8_device(gs_renderer* r, void* dst_dev, size_t bytes) {
  if (!r || !dst_dev || r->grp || bytes < r->bgr_bytes) return GS_EINVAL;
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  GS_HIP(hipMemcpyAsync(dst_dev, r->last_bgr, r->bgr_bytes, hipMemcpyDeviceToDevice, r->stream));
  return GS_OK;
}

int gs_set_bgr8_target(gs_renderer* r, void* dst_dev, size_t bytes) {
  if (!r) return GS_EINVAL;
  if (r->grp) {
    set_error("gs_set_bgr8_target: a row-band group writes its bands into its own all-gather buffers");
    return GS_EINVAL;
  }
  if (dst_dev && bytes < r->bgr_bytes) {
    set_error("gs_set_bgr8_target: destination smaller than the padded band");
    return GS_EINVAL;
  }
  r->bgr_target = (uint8_t*)dst_dev;
  return GS_OK;
}

int gs_kernel_times(gs_renderer* r, double* avg_ms, uint64_t* launches, int n) {
  if (!r || !avg_ms) return GS_EINVAL;
  if (r->grp) return gsg::kernel_times(r->grp, avg_ms, launches, n);
  if (!r->profile) {
    set_error("gs_kernel_times: renderer created without GS_FLAG_PROFILE");
    return GS_EINVAL;
  }
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  for (auto& s : r->ring)
    if ((rc = profile_harvest(r, s)) != GS_OK) return rc;
  for (int k = 0; k < n && k < GS_K_COUNT; ++k) {
    avg_ms[k] = r->k_launches[k] ? r->k_ms[k] / (double)r->k_launches[k] : 0.0;
    if (launches) launches[k] = r->k_launches[k];
  }
  return GS_OK;
}

int gs_set_profile_interval(gs_renderer* r, uint32_t every) {
  if (!r || every == 0) return GS_EINVAL;
  if (r->grp) return gsg::set_profile_interval(r->grp, every);
  r->profile_every = every;
  r->frame_seq = 0;
  return GS_OK;
}

int gs_reset_kernel_times(gs_renderer* r) {
  if (!r) return GS_EINVAL;
  if (r->grp) return gsg::reset_kernel_times(r->grp);
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  for (auto& s : r->ring)
    if ((rc = profile_harvest(r, s)) != GS_OK) return rc;
  for (int k = 0; k < GS_K_COUNT; ++k) {
    r->k_ms[k] = 0.0;
    r->k_launches[k] = 0;
  }
  return GS_OK;
}

int gs_get_lattice_stats(gs_renderer* r, gs_lattice_stats* st) {
  if (!r || !st) return GS_EINVAL;
  if (r->grp || !r->lattice) {
    set_error("gs_get_lattice_stats: renderer created without GS_FLAG_LATTICE");
    return GS_EINVAL;
  }
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  if ((rc = finish_frame(r)) != GS_OK) return rc;
  std::memset(st, 0, sizeof(*st));
  st->frames = r->lat_frames;
  st->total_slots = r->lat_slots;
  if (r->lat_frames) {
    const uint32_t* c = r->h_counters;
    st->dropped = c[12];
    st->send_failed = c[13];
    st->zbuf_overrun = c[14];
  }
  st->records_per_tile = (uint32_t)r->lat_gpt;
  st->extra_records = (uint32_t)r->lat_rem;
  st->slots_per_tile = (uint32_t)(r->lat_gpt + gsk::kLatExtra);
  st->channel_slots = (uint32_t)gsk::kLatChan;
  return GS_OK;
}

int gs_read_lattice_slots(gs_renderer* r, float* gids, size_t n) {
  if (!r || !gids) return GS_EINVAL;
  if (r->grp || !r->lattice) {
    set_error("gs_read_lattice_slots: renderer created without GS_FLAG_LATTICE");
    return GS_EINVAL;
  }
  if (n < r->lat_slots) {
    set_error("gs_read_lattice_slots: destination too small");
    return GS_EINVAL;
  }
  int rc = select_device(r);
  if (rc != GS_OK) return rc;
  if ((rc = finish_frame(r)) != GS_OK) return rc;
  // the gid is the last float of every 64-B slot: one strided copy
  GS_HIP(hipMemcpy2D(gids, sizeof(float), (const char*)r->lat.slots + 60, 64, sizeof(float), r->lat_slots,
                     hipMemcpyDeviceToHost));
  return GS_OK;
}

int gs_group_bands(gs_renderer* r, uint32_t* bounds, size_t n) {
  if (!r || !bounds) return GS_EINVAL;
  if (!r->grp) {
    set_error("gs_group_bands: not a row-band group");
    return GS_EINVAL;
  }
  return gsg::bands(r->grp, bounds, n);
}

int gs_balanced_bands(const double* row_work, uint32_t rows, uint32_t world, uint32_t* bounds) {
  if (!row_work || !bounds || world == 0 || rows < world) {
    set_error("gs_balanced_bands: need rows >= world >= 1");
    return GS_EINVAL;
  }
  gsg::balanced_bands(row_work, (int)rows, (int)world, bounds);
  return GS_OK;
}

}  // extern "C"
