// gs_internal.hpp -- the renderer object behind the C ABI handle, shared by
// gs_renderer.hip (one band on one device) and gs_group.hip (the row-band
// group: several band renderers, one per device, and the all-gather).
// Internal to libgsplat.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gsplat.h"
#include "gs_kernels.hpp"

namespace gsg {
struct Group;
}

namespace gsr {

constexpr int kProfileRing = 64;
constexpr int kStages = gsk::GS_STAGE_EVENTS - 1;  // project .. blend, blend continuation
// the kernel id (GS_K_*) of profile stage k
constexpr int kStageKernel[kStages] = {GS_K_PROJECT, GS_K_SCAN, GS_K_EMIT, GS_K_SORT, GS_K_BLEND, GS_K_BLEND_CONT};

struct ProfileSlot {
  hipEvent_t ev[gsk::GS_STAGE_EVENTS];
  bool pending = false;
};

}  // namespace gsr

struct gs_renderer {
  gs_config cfg{};
  int device = 0;
  size_t n = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;

  // a row-band group handle (gs_create with num_gpus, gs_create_rank): every
  // call of the C ABI goes to the group; the fields below are unused then
  gsg::Group* grp = nullptr;

  // frame inputs (row-major as on the reference's wire)
  float view_rm[16];
  float proj_rm[16];
  float fov = 0.6981317f;  // glm::radians(40.f) (splat.cpp:170)
  float scale_div = 0.1f;  // lambda1 / 10 with lambda1 = 1 (InterfaceServer.hpp:238)
  // gs_set_sh: the SH coefficients on the device ([16 x 3][n], device order)
  void* d_sh = nullptr;
  bool owns_sh = false;
  int sh_degree = -1;  // < 0: off

  std::vector<uint32_t> perm;  // device index -> input index

  // geometry
  int tiles_x = 0, tiles_y = 0, band_ty0 = 0, band_stride = 1, band_nrows = 0, band_py0 = 0,
      band_rows = 0;
  int band_rows_padded = 0, n_tiles = 0;
  int t_cap = 0;     // tiles the per-tile buffers were sized for (>= n_tiles)
  int rows_cap = 0;  // tile rows the framebuffer was sized for (>= padded band rows)
  uint64_t pair_cap = 0;

  // device memory
  void* d_scene = nullptr;      // 4 x float4 x n + perm, inv_perm
  bool owns_scene = true;       // false: shares another renderer's scene on this device
  bool scene_w1 = false;        // every mean has w == 1: the projection reads mean_op (xyz + opacity)
  void* d_gauss = nullptr;      // rec (48 B) + tail, rect, crect (8 B each) + depth key (4 B) per Gaussian
  void* d_zero = nullptr;       // counters[16] + tile_count[t_cap] (memset every frame)
  void* d_tiles = nullptr;      // tile_start[t_cap+1], tile_cursor, big_tiles
  void* d_pairs = nullptr;      // pairs, pairs_alt, list
  void* d_out = nullptr;        // rgba f32 + bgr8
  void* d_chunk = nullptr;      // chunk histogram / offset matrix (chunked binning)
  void* d_lazy = nullptr;       // lazy big lists (16x16 tiles): per-tile tables + saved blend waves
  void* d_agg = nullptr;        // aggregated binning: per projection block its tile box and offsets
  void* d_dir = nullptr;        // direct band binning: the blend's ticket and the overflow word
  void* d_cov = nullptr;        // the scene's 3D covariances (Buffers::cov3): 9 float planes, 36 B per
                                // Gaussian, an empty slot marked by Sigma[2][2] < 0; null: computed per frame
  float cov_sd = 0.0f;          // ... computed for this fxy[1]
  bool cov_valid = false;
  void* d_probe = nullptr;      // (GS_PROBE builds, GSPLAT_PROBE_FILE) the kernels' per-frame start / end ring
  int probe_n = 0;              // frames recorded in it
  // GS_FLAG_LATTICE: the lattice-migration emulator's state (gs_lattice.hip)
  void* d_lat = nullptr;
  bool lattice = false;
  gsk::LatticeBufs lat{};
  int lat_gpt = 0, lat_rem = 0;  // initial records per tile, extra records of the last tile
  size_t lat_slots = 0;          // vertsIn slots over all tiles
  uint64_t lat_frames = 0;       // frames stepped (the exchange parity)
  int bin_global = 0, chunk_size = 0, n_chunks = 0;
  size_t chunk_entries = 0;     // chunk table size (chunks x tiles)
  bool chunk_adaptive = false;  // bands: more, smaller chunks (make_params)
  bool bin_agg = false;         // aggregated binning (gs_kernels.hip: agg_count, gs_agg_scan/emit)
  bool pair_cull = false;       // chunked binning into the alpha-box tiles only
  size_t zero_bytes = 0;
  size_t bgr_bytes = 0;
  gsk::Buffers buf{};

  // host mirrors
  uint32_t* h_counters = nullptr;  // mapped pinned mirror of d_zero: counters[16] + tile_count[T]
  std::vector<uint32_t> hist_snapshot;
  std::mutex hist_mu;
  bool hist_moved = false;  // (under hist_mu) gs_set_band_rows after the snapshot's frame
  bool frame_pending = false;
  // gs_set_band_rows moved the band after the last enqueued frame: that
  // frame's readbacks are refused (its geometry is not the renderer's now)
  bool band_moved = false;
  uint8_t* own_bgr = nullptr;     // the renderer's BGR8 band buffer
  uint8_t* bgr_target = nullptr;  // gs_set_bgr8_target: frames write their BGR8 here instead
  uint8_t* last_bgr = nullptr;    // where the last enqueued frame wrote its BGR8
  bool have_frame = false;
  gs_frame_stats stats{};
  // the parameters of the last enqueued frame: the debug readbacks
  // (gs_read_projected, gs_read_bins) reproduce THAT frame, not the current
  // camera (a gs_set_view after the frame changes nothing they return)
  gsk::FrameParams last_fp{};
  bool have_fp = false;

  // profiling
  bool profile = false;
  uint32_t profile_every = 1;  // stage events on every n-th frame
  void* d_bcount = nullptr;    // blend_count (profile renderers)
  size_t bcount_words = 0;
  bool last_counted = false;   // the last enqueued frame counted its blend records
  uint64_t frame_seq = 0;
  uint64_t x_frames = 0;  // (GS_X_BAND measurement builds only: this renderer's frames)
  // direct band binning: frames are numbered (FrameParams::frame_seq, echoed
  // in the host mirror's word 15); cam_first_seq = the first frame enqueued
  // with the current camera, projection, focal lengths and band; layout_seq =
  // the last frame binned by a scan (its tile_start is the direct frames'
  // layout; 0 after an overflow); direct_veto: an overflow since then (the
  // test hook's forced direct frames wait for a scan too)
  uint32_t seq_next = 1, cam_first_seq = 0, layout_seq = 0;
  bool direct_veto = false;
  bool cam_key_set = false;
  float cam_key[40] = {0};
  gsr::ProfileSlot ring[gsr::kProfileRing];
  int ring_head = 0;
  double k_ms[GS_K_COUNT] = {0};
  uint64_t k_launches[GS_K_COUNT] = {0};
};

namespace gsr {

int hip_fail(hipError_t e, const char* what);
void poison(void* p, size_t bytes, const char* name);  // GSPLAT_DEBUG_POISON (gs_renderer.hip)

#define GS_HIP(call)                                        \
  do {                                                      \
    hipError_t e_ = (call);                                 \
    if (e_ != hipSuccess) return gsr::hip_fail(e_, #call);  \
  } while (0)

// One band renderer on one device.  share: another renderer on the same
// device whose scene (and device order) this one uses instead of uploading
// its own copy (nullptr: upload).
int create(const gs_gaussian3d* g, size_t n, const gs_config* cfg, const gs_renderer* share,
           gs_renderer** out);
void destroy(gs_renderer* r);
// Move a renderer created over tile rows [0, rows_cap) to the contiguous band
// [ty0, ty1), its BGR8 padded to pad_rows tile rows (for the next frames).
int set_band_rows(gs_renderer* r, int ty0, int ty1, int pad_rows);
int enqueue_frame(gs_renderer* r);
int finish_frame(gs_renderer* r);
uint32_t frame_paths(const gs_renderer* r);  // gs_frame_stats.paths of the last enqueued frame
// after GS_EOVERFLOW: grow the pair buffers to hold the last frame's pairs
// (force: at least double them, even if the last frame fit)
int grow_pairs(gs_renderer* r, bool force);
int alloc_pairs(gs_renderer* r, uint64_t cap);
int profile_harvest(gs_renderer* r, ProfileSlot& s);
int read_bins(gs_renderer* r, uint64_t* tile_start, size_t n_start, uint32_t* list, size_t n_list);
int read_projected(gs_renderer* r, float* dst, size_t n_floats);
int read_rgba32f(gs_renderer* r, float* dst, size_t n_floats, int layout);
// share: a renderer on the same device whose coefficients (set by the same
// call just before) this one uses instead of uploading its own copy
int set_sh(gs_renderer* r, const float* f_dc, const float* f_rest, size_t n, int degree,
           const gs_renderer* share = nullptr);
// the camera position (scene frame) of a row-major view matrix: -A^-1 t, double, rounded once
void camera_position(const float* view_rm, float* campos);
// the IPU tile-major layout (codelets.cpp:174-176) of a row-major RGBA f32 band
void retile(const float* rm, size_t rows, size_t W, size_t tw, size_t th, int tiles_x, int n_tiles,
            float* dst);

}  // namespace gsr

// the row-band group (gs_group.hip)
namespace gsg {

int create(const gs_gaussian3d* g, size_t n, const gs_config* cfg, const gs_comm_id* id, int rank,
           int world, gs_renderer** out);
void destroy(Group* grp);
int set_view(Group* grp, const float* rm);
int set_projection(Group* grp, const float* rm);
int set_focal(Group* grp, float fov, float sd);
int render(Group* grp);
int render_async(Group* grp);
int sync(Group* grp);
int get_stream(Group* grp, void** s);
int read_bgr8(Group* grp, uint8_t* dst, size_t bytes);
int read_rgba32f(Group* grp, float* dst, size_t n_floats, int layout);
int read_tile_histogram(Group* grp, uint32_t* dst, size_t n);
int get_stats(Group* grp, gs_frame_stats* st);
int read_bins(Group* grp, uint64_t* tile_start, size_t n_start, uint32_t* list, size_t n_list);
int read_projected(Group* grp, float* dst, size_t n_floats);
int kernel_times(Group* grp, double* avg_ms, uint64_t* launches, int n);
int reset_kernel_times(Group* grp);
int set_profile_interval(Group* grp, uint32_t every);
int bands(Group* grp, uint32_t* bounds, size_t n);
int info(Group* grp, gs_group_info* out);
int set_sh(Group* grp, const float* f_dc, const float* f_rest, size_t n, int degree);
// the split rule (also exported as gs_balanced_bands)
void balanced_bands(const double* work, int rows, int world, uint32_t* bounds);

}  // namespace gsg
