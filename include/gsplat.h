/*
 * gsplat.h -- C ABI of the MI355X Gaussian-splat tile rasteriser (libgsplat.so).
 *
 * This is the drop-in boundary for the reference's operator
 * `splat::IpuSplatter` (include/splat/ipu_rasteriser.hpp:20-55 in
 * Nmjfry/gaussian_splat_ipu).  Every entry point below names the reference
 * interface it replaces.  Plain C types only: no C++, HIP or torch types cross
 * this ABI, no exceptions cross it; every call returns a gs_status and the
 * reason for a failure is available from gs_last_error() (thread-local).
 *
 * Threading (reference: one render thread drives updateModelView, execute and
 * getFrameBuffer,
 * the UI thread reads the histogram, splat.cpp:208-225,257-265): calls on one
 * handle must be serialised by the caller, except gs_read_tile_histogram, which
 * reads a mutex-protected host snapshot and is safe from any thread.
 */
#ifndef GSPLAT_H
#define GSPLAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSPLAT_ABI_VERSION 14

typedef enum gs_status {
  GS_OK = 0,
  GS_EINVAL = 1,     /* bad argument (std::logic_error in the reference) */
  GS_EDEVICE = 2,    /* HIP runtime / device failure (no GPU, launch error) */
  GS_EOOM = 3,       /* device or pinned-host allocation failed */
  GS_EOVERFLOW = 4,  /* (tile, Gaussian) pair list exceeded capacity; the
                        reference drops Gaussians silently (codelets.cpp:544) */
  GS_EIO = 5         /* file could not be read / parsed */
} gs_status;

/* One world-space Gaussian, 64 bytes: splat::Gaussian3D
 * (include/splat/ipu_geometry.hpp:305-311) as flattened by the IpuSplatter
 * constructor (src/splat/ipu_rasteriser.cpp:49-68). */
typedef struct gs_gaussian3d {
  float mean[4];    /* x, y, z, w (w = 1)                         */
  float colour[4];  /* r, g, b, raw opacity logit (no sigmoid)    */
  float rot[4];     /* quaternion, rot[0] is the real part        */
  float scale[3];   /* raw log-scales                             */
  float gid;        /* i + 1; gid <= 0 marks an empty slot        */
} gs_gaussian3d;

/* Renderer configuration: the TiledFramebuffer (tile_config.hpp:19-41) and
 * the hard-coded constants of the codelet (codelets.cpp:620-622). */
typedef struct gs_config {
  uint32_t width, height;             /* IMWIDTH, IMHEIGHT                  */
  uint32_t tile_width, tile_height;   /* IPU_TILEWIDTH, IPU_TILEHEIGHT      */
  uint32_t guard_tile_width;          /* tile size used by the guard band;  */
  uint32_t guard_tile_height;         /*   0 = same as the render tile      */
  float guard_band;                   /* clipSize (15)                      */
  int32_t device;                     /* HIP device ordinal, -1 = current   */
  uint32_t band_index, band_count;    /* row-band shard: tile rows split into
                                         band_count contiguous bands, or
                                         interleaved (GS_FLAG_BAND_INTERLEAVED:
                                         rows r with r % band_count ==
                                         band_index)                         */
  uint64_t pair_capacity;             /* initial (tile,Gaussian) capacity, 0 = auto */
  uint32_t flags;                     /* GS_FLAG_*                          */
  /* ABI 4: an explicit contiguous band, tile rows [band_row_begin,
   * band_row_end), used instead of band_index / band_count when
   * band_row_end > band_row_begin (work-balanced bands chosen by the caller,
   * e.g. from a frame's row histogram: dist.balanced_bands).  band_pad_rows:
   * the BGR8 band is padded to this many tile rows (>= the band's), so every
   * rank of an all-gather contributes the same number of bytes.  0 = none. */
  uint32_t band_row_begin, band_row_end, band_pad_rows;
  /* ABI 6: row-band group (SURVEY §8 b/e: "multi-GPU fan-out is internal to
   * gs_render").  num_gpus >= 1 makes gs_create return ONE handle over
   * num_gpus devices of this process (device_ids[0..num_gpus)): the tile rows
   * are split into num_gpus contiguous bands, one per device, re-balanced from
   * the tile histograms of earlier frames, and every frame ends with one
   * all-gather of the BGR8 bands (RCCL, ncclCommInitAll over the devices).
   * The band fields above are then ignored.  num_gpus = 0: one renderer (the
   * band fields apply).  frames_in_flight (group only, 0 = 1): frames a group
   * keeps in flight under gs_render_async, each on its own HIP stream. */
  uint32_t num_gpus;
  int32_t device_ids[16];
  uint32_t frames_in_flight;
} gs_config;

#define GS_MAX_GPUS 16

#define GS_FLAG_NO_RGBA32F 1u  /* skip the RGBA f32 framebuffer store (BGR8 only) */
#define GS_FLAG_PROFILE 2u     /* record HIP events around every kernel     */
#define GS_FLAG_BIN_GLOBAL 4u  /* bin with global atomics instead of the chunked
                                  LDS histograms (automatic for > 81920 tiles) */
#define GS_FLAG_INPUT_ORDER 8u /* keep the Gaussians in input order on the device
                                  (default: 3D Morton order, which makes the
                                  binning writes and the blend's record reads
                                  local; results are identical either way) */
#define GS_FLAG_BAND_INTERLEAVED 16u /* band = tile rows band_index,
                                  band_index + band_count, ...: every band gets
                                  an equal share of a scene's dense rows */
#define GS_FLAG_BAND_CULL 32u  /* skip the full projection of Gaussians whose
                                  conservative screen extent misses every row
                                  of this band (frames, lists and histograms
                                  are unchanged; n_rendered then counts only
                                  the Gaussians that reach the band) */
#define GS_FLAG_NO_PAIR_CULL 64u /* bin every tile of the reference rectangle.
                                  By default a Gaussian is binned only into the
                                  tiles its alpha >= 1/255 box meets (the
                                  frame is bit-identical; the histogram and
                                  gs_read_bins keep the reference lists) */
#define GS_FLAG_NO_REBALANCE 128u /* group: keep the first split (equal tile-row
                                  bands) instead of re-balancing it from the
                                  histograms of earlier frames */
#define GS_FLAG_GATHER_COPY 256u /* group, one process: gather the bands with
                                  device-to-device copies instead of RCCL
                                  (automatic when device_ids repeat a device:
                                  several bands emulated on one GPU) */
#define GS_FLAG_LATTICE 512u     /* ABI 7, SURVEY §8 f4: emulate the reference's
                                  multi-frame lattice migration instead of the
                                  converged single-frame binning.  Every
                                  gs_render is one step of the IPU program --
                                  the GSplat codelet of every tile and the
                                  channel exchange (ipu_rasteriser.cpp:393-399,
                                  codelets.cpp:143-641, edge_builder.cpp:35-84)
                                  -- from the reference's initial distribution
                                  of the records by index, so the frames are its
                                  transient ones (75-record channels, y-first
                                  routing, silent drops, the off-by-one
                                  quicksort, the stale splatted counters).
                                  Needs width % tile_width == 0, height %
                                  tile_height == 0, one band, one device; the
                                  guard band uses the tile's own diagonal;
                                  gs_read_bins is unavailable. */
#define GS_FLAG_FAST_EXP 1024u   /* ABI 8, opt-in: the blend takes exp() from the
                                  hardware exp2 on an fma-split argument
                                  (a few ulp; the oracle's portable expf is
                                  not reproduced).  Tile lists, histograms and
                                  stats stay bit-exact; per-pixel RGBA is within
                                  the tolerance DESIGN.md states and
                                  tests/test_gpu_fast_exp.py checks (SURVEY §8:
                                  "per-pixel RGB within a stated float
                                  tolerance").  Not the default: without it
                                  every frame is bit-exact. */

typedef enum gs_layout {
  GS_LAYOUT_ROW_MAJOR = 0,      /* H x W x 4, row-major                     */
  GS_LAYOUT_REF_TILE_MAJOR = 1  /* the IPU framebuffer layout: one tile's
                                   tw*th*4 floats after another, pixel (x,y)
                                   at (x + y*tw)*4 (codelets.cpp:174-176)   */
} gs_layout;

typedef struct gs_frame_stats {
  uint64_t n_gaussians;   /* N                                  */
  uint64_t n_rendered;    /* V: pass guard band and z < 0       */
  uint64_t n_pairs;       /* P: sum over tiles of the reference list
                             lengths (the histogram)            */
  uint64_t max_list;      /* max reference tile list length     */
  uint64_t pair_capacity;
  uint32_t n_tiles;       /* tiles in this renderer's band      */
  uint32_t tiles_x, tiles_y;
  uint32_t band_y0, band_rows;  /* pixel rows of this band: contiguous
                                   bands start at band_y0; interleaved bands
                                   hold their tile rows back to back, padded
                                   to whole tiles                   */
  uint32_t n_big_tiles;   /* tiles sorted by the large-list path */
  uint32_t band_stride;   /* tile-row stride of the band (1: contiguous) */
  uint64_t n_pairs_binned; /* pairs binned, sorted and blended: P minus
                              the pairs culled by the alpha box (= P with
                              GS_FLAG_NO_PAIR_CULL)                   */
  uint32_t bin_global;    /* ABI 5: 1 = the global-atomic binning path (tile
                             grids beyond one CU's LDS, or GS_FLAG_BIN_GLOBAL) */
  uint32_t paths;         /* ABI 11: the last frame's binning / sort paths:
                             bit 0 (GS_PATH_BIN_AGG) the aggregated binning,
                             bit 1 (GS_PATH_BLEND_SORT) the tile sort inside
                             the blend's workgroups (no tile-sort launch) */
  uint64_t blend_records;      /* ABI 8, GS_FLAG_PROFILE renderers (frames with
                                  stage events; else 0): tile-list records the
                                  blend read in the last frame, per tile the
                                  longest prefix any of its waves staged
                                  (a wave stops when its pixels have
                                  saturated; lazy big lists: the sorted
                                  prefixes only)                             */
  uint64_t blend_cont_records; /* ... and the records the continuation staged */
  uint64_t cont_keys;     /* ABI 8, profiled lazy frames: keys the continuation
                             sorted (past the prefixes, alpha box meeting the
                             saved waves' live pixels), summed over its lists */
  uint32_t cont_lists;    /* big lists the continuation ran on             */
  uint32_t cont_max;      /* the longest of their continuation key lists   */
  uint32_t prefix_overflows; /* big lists whose keys below the depth bound
                             outnumbered one workgroup's sort (the whole
                             list went to the continuation)              */
  uint32_t cont_full_sorts; /* of the continued lists, those whose live pixels
                             outlived the sorted window past the prefix (the
                             full sample sort of the rest ran for them)   */
  uint64_t big_pairs;     /* ABI 9, profiled frames: binned pairs in the big
                             lists (> 2048 keys; bench.py's sort bytes)    */
  uint64_t big_prefix_keys; /* ABI 9, profiled lazy frames: keys the prefix
                             select kept and sorted before the blend        */
  uint64_t big_window_keys; /* ABI 9, profiled lazy frames: keys kept for the
                             continuation's windows                        */
} gs_frame_stats;

/* gs_frame_stats.paths bits (ABI 11; bits 2-4 ABI 12, 5-6 ABI 13, 7 ABI 14): which kernels the
   last frame launched, so a profile's per-kernel counters can be matched to
   the frame path (bench.py's roofline) */
enum {
  GS_PATH_BIN_AGG = 1,     /* aggregated binning (gs_agg_scan / gs_agg_emit)     */
  GS_PATH_BLEND_SORT = 2,  /* tile sort inside the blend (gs_blend_sort)         */
  GS_PATH_BLEND_PX2 = 4,   /* two pixels per blend lane (gs_blend_px2)           */
  GS_PATH_LAZY = 8,        /* lazy big lists (prefix select / sort, continuation) */
  GS_PATH_BIG_LISTS = 16,  /* the big-list launches ran (lists > 2048 keys)       */
  GS_PATH_PROJ_BAND = 32,  /* ABI 13: the row band's projection (gs_project_band) */
  GS_PATH_PROJ_ANY = 64,   /* ABI 13: the every-path projection (gs_project_any:
                              readback records, SH, global atomics, non-power-of-
                              two tiles); neither bit: gs_project (whole frames) */
  GS_PATH_BIN_DIRECT = 128 /* ABI 14: a row band's direct binning: the projection
                              placed the pairs in fixed per-tile segments, no
                              gs_agg_scan / gs_agg_emit launch */
};

/* Kernel ids for gs_kernel_times (GS_FLAG_PROFILE). */
enum {
  GS_K_PROJECT = 0,
  GS_K_SCAN = 1,
  GS_K_EMIT = 2,
  GS_K_SORT = 3,
  GS_K_BLEND = 4,
  GS_K_GATHER = 5,  /* group: the frame's all-gather on the communication
                       stream, from the local band's completion to the
                       gathered frame (includes waiting for the slowest rank) */
  GS_K_BLEND_CONT = 6, /* ABI 8: lazy big lists (16x16 tiles, lists > 2048): the
                          full sort of the lists whose blend outlived the sorted
                          prefix + the continued blend (gs_blend_cont) */
  GS_K_COUNT = 7
};

typedef struct gs_renderer gs_renderer;

/* ------------------------------------------------------------ lifetime */
int gs_abi_version(void);
const char* gs_last_error(void);
int gs_device_count(int* count);
/* Defaults: 1280x720, 32x20 tiles, guard band 15 (the reference build). */
int gs_config_init(gs_config* cfg);

/* Replaces IpuSplatter::IpuSplatter(const Gaussians&, TiledFramebuffer&, bool)
 * (ipu_rasteriser.cpp:49-83) + GraphManager::compileOrLoad/prepareEngine
 * (splat.cpp:166-168,199).  Copies the records to the device once (the
 * reference's "write_verts" program, ipu_rasteriser.cpp:401-418); the caller
 * keeps ownership of `g`. */
int gs_create(const gs_gaussian3d* g, size_t n, const gs_config* cfg, gs_renderer** out);
/* Replaces IpuSplatter::~IpuSplatter. */
void gs_destroy(gs_renderer* r);

/* ABI 6: one process per GPU.  The row-band group of gs_create (num_gpus) as
 * one rank of `world` processes: this process renders band `rank` on
 * cfg->device and every frame ends with one ncclAllGather over a communicator
 * built from `id` (ncclCommInitRank).  Rank 0 creates the id
 * (gs_comm_id_create) and the caller hands its bytes to the other ranks (e.g.
 * a torch.distributed broadcast).
 * Collective calls: gs_render, gs_render_async and gs_sync -- every rank calls
 * them for the same frames, in the same order (each frame ends with an
 * all-gather); camera inputs must be the same on every rank.  Their status and
 * the split of later frames are decided from the gathered footers only, the
 * same bytes on every rank (gs_group_decide), so every rank returns the same
 * status and a blocking gs_render re-renders on all ranks or on none.
 * Local calls: the readbacks (gs_read_*, gs_get_stats, gs_kernel_times, ...)
 * wait for this rank's frames and return the last frame's status, but change
 * neither the split nor the overflow state, so any subset of ranks may call
 * them.  gs_read_bgr8 and gs_read_tile_histogram return the whole frame on
 * every rank. */
typedef struct gs_comm_id {
  unsigned char bytes[128]; /* ncclUniqueId */
} gs_comm_id;
int gs_comm_id_create(gs_comm_id* out);
int gs_create_rank(const gs_gaussian3d* g, size_t n, const gs_config* cfg, const gs_comm_id* id,
                   int rank, int world, gs_renderer** out);
/* Group: the split of the last enqueued frame as world + 1 tile-row bounds
 * (band r = tile rows [bounds[r], bounds[r + 1])). */
int gs_group_bands(gs_renderer* r, uint32_t* bounds, size_t n);
/* ABI 10: what a group is and how its bands ran.  One process driving several
 * devices (gs_create with num_gpus > 1) enqueues each member's band and its
 * all-gather call on a host thread of its own (threaded = 1).  The per-band
 * times are HIP events of GS_FLAG_PROFILE frames (every
 * gs_set_profile_interval-th frame) since the last gs_reset_kernel_times:
 * band_ms = the band's first kernel to its last (its renderer's stream),
 * gather_ms = band written to frame gathered (its communication stream; this
 * includes waiting for the slowest band).  A rank of a multi-process group
 * (gs_create_rank) reports its own band only (local_bands = 1). */
typedef struct gs_group_info {
  uint32_t world;             /* bands of the frame (ranks)                     */
  uint32_t local_bands;       /* bands this process renders                     */
  int32_t comm_ranks;         /* ncclCommCount of this process's first
                                 communicator; -1 = copy gather (no RCCL)       */
  uint32_t multi_process;     /* 1 = gs_create_rank                             */
  uint32_t threaded;          /* 1 = one host thread per local band             */
  uint32_t frames_in_flight;
  uint64_t frames;            /* frames enqueued                                */
  uint64_t rebalances;        /* splits moved since gs_create                   */
  uint64_t timed_frames;      /* frames behind band_ms / gather_ms             */
  uint32_t bounds[GS_MAX_GPUS + 1]; /* split of the last enqueued frame (world + 1) */
  int32_t band_rank[GS_MAX_GPUS];   /* local band k renders band band_rank[k]     */
  int32_t device[GS_MAX_GPUS];      /* ... on this HIP device                     */
  double band_ms[GS_MAX_GPUS];      /* local band k: average band time            */
  double gather_ms[GS_MAX_GPUS];    /* local band k: average gather time          */
} gs_group_info;
int gs_group_get_info(gs_renderer* r, gs_group_info* out);
/* The group's split rule (host only, no device): `world` contiguous bands of
 * nearly equal work over `rows` tile rows, every band at least one row;
 * bounds = world + 1 entries.  Deterministic, so every rank derives the same
 * split from the same gathered histograms. */
int gs_balanced_bands(const double* row_work, uint32_t rows, uint32_t world, uint32_t* bounds);
/* ABI 8: the group's decision rule over one gathered frame (host only, no
 * device), the function every rank applies to the same bytes.  footers: world
 * x foot_words u32, band r's footer at r * foot_words: words 0..15 the band's
 * frame counters (3 = this frame overflowed, 5/6 = binned pairs low/high, 15 =
 * its GPU's sticky overflow bit since the last gs_sync), then the band's tile
 * list lengths (rows frame_bounds[r] .. frame_bounds[r + 1] of tiles_x tiles).
 * Returns GS_EOVERFLOW iff some band overflowed, else GS_OK.  next_bounds
 * (world + 1, may be NULL) = the split of later frames: cur_bounds unless
 * `rebalance` and the balanced split of this frame's histogram lowers the
 * slowest band's work by more than 3 % (never after an overflow).  need_pairs
 * (may be NULL) = the longest band pair list (capacity growth). */
int gs_group_decide(const uint32_t* footers, size_t foot_words, uint32_t world, uint32_t tiles_x,
                    uint32_t tiles_y, const uint32_t* frame_bounds, const uint32_t* cur_bounds, int rebalance,
                    uint32_t* next_bounds, uint64_t* need_pairs);

/* GS_FLAG_LATTICE renderers: the emulated lattice after the last frame. */
typedef struct gs_lattice_stats {
  uint64_t frames;         /* frames stepped since gs_create                 */
  uint64_t total_slots;    /* vertsIn slots over all tiles                   */
  uint64_t dropped;        /* last frame: vertsIn inserts that found no empty
                              slot (the reference drops them silently)      */
  uint64_t send_failed;    /* last frame: channel inserts into a full channel */
  uint64_t zbuf_overrun;   /* last frame: render-list entries past a tile's
                              z-buffer (the reference reads past it; here
                              they are empty records)                        */
  uint32_t records_per_tile; /* gpt: the initial records per tile           */
  uint32_t extra_records;    /* rem: the last tile's extra initial records  */
  uint32_t slots_per_tile;   /* gpt + 600 (the last tile: + rem)            */
  uint32_t channel_slots;    /* 75 records per channel                      */
} gs_lattice_stats;
int gs_get_lattice_stats(gs_renderer* r, gs_lattice_stats* st);
/* The gid of every vertsIn slot (0 = empty), tile-major: tile t's slots start
 * at t * slots_per_tile.  n >= total_slots. */
int gs_read_lattice_slots(gs_renderer* r, float* gids, size_t n);

/* ------------------------------------------------------------ per-frame inputs */
/* Replaces IpuSplatter::updateModelView (ipu_rasteriser.cpp:86-93): the
 * argument is the row-major float[16] the reference streams to the device
 * (glm::transpose(mv) flattened). */
int gs_set_view(gs_renderer* r, const float rowmajor[16]);
/* Replaces IpuSplatter::updateProjection (ipu_rasteriser.cpp:95-102). */
int gs_set_projection(gs_renderer* r, const float rowmajor[16]);
/* Replaces IpuSplatter::updateFocalLengths(fx, fy) (ipu_rasteriser.cpp:108-110):
 * fxy = (fov radians, scale divisor lambda1/10). */
int gs_set_focal(gs_renderer* r, float fov_rad, float scale_divisor);
/* ABI 8, opt-in view-dependent colour (the reference reads f_dc
 * only, file_io.cpp:66-68): spherical-harmonic coefficients of the n
 * Gaussians in INPUT order -- f_dc (n x 3) and f_rest (n x 3 x 15, the 3DGS
 * PLY's f_rest_0..44: channel-major, 15 coefficients per channel; may be NULL
 * when degree == 0) -- evaluated per frame for the direction from the camera
 * (the inverse of the view matrix) to the mean, 3DGS convention, degree 0..3.
 * degree < 0 switches it off (the gs_gaussian3d colours again).  Degree 0
 * gives the scene preparation's own colour bit for bit.  Not parity-pinned by
 * the reference (it never evaluates SH); the oracle restates the same fp32
 * operations (or_sh_colours). */
int gs_set_sh(gs_renderer* r, const float* f_dc, const float* f_rest, size_t n, int degree);
/* ABI 8: move a single-GPU renderer's contiguous band to tile rows
 * [row_begin, row_end), padded to pad_rows tile rows in the BGR8 band (0 =
 * no padding past the band).  The renderer must have been created with at
 * least that many rows (band_row_begin/end or band_pad_rows) -- e.g. the whole
 * frame, then moved per frame to a work-balanced split, as the row-band group
 * does for its members.  A frame still in flight is completed first (its
 * results stay readable).  GS_EINVAL for a group handle or rows outside the
 * renderer's capacity. */
int gs_set_band_rows(gs_renderer* r, uint32_t row_begin, uint32_t row_end, uint32_t pad_rows);
/* HIP stream (hipStream_t as void*) the frame is enqueued on; NULL = the
 * renderer's own stream. */
int gs_set_stream(gs_renderer* r, void* hip_stream);
/* The HIP stream frames are currently enqueued on (the renderer's own
 * non-blocking stream unless gs_set_stream chose another), e.g. to order a
 * caller's copy or collective after the frame. */
int gs_get_stream(gs_renderer* r, void** hip_stream);

/* ------------------------------------------------------------ execute */
/* Replaces GraphManager::execute -> IpuSplatter::execute (ipu_rasteriser.cpp:
 * 408-420): synchronous.  Grows the pair capacity and re-renders on overflow. */
int gs_render(gs_renderer* r);
/* Enqueue one frame on the stream and return; gs_sync waits and reports
 * GS_EOVERFLOW if the capacity was exceeded by any frame since the last
 * gs_sync (then call gs_render).  Row-band groups: collective, see
 * gs_create_rank. */
int gs_render_async(gs_renderer* r);
int gs_sync(gs_renderer* r);

/* ------------------------------------------------------------ outputs */
/* Replaces IpuSplatter::getFrameBuffer (ipu_rasteriser.cpp:131-144): 8-bit
 * BGR, row-major, band_rows x width x 3 (the full H x W x 3 for one band). */
int gs_read_bgr8(gs_renderer* r, uint8_t* dst, size_t bytes);
/* The f32 RGBA framebuffer the reference streams out (frame_buffer,
 * ipu_rasteriser.cpp:398) in either layout. */
int gs_read_rgba32f(gs_renderer* r, float* dst, size_t n_floats, int layout);
/* Replaces IpuSplatter::getIPUHistogram (ipu_rasteriser.cpp:104-106): per
 * tile render-list length of the last completed frame (thread-safe). */
int gs_read_tile_histogram(gs_renderer* r, uint32_t* dst, size_t n);
int gs_get_stats(gs_renderer* r, gs_frame_stats* st);
/* Parity/debug: tile_start (n_tiles+1 entries) and the depth-sorted per-tile
 * Gaussian index lists (n_pairs entries, 0-based Gaussian indices). */
int gs_read_bins(gs_renderer* r, uint64_t* tile_start, size_t n_start, uint32_t* list,
                 size_t n_list);
/* Parity/debug: per-Gaussian projection: mean2d[2], conic[4] (w = opacity or 0),
 * clip z, radius, rect[4] (tx0,ty0,tx1,ty1; empty if tx0 > tx1) as floats:
 * 12 floats per Gaussian. */
int gs_read_projected(gs_renderer* r, float* dst, size_t n_floats);
/* Device pointer of this band's BGR8 output (band_rows_padded x width x 3)
 * and its padded byte size, for an in-place RCCL all-gather. */
int gs_bgr8_device(gs_renderer* r, void** dev_ptr, size_t* bytes);
/* Enqueue a device-to-device copy of the band's BGR8 (padded) into dst. */
int gs_copy_bgr8_device(gs_renderer* r, void* dst_dev, size_t bytes);
/* Frames enqueued from now on write their (padded) BGR8 band straight into
 * dst_dev (>= the padded band bytes; NULL = the renderer's own buffer), e.g.
 * a slot of a caller's all-gather buffer: no copy.  The caller orders its
 * reads of dst_dev after the frame (gs_get_stream).  gs_read_bgr8 and
 * gs_copy_bgr8_device read the last frame's destination. */
int gs_set_bgr8_target(gs_renderer* r, void* dst_dev, size_t bytes);
/* Average device milliseconds per launch of each kernel (GS_K_*) over the
 * frames since the last reset (requires GS_FLAG_PROFILE). */
int gs_kernel_times(gs_renderer* r, double* avg_ms, uint64_t* launches, int n);
int gs_reset_kernel_times(gs_renderer* r);
/* Record the stage events on every `every`-th frame only (default 1): each
 * event costs device time, so throughput runs sample. */
int gs_set_profile_interval(gs_renderer* r, uint32_t every);

/* ------------------------------------------------------------ host-side data path */
/* PLY / XYZ ingest (src/splat/file_io.cpp:11-77): all 14 3DGS properties are
 * required for .ply (fillPlyProperties); f_rest_* are kept when present. */
typedef struct gs_ply gs_ply;
int gs_ply_load(const char* path, gs_ply** out);
int gs_ply_save(const gs_ply* p, const char* path);
void gs_ply_free(gs_ply* p);
int64_t gs_ply_count(const gs_ply* p);
int gs_ply_has(const gs_ply* p, const char* name);
int gs_ply_get(const gs_ply* p, const char* name, float* dst, size_t n);

/* Seeded synthetic scene (SURVEY §8 d): xoshiro256** PRNG. */
typedef struct gs_synth_params {
  uint64_t n;
  uint64_t seed;
  int32_t sh_degree;          /* 0 or 3 (45 f_rest)                      */
  float bb_min[3], bb_max[3]; /* uniform positions inside this box       */
  float log_scale_mu, log_scale_sigma;
  float opacity_lo, opacity_hi;
  const float* cluster_xyz;   /* optional: positions resampled from these */
  uint64_t n_cluster;         /*   points with N(0, cluster_sigma) jitter */
  float cluster_sigma;
} gs_synth_params;
int gs_synth_params_init(gs_synth_params* sp);
int gs_ply_synthetic(const gs_synth_params* sp, gs_ply** out);

/* Scene preparation of the render server (splat.cpp:83-163): centre the
 * bounding box, negate z, colour = max(SH_C0 * f_dc + 0.5, 0), raw opacity,
 * raw log-scale, raw rotation, gid = i + 1.  bb_out = min[3], max[3] of the
 * centred points (may be NULL). */
int gs_scene_prepare(const gs_ply* p, gs_gaussian3d* out, size_t n, float* bb_out);

/* The render server's `--device cpu` path (src/splat/cpu_rasteriser.cpp:9-92,
 * splat.cpp:250-256): the reference's CPU POINT splatter, not a Gaussian
 * rasteriser and not a fallback of gs_render.  Projects every point with
 * projection * view (row-major wire matrices), adds `value` (the reference:
 * 25) to the three channels of its pixel of the W x H BGR8 image (saturating;
 * the caller zeroes the image per frame, splat.cpp:247), counts the points
 * that land in the image (*splatted) and, if tile_hist is not NULL, per tile
 * of the (W / tile_w) x (H / tile_h) grid (buildTileHistogram).  nthreads <= 0:
 * all hardware threads. */
int gs_cpu_point_splat(const float* xyz, size_t n, const float* view_rm, const float* proj_rm,
                       uint32_t width, uint32_t height, uint32_t tile_w, uint32_t tile_h, uint8_t value,
                       uint8_t* bgr, uint32_t* tile_hist, uint32_t* splatted, int nthreads);

/* ------------------------------------------------------------ camera (glm, column-major) */
int gs_mat4_mul(const float* a, const float* b, float* out);
int gs_mat4_mul_vec4(const float* m, const float* v, float* out);
int gs_mat4_transpose(const float* m, float* out);
int gs_cam_look_at(const float* eye, const float* center, const float* up, float* out);
int gs_cam_frustum(float l, float r, float b, float t, float n, float f, float* out);
/* splat::fitFrustumToBoundingBox (src/splat/geometry.cpp:9-24) */
int gs_cam_fit_frustum(const float* bb_min, const float* bb_max, float fov, float aspect,
                       float* out);
/* splat::lookAtBoundingBox (src/splat/camera.cpp:10-15) */
int gs_cam_look_at_bbox(const float* bb_min, const float* bb_max, const float* up, float scale,
                        float* out);
int gs_cam_rotate(const float* m, float angle_rad, const float* axis, float* out);
int gs_cam_translate(const float* m, const float* v, float* out);
/* The hard-coded first-frame view `mvpStart` (splat.cpp:235-241). */
int gs_cam_mvp_start(float* out);
/* The headless camera of the render server (splat.cpp:186-199,235-244):
 * view = mvpStart, projection = fitFrustumToBoundingBox(bb in camera space,
 * fov, width/height).  Outputs are ROW-MAJOR (ready for gs_set_view/projection). */
int gs_cam_headless(const float* bb6, uint32_t width, uint32_t height, float fov,
                    float* view_rm, float* proj_rm);

/* ------------------------------------------------------------ test hooks
 * ABI 12.  For the parity tests only: process-wide values that gs_create
 * reads, so a small scene reaches a path that otherwise needs a large one.
 * No environment variable selects a kernel or a path: a production caller
 * that never calls this gets the documented automatic choices.
 *   "bin_chunk_size"  Gaussians per binning chunk (0 = automatic): small
 *                     chunks reach the > 256-chunk column scan at 120 k
 *                     Gaussians instead of 16.7 M
 *   "bin_agg"         -1 = automatic; 0 = row bands bin with the chunked
 *                     passes too (the path of bands wider than 16 384 tiles)
 *   "debug_poison"    1 = every device buffer starts as 0xA5 bytes instead
 *                     of zeros (reads of memory no stage wrote show up)
 *   "cov_cache"       -1 = automatic; 0 = no 3D covariance cache (the
 *                     projection computes them from the rotation and the
 *                     scales every frame: the path a failed cache
 *                     allocation takes)
 * Returns GS_EINVAL for an unknown key or value. */
int gs_test_set(const char* key, int64_t value);

#ifdef __cplusplus
}
#endif

#endif /* GSPLAT_H */
