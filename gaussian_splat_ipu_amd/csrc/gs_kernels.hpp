// gs_kernels.hpp -- launch interface of the HIP kernels of the frame path
// (project -> bin -> sort -> blend).  Internal to libgsplat.so.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsk {

// Per-frame constants, passed by value as kernel arguments.
// Timeline probe builds (-DGS_PROBE=1, tools/build_x.sh; never the
// default library): every kernel records, per frame, its first wave's start
// and its last wave's end (wall_clock64, 100 MHz), for tools/probe_timeline.py
#ifndef GS_PROBE
#define GS_PROBE 0
#endif
// (per frame and kernel, kProbeSlots (start, end) pairs: the waves spread
// their atomics over them -- one address per kernel serialised 15 k waves'
// atomics and stretched the projection 15x)
constexpr int kProbeFrames = 512, kProbeKernels = 16, kProbeSlots = 256;
// Blend lane-count builds (-DGS_LANES=1, tools/blend_lanes.py; never the
// default library): the two-pixel blend adds, per frame, its wave record
// steps, lane record steps, pixel evaluations (live pixels), the evaluations
// whose record's alpha box holds the pixel, and the hits (updates and
// breaks) into Buffers::lanes
#ifndef GS_LANES
#define GS_LANES 0
#endif

struct FrameParams {
  float mvp[16];      // proj * view, glm column-major (codelets.cpp:443)
  float tanfov;       // (float)tan(0.5 * fxy[0])   (codelets.cpp:444)
  float focal_x;      // W / (2 tanf(fxy[0]/2))    (codelets.cpp:447)
  float focal_y;
  float guard_thr;    // tb.diagonal().length() * clipSize (codelets.cpp:470)
  float scale_div;    // fxy[1]                    (codelets.cpp:463)
  float W, H;         // viewport (codelets.cpp:621)
  float tw, th;       // tile size as float (tile_config.hpp:57-71)
  int width, height;
  int tile_w, tile_h;
  int tiles_x;        // ceil(W / tw)
  int band_ty0;       // first tile row of this band (absolute)
  int band_stride;    // tile-row stride: band row k is absolute row band_ty0 + k * stride
  int band_nrows;     // tile rows in this band
  int tiles_y;        // tile rows of the whole frame
  int band_rows;      // pixel rows of this band's output
  int band_cull;      // skip Gaussians whose extent bound misses the band (GS_FLAG_BAND_CULL)
  int n;              // Gaussians
  int n_tiles;        // tiles_x * (band_ty1 - band_ty0)
  int chunks_per_tile;  // blend waves per tile (16 pixel quads each)
  int blend_bqw;        // blend wave = 4x4 quads (8x8 px) | 8x2 quads (16x4 px) | 0: quad run
  int blend_lpt;        // blend tiles longest list first (row bands), else in tile order
  int blend_seg;        // (blend_lpt, two-pixel lanes, the sort launch sorts every list) the
                        //   sort launch writes each slot's (tile, start, length), the blend
                        //   reads it in one load
  int emit_grid;        // the aggregated emit's workgroups, walking the projection blocks
  int blend_sort;       // each blend workgroup (one 16x16 tile) sorts its tile's list first: no
                        //   tile-sort launch (row bands)
  int blend_px2;        // two pixels per blend lane (16x16 tiles, whole frames without lazy lists)
  unsigned long long pair_cap;
  int write_rgba;
  int bgr_pitch;      // bytes per row of the BGR8 output
  int bin_global;     // 1: fallback binning with global atomics
  int bin_agg;        // 1: aggregated binning (per-tile counters summed by the projection's
                      //   workgroups, gs_agg_scan_kernel, gs_agg_emit_kernel): no chunk matrix
  int chunk_size;     // Gaussians per binning chunk (<= 65535)
  int n_chunks;
  int emit_wide;      // emit with one u32 LDS cursor per tile (n_tiles * 4 <= kBinLdsMax)
  int full_record;    // also write the readback-only record tail (radius, clip z)
  int pair_cull;      // bin only the tiles the alpha box meets (crect); the
                      // reference list lengths are counted alongside
  int mean_w1;        // every mean has w == 1: the projection reads mean_op (xyz + opacity,
                      //   16 B) and neither the mean nor the colour (32 B)
  int rect8;          // pair_cull with <= 256 tile columns and band rows: rect and crect hold
                      //   4 B per Gaussian, 8 bits per bound (rect8_pack)
  int big_separate;   // big lists sorted by gs_sort_big_kernel (launched before the tile sort)
  int lazy;           // big lists: only their nearest keys are sorted before the blend; the
                      //   blocks whose pixels outlive that prefix continue after a full sort
  int big_pass;       // big-list kernels: 0 = every big list; lazy continuation: 1 = the lists
                      //   flagged by the blend (window), 2 = those flagged again (full sort)
  int blend_cont;     // blend: 1 = the continuation of the flagged big-list blocks
  int count_records;  // blend: each wave writes the records it composited to blend_count
  int probe_frame;    // (GS_PROBE builds) the frame's slot in the probe ring
  int fast_exp;       // blend: hardware exp2 (GS_FLAG_FAST_EXP, within a stated tolerance)
  int sh_degree;      // > 0: view-dependent colour from spherical harmonics (gs_set_sh)
  float campos[3];    // camera position in the scene's (prepared) frame, for the SH direction
  int cov_cache;      // Buffers::cov3 holds every Gaussian's 3D covariance for this frame's
                      //   fxy[1] (gs_cov3d_kernel): the projection reads it instead of the
                      //   rotation and scales
  int pow2;           // tile size, band stride and fxy[1] are powers of two: the
                      // projection divides by them with exact multiplies / shifts
  float inv_tw, inv_th, inv_sd;  // 1 / tw, 1 / th, 1 / fxy[1]   (pow2 only)
  int sh_tw, sh_th, sh_stride;   // log2 tile_w, tile_h, band_stride (pow2 only)
  // (appended last, so the other kernels' argument offsets stay as they were)
  int bin_direct;     // (bin_agg row bands with the sort in the blend) tile t's pairs go to
                      //   [tile_start[t], tile_start[t + 1]) as the view's last scan laid
                      //   them out: the projection's workgroups place them at once (no
                      //   scan, no emit launch); the blend's workgroups read the lengths
                      //   from the tile counters, reset them, and the last one writes the
                      //   frame counters
  unsigned int frame_seq;  // the renderer's frame number (1, 2, ...): the aggregated binning's
                           //   host mirror word 15, which frame its counters are from
};

// Device workspace of one renderer.
struct Buffers {
  unsigned long long* probe;      // (GS_PROBE builds, GSPLAT_PROBE_FILE) [kProbeFrames][kProbeKernels][kProbeSlots][2] or null
  unsigned long long* lanes;      // (GS_LANES builds, GSPLAT_LANES_FILE) [8] blend counters or null
  // scene (SoA of the 64-B Gaussian3D record, ipu_geometry.hpp:305-311)
  const float4* mean;       // x y z w
  const float4* colour;     // r g b opacity
  const float4* rot;        // quaternion (w x y z)
  const float4* scale_gid;  // sx sy sz gid
  const float4* cull;       // band cull: mean xyz + largest log-scale (NaN: empty slot, inf: never culled)
  const float4* mean_op;    // mean xyz + opacity (FrameParams::mean_w1: every mean's w is 1)
  float* cov3;              // [9][n] per Gaussian: ComputeCov3D's 9 entries (m[c][r] at c * 3 + r),
                            //   SoA (FrameParams::cov_cache; static per fxy[1]); an empty slot
                            //   (gid <= 0) has m[2][2] = -1, a live one's is >= +0 or NaN
  // device order: record i is the input Gaussian perm[i] (3D Morton order by
  // default); the depth sort breaks ties by the input index, as the reference
  const uint32_t* perm;     // [n] device index -> input index
  const uint32_t* inv_perm; // [n] input index -> device index
  // per-Gaussian projection outputs
  float4* rec;              // frames: 2 x float4 (32 B): mx my k0 k2 | k1 pcut boxx boxy (the colour
                            //   is the scene's, or col_out); full_record (readback): 3 x float4
                            //   (48 B): mx my k0 k2 | k1 pcut r g | b op boxx boxy
  float4* col_out;          // [n] gs_set_sh frames: the view-dependent colour + opacity (in the
                            //   record region past the 32-B records)
  float2* rec_tail;         // radius, clip z: readback only (written with full_record)
  uint32_t* depth_key;      // order-preserving key of clip z
  uint2* rect;              // (tx0 | tx1 << 16, ty0 | ty1 << 16), band-relative rows
                            //   (rect8: a u32 per Gaussian, tx0 | tx1 << 8 | ty0 << 16 | ty1 << 24)
  uint2* crect;             // rect cut to the tiles the alpha box meets (pair_cull)
  // binning
  uint32_t* tile_count;     // [n_tiles]      (memset 0 each frame)
  unsigned long long* tile_cnt64;  // [n_tiles] aggregated binning: binned | reference << 32 per
                                   //   tile (zero between frames: the scan resets it)
  uint32_t* tile_ref;       // [n_tiles] aggregated binning: the reference list lengths (the
                            //   histogram; copied to the host mirror at sync, not per frame)
  uint32_t* tile_fb;        // [n_tiles] aggregated binning: binned pairs of the fallback
                            //   (box too wide) workgroups, placed after the aggregated ones
  uint4* agg_box;           // [ceil(n / 256)] per projection block: its box of tiles (x0, y0,
                            //   width, area; area kAggSpread = the fallback)
  uint32_t* agg_off;        // [ceil(n / 256) x kAggCap] the block's offset among each tile's
                            //   aggregated pairs (returned by the projection's reservation)
  uint32_t* tile_start;     // [n_tiles + 1]
  uint32_t* tile_cursor;    // [n_tiles]
  unsigned long long* pairs;      // [pair_cap]  (depth_key << 32 | input index)
  unsigned long long* pairs_alt;  // [pair_cap]  scratch of the large-list sort
  uint32_t* list;           // [pair_cap]  depth-sorted Gaussians (device indices)
  uint32_t* big_tiles;      // [n_tiles]  lists > kSortLdsCap (radix sort queue)
  uint32_t* big_item;       // [pair_cap / 2048 + n_tiles + 1]  segment k of the big lists -> big-list slot
  // big-list sample sort: buckets of all big lists, [pair_cap / 1024 + n_tiles + 1] each
  unsigned long long* bk_spl;  // splitters (bucket t's upper bound, t < B - 1 of its list)
  uint32_t* bk_start;       // bucket start within its list
  uint32_t* bk_cnt;         // bucket key count, then the scatter's reservation cursor
  uint32_t* bk_list;        // bucket -> big-list slot
  uint32_t* bk_off;         // [n_tiles + 1]  big-list slot -> first bucket
  uint32_t* medium_tiles;   // [n_tiles]  lists in (kSortRegCap, kSortLdsCap] (block sort queue)
  uint32_t* small_tiles;    // [n_tiles]  lists in [0, kSortRegCap] (one-wave sort queue)
  uint4* blend_seg;         // [n_tiles]  (tile, list start, list length, 0) in the blend's
                            //   longest-first slot order, written by the sort launch
                            //   (FrameParams::blend_seg)
  uint32_t* chunk_off;      // [n_chunks][n_tiles] chunk histograms -> offsets
  uint4* tile_agg;          // [2 * ceil(n_tiles / 64)] per 64 tiles: list-length sum (lo, hi),
                            //   small | medium << 8 | big << 16 counts, max length;
                            //   then the reference list-length sum (lo, hi), 0, 0
  uint32_t* block_rendered; // [ceil(n / 256)] V per project workgroup
  uint32_t* host_counters;  // mapped pinned mirror of counters[16] + tile_count[n_tiles],
                            //   written by the chunked scan (no D2H copy per frame)
  uint32_t* host_sticky;    // mapped pinned word: set by the scan of any frame that
                            //   overflowed the pair capacity, cleared by the host at sync
  uint32_t* counters;       // [16]: 0 n_big, 1 big_next, 2 n_rendered, 3 overflow,
                            //  4 max_list, 5 n_pairs (low), 6 n_pairs (high),
                            //  7 n_medium, 8 medium_next, 9 n_small,
                            //  10 / 11 reference pairs (low / high: unculled lists),
                            //  12 big-list work items, 13 longest big list, 14 big-list buckets
  // outputs
  float4* rgba;             // band_rows x width, row-major
  uint8_t* bgr;             // band rows (padded) x width x 3
  // lazy big lists (FrameParams::lazy); all per tile / per big-list slot
  uint32_t* tile_big;       // [n_tiles] big-list slot of a tile (~0: not a big list)
  uint32_t* big_len;        // [n_tiles] keys sorted before the blend (the prefix)
  uint32_t* big_thr;        // [n_tiles] the prefix's depth bound (keys of lower depth)
  uint32_t* big_cnt;        // [n_tiles] keys below the bound
  uint32_t* big_flag;       // [n_tiles] 1: a pixel outlived the prefix (continuation)
  uint32_t* cont_flag;      // [n_tiles * 4] per slot and blend wave: its state is saved
  float* cont_state;        // [n_tiles * 4 * 6 * 64] T, colour, done of the saved waves
  uint2* cont_box;          // [n_tiles * 4] per slot and blend wave: the saved live pixels' box
                            //   (x0 | x1 << 16, y0 | y1 << 16)
  uint32_t* cont_len;       // [n_tiles] keys the continuation walks (the list's keys past the
                            //   prefix whose alpha box meets its live pixels, sorted)
  // the continuation's window (pass 1): keys of depth in [big_thr, big_thr2), kept unsorted at
  // the end of the list's pairs_alt region by the prefix select
  uint32_t* big_thr2;       // [n_tiles] the window's depth bound (~0: to the end of the list)
  uint32_t* big_cnt2;       // [n_tiles] keys in the window
  uint32_t* big_flag2;      // [n_tiles] 1: a pixel outlived the window too (full sort, pass 2)
  uint32_t* cont_full;      // [n_tiles] 1: the window's sorted keys are the rest of the list
  uint32_t* cont_thr;       // [n_tiles] pass 2 takes the keys of depth >= this
  uint32_t* footer;         // row-band group: counters[16] + reference list lengths[n_tiles]
                            //   of this frame, next to its BGR8 band in the all-gather slot
                            //   (written by the chunked scan; nullptr = none)
  uint32_t* blend_count;    // [n_tiles * chunks_per_tile] records each blend wave staged
  uint32_t* blend_count_cont;  //   ... and each continuation wave (GS_FLAG_PROFILE frames only)
  const float* sh;          // gs_set_sh: [16 coefficients x 3 channels][n] (coefficient-major, device
                            //   order): DC then f_rest 1..15 per channel (nullptr = off)
  uint32_t* group_sticky;   // row-band group: one device word per GPU, set by the scan of any
                            //   frame of any of its band renderers that overflowed; copied into
                            //   footer word kFootSticky before each all-gather (nullptr = none)
  uint32_t* dir_word;       // (bin_direct) [2]: the blend workgroups' ticket, a tile segment's
                            //   overflow flag (both reset by the frame's last blend workgroup)
};

// footer word that carries the group's sticky overflow bit (counters[15] is unused)
constexpr int kFootSticky = 15;

constexpr int GS_STAGE_EVENTS = 7;  // profile events: before project .. after blend, after the continuation
constexpr int kSortLdsCap = 2048;  // largest tile list sorted by one workgroup (registers + LDS)
constexpr uint32_t kSortRegCap = 256;  // largest tile list sorted in the registers of one wave
constexpr size_t kBinLdsMax = 160 * 1024;  // LDS of one CU: chunk histograms up to 81920 tiles
constexpr int kAggCap = 512;  // aggregated binning: tiles of a projection block's LDS box

size_t bin_lds_bytes(int n_tiles);
bool bin_lds_fits(int n_tiles);
hipError_t init_kernel_attributes();

// the projection's instantiation for fp: 1 = a whole frame's lean one
// (gs_project), 2 = a row band's (gs_project_band), 3 = a direct-binned
// band's (gs_project_direct), 0 = every path (gs_project_any)
int project_kind(const FrameParams& fp, const Buffers& b);
void launch_project(const FrameParams& fp, const Buffers& b, hipStream_t s);
// the 3D covariances of the scene for fp's fxy[1] into Buffers::cov3
void launch_cov3d(const FrameParams& fp, const Buffers& b, hipStream_t s);
void launch_scan(const FrameParams& fp, const Buffers& b, hipStream_t s);
void launch_emit(const FrameParams& fp, const Buffers& b, hipStream_t s);
void launch_sort(const FrameParams& fp, const Buffers& b, hipStream_t s);
// launch_sort's two independent halves: the big lists (big_separate) and the others
void launch_sort_big(const FrameParams& fp, const Buffers& b, hipStream_t s);
void launch_sort_tiles(const FrameParams& fp, const Buffers& b, hipStream_t s);
void launch_blend(const FrameParams& fp, const Buffers& b, hipStream_t s);
// lazy big lists: the full sort of the lists the blend flagged + the continued blend (no-op otherwise)
void launch_blend_cont(const FrameParams& fp, const Buffers& b, hipStream_t s);
// *dst = *src, one word, ordered on stream s (the group's sticky bit into a footer)
void launch_copy_word(hipStream_t s, uint32_t* dst, const uint32_t* src);

// ---- the lattice-migration emulator (gs_lattice.hip, GS_FLAG_LATTICE)
constexpr int kLatChan = 75;        // records per channel (edge_builder.cpp:18, ipu_rasteriser.cpp:307-308)
constexpr int kLatExtra = 600;      // extra vertsIn slots per tile (ipu_rasteriser.cpp:309)
constexpr int kLatMaxSlots = 2048;  // vertsIn slots of one tile the kernel's LDS holds

struct LatticeParams {
  float mvp[16];
  float tanfov, focal_x, focal_y, guard_thr, scale_div;
  float W, H, tw, th;
  float across;       // TiledFramebuffer::numTilesAcross (a float)
  int width, height, tile_w, tile_h, tiles_x, n_tiles;
  int gpt, rem;       // records per tile of the initial distribution, extra records of the last tile
  int parity;         // this frame writes out-channel set `parity`, reads the other
  int write_rgba;
  int bgr_pitch;
};

struct LatticeBufs {
  float4* slots;      // vertsIn: every tile's slots (tile t from t * (gpt + 600)), 4 float4 (Gaussian3D) each
  float4* chan;       // out-channels [2][T][4 directions][75 slots][4]
  float4* zbuf;       // z-buffer (persistent): 3 float4 per entry: colour | cov a b c, z | mean x y
  float4* zscratch;   // the sort's permutation scratch (same size)
  uint32_t* splatted; // [T] the reference's splatted counter (kept while a tile renders nothing)
  uint32_t* tile_stat;  // [T][4] render list, dropped, failed sends, z-buffer overruns (last frame)
  float4* rgba;       // row-major W x H
  uint8_t* bgr;
  uint32_t* host_counters;  // mapped: counters[16] + splatted[T]
};

void launch_lattice(const LatticeParams& lp, const LatticeBufs& lb, hipStream_t s);

}  // namespace gsk
