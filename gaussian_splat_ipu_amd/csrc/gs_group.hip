// gs_group.hip -- the row-band group behind one C ABI handle (SURVEY §8 b/e):
// the framebuffer's tile rows are split into contiguous bands, one per GPU;
// every GPU renders its band (project -> bin -> sort -> blend, gs_kernels.hip)
// and every frame ends with ONE all-gather of the BGR8 bands over RCCL.  This
// replaces the reference's single-IPU execute (ipu_rasteriser.cpp:408-420,
// splat.cpp:257-265), which has no multi-device path.
//
// Two ways to form a group:
//   * gs_create with cfg->num_gpus = G: one process drives G devices
//     (ncclCommInitAll; one host thread per device enqueues its band and then,
//     once every band is enqueued, its own ncclAllGather);
//   * gs_create_rank: one process per GPU (ncclCommInitRank from an id rank 0
//     made), as torchrun launches bench.py.
//
// Per frame, each rank's all-gather slot holds its padded BGR8 band followed
// by a footer: the band's frame counters and reference tile-list lengths.
// After the gather every rank holds every band's footer, so every rank derives
// the same next split from the same numbers (no extra collective) and reports
// the whole frame's histogram.  Overflow is decided from the footers too (the
// frame's own bit, and a per-GPU sticky bit copied into the footer before the
// gather that covers every frame since the last gs_sync), so gs_sync returns
// the same status on every rank and a blocking gs_render re-renders on every
// rank or on none (decide(), exported as gs_group_decide).
//
// Contract (gsplat.h): gs_render, gs_render_async and gs_sync are collective
// -- every rank calls them for the same frames, in the same order.  The
// readbacks are local: they wait for this rank's frames but change neither the
// split nor the overflow state.
//
// Frames in flight: F band renderers per device take frames round-robin, each
// on its own stream; the all-gathers run in frame order on one communication
// stream per device.  gs_render_async never waits: the split is re-balanced
// every kRebalanceEvery frames from the footers of the frame half that many
// frames back (copied to the host when it was enqueued), the same frame on
// every rank; a blocking gs_render re-balances from its own frame.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gsplat.h"
#include "gs_internal.hpp"
#include "gs_kernels.hpp"
#include "host/gs_host.hpp"

using gsh::set_error;

namespace gsg {

namespace {

constexpr double kTileCost = 128.0;  // fixed work per tile of a row, in pairs (dist.row_work)
constexpr double kRebalanceGain = 0.97;  // switch splits only if the slowest band gains > 3 %
constexpr uint64_t kRebalanceEvery = 8;  // frames between re-balancing decisions
constexpr int kMaxInFlight = 8;

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// RCCL is bound at run time, on first use: the librccl.so.1 already in the
// process (e.g. the one torch loaded) if there is one, else $GSPLAT_RCCL, else
// ROCm's.  Linking it would pull a second ROCm runtime stack into processes
// that load torch's after libgsplat.
struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclCommCount) CommCount = nullptr;  // (optional: the info call only)
  std::string error;
};

const Rccl& rccl() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h)
      if (const char* p = std::getenv("GSPLAT_RCCL")) h = dlopen(p, RTLD_NOW);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!h) {
      const char* e = dlerror();
      R.error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return;
    }
    bool ok = true;
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
      ok = ok && f != nullptr;
    };
    sym(R.GetUniqueId, "ncclGetUniqueId");
    sym(R.CommInitRank, "ncclCommInitRank");
    sym(R.CommInitAll, "ncclCommInitAll");
    sym(R.CommDestroy, "ncclCommDestroy");
    sym(R.AllGather, "ncclAllGather");
    sym(R.GroupStart, "ncclGroupStart");
    sym(R.GroupEnd, "ncclGroupEnd");
    sym(R.GetErrorString, "ncclGetErrorString");
    R.CommCount = reinterpret_cast<decltype(&ncclCommCount)>(dlsym(h, "ncclCommCount"));
    if (!ok) {
      R.error = "librccl.so.1 lacks an RCCL entry point";
      R.GetUniqueId = nullptr;
    }
  });
  return R;
}

int rccl_check() {
  if (rccl().GetUniqueId) return GS_OK;
  set_error(rccl().error);
  return GS_EDEVICE;
}

}  // namespace

struct Member {
  int device = 0;
  int rank = 0;                       // the band this member renders
  std::vector<gs_renderer*> slot;     // F band renderers (each its own stream)
  hipStream_t comm_stream = nullptr;  // all-gathers, in frame order
  ncclComm_t comm = nullptr;
  // F x world x slot_cap: the gathered frames.  The band renders straight
  // into its own part of the slot (rank x the frame's bytes per rank) and
  // the all-gather runs in place (sendbuff = recvbuff + rank x count): no
  // send buffer, no local copy of the band
  uint8_t* d_recv = nullptr;
  std::vector<hipEvent_t> ev_render;    // per slot: the band is rendered
  std::vector<hipEvent_t> ev_gathered;  // per slot: the all-gather has read this member's part
  // set by the scan of any of this GPU's band frames that overflowed since
  // the last sync; copied into footer word kFootSticky before every gather
  uint32_t* d_sticky = nullptr;
  // GS_FLAG_PROFILE, per slot: before the band's first kernel, after its last
  // (both on the band renderer's stream) and after the all-gather (comm stream)
  std::vector<hipEvent_t> ev_t0, ev_t1, ev_t2;
  double band_ms = 0.0, gather_ms = 0.0;  // summed over timed_n frames
  uint64_t timed_n = 0;
  // the status of this member's part of the last frame (worker thread)
  int rc = GS_OK;
  std::string err;
};

// One frame's decisions, the same for every member (enqueue -> the members)
struct FrameCmd {
  int i = 0;             // slot
  int pad = 0;           // padded band tile rows
  size_t bgr_part = 0;   // bytes of the padded BGR8 band
  size_t bytes = 0;      // bytes per rank of the all-gather
  bool was_used = false;  // the slot held an earlier frame (its gather must be done)
  bool timed = false;     // per-member events
  int prev = -1;          // the previous frame's slot (-1: none)
};

struct SlotInfo {
  bool used = false;
  bool gather_timed = false;
  uint64_t frame = 0;
  std::vector<uint32_t> bounds;  // world + 1 tile-row bounds of the frame
  int pad_rows = 0;
  size_t bgr_part = 0;  // bytes of the padded BGR8 band (256-aligned)
  size_t bytes = 0;     // bytes per rank of the all-gather
};

struct Group {
  gs_config cfg{};
  int world = 1, F = 1;
  bool rccl = true;
  bool multi_process = false;
  bool rebalance = true;
  bool profile = false;
  int W = 0, H = 0, tw = 0, th = 0, tiles_x = 0, tiles_y = 0, T = 0;
  size_t n = 0;
  size_t slot_cap = 0;     // bytes per rank per slot (the full frame's band + footer)
  size_t foot_words = 0;   // 16 + T
  std::vector<Member> mem;
  std::vector<uint32_t> bounds;  // split of the next frame
  std::vector<SlotInfo> sinfo;
  uint32_t* h_snap = nullptr;    // pinned: world x foot_words, a frame's footers for re-balancing
  uint32_t* h_last = nullptr;    // pinned: world x foot_words, the last frame's (read at sync)
  hipEvent_t ev_snap = nullptr;  // the snapshot's copy is done (mem[0].comm_stream)
  bool snap_pending = false;
  std::vector<uint32_t> snap_bounds;
  uint64_t frame = 0;
  int last_slot = -1;
  bool last_read = false;
  int last_status = GS_OK;   // the decision of the last frame's footers (repeated syncs return it)
  uint64_t need_pairs = 0;   // the largest band list of the last frame's footers
  uint64_t pair_cap = 0;     // the group's pair capacity per band renderer (the same on every rank)
  float view[16], proj[16];
  float fov = 0.6981317f, sd = 0.1f;
  // the last frame whose footers were read
  std::mutex hist_mu;
  std::vector<uint32_t> hist;
  gs_frame_stats stats{};
  // gather timing (GS_FLAG_PROFILE): member 0's all-gather (GS_K_GATHER)
  uint32_t profile_every = 1;
  double g_ms = 0.0;
  uint64_t g_n = 0;
  uint64_t rebalances = 0;
  int comm_ranks = -1;  // ncclCommCount of member 0's communicator (-1: copy gather)
  // one process driving several devices: members 1.. enqueue their band and
  // its all-gather on host threads of their own, beside member 0 on the
  // caller's thread, so a frame's host time is the slowest member's, not the
  // sum (eight bands of ~20 us of launches each would otherwise cost more host
  // time per frame than the GPUs take to render it)
  bool threaded = false;
  std::vector<std::thread> workers;
  FrameCmd cmd;                       // the posted frame
  std::atomic<uint64_t> post_seq{0};  // frames posted
  std::atomic<uint32_t> done{0};      // workers finished with the posted frame's band
  // phase 2 of a threaded frame: once every member's band is enqueued, the
  // caller posts the verdict (gather_seq = the frame's post_seq); the
  // workers issue their all-gathers only if every band succeeded, so a
  // failed member never leaves the others' collectives half-issued
  std::atomic<uint64_t> gather_seq{0};
  std::atomic<bool> gather_ok{false};
  std::atomic<uint32_t> gathered{0};  // workers past phase 2 of the posted frame
  // a frame failed in one member after others had issued device work for it:
  // the group refuses further frames (gs_destroy still releases it)
  bool failed = false;
  std::atomic<int> sleepers{0};
  std::atomic<bool> stop{false};
  std::mutex wmu;
  std::condition_variable wcv;
};

void balanced_bands(const double* work, int rows, int world, uint32_t* bounds) {
  std::vector<double> c((size_t)rows + 1, 0.0);
  for (int i = 0; i < rows; ++i) c[i + 1] = c[i] + work[i];
  bounds[0] = 0;
  for (int k = 1; k < world; ++k) {
    const double target = c[rows] * k / world;
    int b = (int)(std::lower_bound(c.begin(), c.end(), target) - c.begin());
    if (b > 0 && std::fabs(c[b - 1] - target) <= std::fabs(c[std::min(b, rows)] - target)) b -= 1;
    b = std::max((int)bounds[k - 1] + 1, std::min(b, rows - (world - k)));
    bounds[k] = (uint32_t)b;
  }
  bounds[world] = (uint32_t)rows;
}

namespace {

double max_band_work(const std::vector<double>& w, const std::vector<uint32_t>& b) {
  double mx = 0.0;
  for (size_t r = 0; r + 1 < b.size(); ++r) {
    double s = 0.0;
    for (uint32_t y = b[r]; y < b[r + 1]; ++y) s += w[y];
    mx = std::max(mx, s);
  }
  return mx;
}

int set_dev(int d) {
  hipError_t e = hipSetDevice(d);
  return e == hipSuccess ? GS_OK : gsr::hip_fail(e, "hipSetDevice");
}

int nccl_fail(ncclResult_t r, const char* what) {
  set_error(std::string(what) + ": " + rccl().GetErrorString(r));
  return GS_EDEVICE;
}

#define GS_NCCL(call)                                   \
  do {                                                  \
    ncclResult_t r_ = (call);                           \
    if (r_ != ncclSuccess) return nccl_fail(r_, #call); \
  } while (0)

}  // namespace

// Every decision the group takes is a function of ONE gathered frame's
// footers (world x foot_words at h; `frame_bounds` = that frame's split), the
// same bytes on every rank, so every rank takes the same decision without a
// collective of its own:
//   * the status: GS_EOVERFLOW iff some band's frame overflowed (word 3) or
//     some band's GPU had an overflowing frame since its last sync (word
//     kFootSticky, the group's sticky bit copied in before the gather);
//   * need_pairs: the longest band pair list of the frame (capacity growth);
//   * next_bounds: the split of later frames (cur_bounds unless re-balancing
//     lowers the slowest band's work by more than 3 %; never after overflow);
//   * with `hist` / `st`: the whole frame's histogram and stats.
// The blocking contract it serves: IpuSplatter::execute, ipu_rasteriser.cpp:408-420.
int decide(const uint32_t* h, size_t foot_words, int world, int tiles_x, int tiles_y,
           const uint32_t* frame_bounds, const uint32_t* cur_bounds, bool rebalance, bool chunked,
           uint32_t* next_bounds, uint64_t* need_pairs, std::vector<uint32_t>* hist_out, gs_frame_stats* st) {
  const size_t T = (size_t)tiles_x * tiles_y;
  bool ovf = false;
  uint64_t P = 0, Pb = 0, V = 0, nbig = 0, need = 0;
  std::vector<uint32_t> hist(T, 0u);
  for (int r = 0; r < world; ++r) {
    const uint32_t* f = h + (size_t)r * foot_words;
    ovf = ovf || f[3] != 0 || f[gsk::kFootSticky] != 0;
    const uint64_t pb = (uint64_t)f[5] | ((uint64_t)f[6] << 32);
    Pb += pb;
    need = std::max(need, pb);
    P += chunked ? ((uint64_t)f[10] | ((uint64_t)f[11] << 32)) : pb;
    V = std::max<uint64_t>(V, f[2]);
    nbig += f[0];
    const size_t t0 = (size_t)frame_bounds[r] * tiles_x, t1 = (size_t)frame_bounds[r + 1] * tiles_x;
    if (t1 > t0 && t1 <= T && 16 + (t1 - t0) <= foot_words) std::memcpy(hist.data() + t0, f + 16, (t1 - t0) * 4);
  }
  if (need_pairs) *need_pairs = need;
  if (next_bounds) {
    std::copy(cur_bounds, cur_bounds + world + 1, next_bounds);
    if (rebalance && world > 1 && !ovf) {
      std::vector<double> w((size_t)tiles_y, 0.0);
      for (int y = 0; y < tiles_y; ++y) {
        double sum = 0.0;
        for (int x = 0; x < tiles_x; ++x) sum += hist[(size_t)y * tiles_x + x];
        w[y] = sum + kTileCost * tiles_x;
      }
      std::vector<uint32_t> nb((size_t)world + 1), cb(cur_bounds, cur_bounds + world + 1);
      balanced_bands(w.data(), tiles_y, world, nb.data());
      if (nb != cb && max_band_work(w, nb) < kRebalanceGain * max_band_work(w, cb))
        std::copy(nb.begin(), nb.end(), next_bounds);
    }
  }
  if (st) {
    uint32_t mx = 0;
    for (uint32_t v : hist) mx = std::max(mx, v);
    st->n_rendered = V;
    st->n_pairs = P;
    st->n_pairs_binned = Pb;
    st->max_list = mx;
    st->n_big_tiles = (uint32_t)nbig;
  }
  if (hist_out) hist_out->swap(hist);
  return ovf ? GS_EOVERFLOW : GS_OK;
}

namespace {

// The footers of one gathered frame: its status, and with `stats` the whole
// frame's histogram and stats (gs_get_stats / gs_read_tile_histogram); with
// `split`, the split of later frames.  Only called where every rank calls it
// for the same frame: at the frame indices of the re-balancing snapshot
// (enqueue), in a blocking gs_render, and in gs_sync (status and stats only).
int parse_footers(Group* g, const uint32_t* h, const std::vector<uint32_t>& bounds, bool stats, bool split) {
  const bool chunked = !g->mem[0].slot[0]->bin_global && g->mem[0].slot[0]->n_chunks > 0;
  std::vector<uint32_t> nb((size_t)g->world + 1), hist;
  gs_frame_stats st{};
  uint64_t need = 0;
  const int rc = decide(h, g->foot_words, g->world, g->tiles_x, g->tiles_y, bounds.data(), g->bounds.data(),
                        split && g->rebalance, chunked, nb.data(), &need, stats ? &hist : nullptr,
                        stats ? &st : nullptr);
  if (split && nb != g->bounds) {
    g->bounds = nb;
    g->rebalances += 1;
  }
  if (stats) {
    g->need_pairs = need;
    std::lock_guard<std::mutex> lk(g->hist_mu);
    g->hist.swap(hist);
    g->stats.n_rendered = st.n_rendered;
    g->stats.n_pairs = st.n_pairs;
    g->stats.n_pairs_binned = st.n_pairs_binned;
    g->stats.max_list = st.max_list;
    g->stats.n_big_tiles = st.n_big_tiles;
    g->stats.paths = st.paths;
  }
  return rc;
}

// every band's footer of the frame in slot i -> h (one strided copy on s)
int copy_footers(Group* g, int i, uint32_t* h, hipStream_t s, bool async) {
  const SlotInfo& si = g->sinfo[i];
  const uint8_t* src = g->mem[0].d_recv + (size_t)i * g->world * g->slot_cap + si.bgr_part;
  const size_t width = (16 + (size_t)si.pad_rows * g->tiles_x) * 4;
  if (async)
    GS_HIP(hipMemcpy2DAsync(h, g->foot_words * 4, src, si.bytes, width, (size_t)g->world, hipMemcpyDeviceToHost, s));
  else
    GS_HIP(hipMemcpy2D(h, g->foot_words * 4, src, si.bytes, width, (size_t)g->world, hipMemcpyDeviceToHost));
  return GS_OK;
}

// Per-member event timings of the frame in slot i (GS_FLAG_PROFILE frames):
// band = its first kernel -> its last; gather = band written -> frame
// gathered.  block: wait for the events (else a frame still running is
// skipped).
int harvest_timing(Group* g, int i, bool block) {
  SlotInfo& si = g->sinfo[i];
  if (!si.gather_timed) return GS_OK;
  si.gather_timed = false;
  for (Member& m : g->mem) {
    int rc = set_dev(m.device);
    if (rc != GS_OK) return rc;
    if (!block && hipEventQuery(m.ev_t2[i]) != hipSuccess) return GS_OK;
  }
  for (size_t k = 0; k < g->mem.size(); ++k) {
    Member& m = g->mem[k];
    int rc = set_dev(m.device);
    if (rc != GS_OK) return rc;
    float band = 0.0f, gather = 0.0f;
    GS_HIP(hipEventSynchronize(m.ev_t2[i]));
    GS_HIP(hipEventElapsedTime(&band, m.ev_t0[i], m.ev_t1[i]));
    GS_HIP(hipEventElapsedTime(&gather, m.ev_t1[i], m.ev_t2[i]));
    m.band_ms += band;
    m.gather_ms += gather;
    m.timed_n += 1;
    if (k == 0) {
      g->g_ms += gather;
      g->g_n += 1;
    }
  }
  return GS_OK;
}

// member m's part of the frame's all-gather slot: its band and footer,
// at rank x the frame's bytes per rank
inline uint8_t* own_part(const Group* g, const Member& m, const FrameCmd& f) {
  return m.d_recv + (size_t)f.i * g->world * g->slot_cap + (size_t)m.rank * f.bytes;
}

// Member m's band of the frame f: moved to the frame's split, rendered on
// its band renderer's stream into its all-gather send slot.
int member_render(Group* g, Member& m, const FrameCmd& f) {
  int rc = set_dev(m.device);
  if (rc != GS_OK) return rc;
  gs_renderer* c = m.slot[f.i];
  if ((rc = gsr::set_band_rows(c, (int)g->bounds[m.rank], (int)g->bounds[m.rank + 1], f.pad)) != GS_OK) return rc;
  std::memcpy(c->view_rm, g->view, sizeof(g->view));
  std::memcpy(c->proj_rm, g->proj, sizeof(g->proj));
  c->fov = g->fov;
  c->scale_div = g->sd;
  c->bgr_target = own_part(g, m, f);
  c->buf.footer = (uint32_t*)(c->bgr_target + f.bgr_part);
  // the gather of frame k - F read this part of the slot (the copy gather:
  // every member's comm stream read it)
  if (f.was_used) {
    if (g->rccl) {
      GS_HIP(hipStreamWaitEvent(c->stream, m.ev_gathered[f.i], 0));
    } else {
      for (const Member& o : g->mem) GS_HIP(hipStreamWaitEvent(c->stream, o.ev_gathered[f.i], 0));
    }
  }
  if (f.timed) GS_HIP(hipEventRecord(m.ev_t0[f.i], c->stream));
  if ((rc = gsr::enqueue_frame(c)) != GS_OK) return rc;
  GS_HIP(hipEventRecord(m.ev_render[f.i], c->stream));
  if (f.timed) GS_HIP(hipEventRecord(m.ev_t1[f.i], c->stream));
  return GS_OK;
}

// Member m's side of the frame's all-gather over RCCL, on its communication
// stream after its band: this thread's own call on m's communicator (one
// thread per member).
int member_gather_rccl(Group* g, Member& m, const FrameCmd& f) {
  int rc = set_dev(m.device);
  if (rc != GS_OK) return rc;
  uint8_t* part = own_part(g, m, f);
  if (g->world == 1) {
    // nothing to exchange: the frame stays on its render stream (a second
    // stream's event waits cost the one-GPU group ~10 % of its frames), and
    // no sticky copy per frame either (a launch and a wait on the previous
    // frame: 8 079 -> 8 260 frames/s without them) -- with no other rank to
    // agree with, wait_frames reads the sticky word itself, once per sync
    (void)part;
    return GS_OK;
  }
  GS_HIP(hipStreamWaitEvent(m.comm_stream, m.ev_render[f.i], 0));
  // the GPU's sticky overflow bit into the footer: every frame up to this
  // one has finished its render here (the gathers run in frame order)
  gsk::launch_copy_word(m.comm_stream, (uint32_t*)(part + f.bgr_part) + gsk::kFootSticky, m.d_sticky);
  // in place: sendbuff == recvbuff + rank * sendcount.  A world of one has
  // nothing to exchange: its band is the whole gathered slot already (RCCL's
  // one-rank all-gather still copied the 6.2-MB slot onto itself, 14 us)
  if (g->world > 1)
    GS_NCCL(rccl().AllGather(part, m.d_recv + (size_t)f.i * g->world * g->slot_cap, f.bytes, ncclUint8, m.comm,
                             m.comm_stream));
  return GS_OK;
}

int member_gathered(Group* g, Member& m, const FrameCmd& f) {
  int rc = set_dev(m.device);
  if (rc != GS_OK) return rc;
  hipStream_t s = (g->rccl && g->world == 1) ? m.slot[f.i]->stream : m.comm_stream;
  GS_HIP(hipEventRecord(m.ev_gathered[f.i], s));
  if (f.timed) GS_HIP(hipEventRecord(m.ev_t2[f.i], s));
  return GS_OK;
}

inline void cpu_relax() {
#if !defined(__HIP_DEVICE_COMPILE__)
  __builtin_ia32_pause();
#endif
}

// Worker k (k >= 1): waits for posted frames and runs member k's part of each.
// It spins for a while after a frame (frames arrive every ~0.1 ms while a
// pipeline runs), then sleeps on the condition variable.
void worker_main(Group* g, int k) {
  Member& m = g->mem[(size_t)k];
  (void)hipSetDevice(m.device);
  uint64_t seen = 0;
  for (;;) {
    uint64_t s = g->post_seq.load(std::memory_order_acquire);
    auto t_spin = std::chrono::steady_clock::now();
    while (s == seen && !g->stop.load(std::memory_order_acquire)) {
      if (std::chrono::steady_clock::now() - t_spin < std::chrono::microseconds(500)) {
        cpu_relax();
      } else {
        g->sleepers.fetch_add(1);
        {
          std::unique_lock<std::mutex> lk(g->wmu);
          g->wcv.wait(lk, [&] { return g->post_seq.load() != seen || g->stop.load(); });
        }
        g->sleepers.fetch_sub(1);
        t_spin = std::chrono::steady_clock::now();
      }
      s = g->post_seq.load(std::memory_order_acquire);
    }
    if (s == seen) return;  // stop
    seen = s;
    const FrameCmd f = g->cmd;
    m.rc = member_render(g, m, f);
    if (m.rc != GS_OK) m.err = gsh::last_error();
    g->done.fetch_add(1, std::memory_order_acq_rel);
    if (!g->rccl) continue;
    // phase 2: the caller's verdict on every member's band (a short wait: the
    // caller posts it as soon as the last band is enqueued)
    while (g->gather_seq.load(std::memory_order_acquire) != s) cpu_relax();
    if (g->gather_ok.load(std::memory_order_acquire)) {
      int rc = member_gather_rccl(g, m, f);
      if (rc == GS_OK) rc = member_gathered(g, m, f);
      if (rc != GS_OK) {
        m.rc = rc;
        m.err = gsh::last_error();
      }
    }
    g->gathered.fetch_add(1, std::memory_order_acq_rel);
  }
}

void stop_workers(Group* g) {
  if (g->workers.empty()) return;
  g->stop.store(true);
  {
    std::lock_guard<std::mutex> lk(g->wmu);
    g->wcv.notify_all();
  }
  for (std::thread& t : g->workers) t.join();
  g->workers.clear();
}

int enqueue(Group* g) {
  if (g->failed) {
    set_error("row-band group: an earlier frame failed on one member; destroy the group");
    return GS_EDEVICE;
  }
  const int i = (int)(g->frame % (uint64_t)g->F);
  SlotInfo& si = g->sinfo[i];
  int rc = set_dev(g->mem[0].device);
  if (rc != GS_OK) return rc;
  // re-balance from the snapshot of frame k - kRebalanceEvery / 2 (long done)
  if (g->frame % kRebalanceEvery == 0 && g->snap_pending) {
    GS_HIP(hipEventSynchronize(g->ev_snap));
    g->snap_pending = false;
    parse_footers(g, g->h_snap, g->snap_bounds, false, true);
  }
  // the timing of the frame this slot held (profiling only)
  if ((rc = harvest_timing(g, i, false)) != GS_OK) return rc;
  FrameCmd f;
  f.i = i;
  for (int r = 0; r < g->world; ++r) f.pad = std::max(f.pad, (int)(g->bounds[r + 1] - g->bounds[r]));
  f.bgr_part = align256((size_t)f.pad * g->th * g->W * 3);
  f.bytes = align256(f.bgr_part + (16 + (size_t)f.pad * g->tiles_x) * 4);
  f.was_used = si.used;
  f.timed = g->profile && g->frame % g->profile_every == 0;
  f.prev = g->frame > 0 ? (int)((g->frame - 1) % (uint64_t)g->F) : -1;
  if (g->threaded) {
    // members 1.. on their worker threads, member 0 here; over RCCL each
    // member's all-gather is its own thread's call
    // (two phases: every band first, then -- only if all succeeded -- every
    // member's all-gather, each on its own thread)
    g->cmd = f;
    g->done.store(0, std::memory_order_relaxed);
    g->gathered.store(0, std::memory_order_relaxed);
    const uint64_t seq = g->post_seq.fetch_add(1) + 1;
    if (g->sleepers.load() > 0) {
      std::lock_guard<std::mutex> lk(g->wmu);
      g->wcv.notify_all();
    }
    Member& m0 = g->mem[0];
    m0.rc = member_render(g, m0, f);
    if (m0.rc != GS_OK) m0.err = gsh::last_error();
    const uint32_t want = (uint32_t)g->mem.size() - 1;
    while (g->done.load(std::memory_order_acquire) < want) cpu_relax();
    bool ok = true;
    for (const Member& m : g->mem) ok = ok && m.rc == GS_OK;
    if (g->rccl) {
      g->gather_ok.store(ok, std::memory_order_release);
      g->gather_seq.store(seq, std::memory_order_release);
      if (ok) {
        m0.rc = member_gather_rccl(g, m0, f);
        if (m0.rc == GS_OK) m0.rc = member_gathered(g, m0, f);
        if (m0.rc != GS_OK) m0.err = gsh::last_error();
      }
      while (g->gathered.load(std::memory_order_acquire) < want) cpu_relax();
    }
    for (Member& m : g->mem)
      if (m.rc != GS_OK) {
        // a band failed (no collective was issued), or a gather call failed
        // after others were issued: either way the group's streams can no
        // longer be trusted to drain in step
        g->failed = true;
        set_error(m.err);
        return m.rc;
      }
  } else {  // one member (world 1, or one rank of a multi-process group)
    Member& m = g->mem[0];
    if ((rc = member_render(g, m, f)) != GS_OK) return rc;
    if (g->rccl) {
      if ((rc = member_gather_rccl(g, m, f)) != GS_OK) {
        g->failed = true;
        return rc;
      }
    }
  }
  if (!g->rccl) {  // copies read every member's band (emulated bands on one device)
    for (Member& m : g->mem) {
      if ((rc = set_dev(m.device)) != GS_OK) return rc;
      for (Member& o : g->mem) GS_HIP(hipStreamWaitEvent(m.comm_stream, o.ev_render[i], 0));
      uint8_t* recv = m.d_recv + (size_t)i * g->world * g->slot_cap;
      for (const Member& o : g->mem) {
        if (&o != &m)  // (m's own band is already in place)
          GS_HIP(hipMemcpyAsync(recv + (size_t)o.rank * f.bytes, own_part(g, o, f), f.bytes,
                                hipMemcpyDeviceToDevice, m.comm_stream));
        // o's sticky bit into its gathered footer (this stream has waited for
        // every frame of o up to this one)
        GS_HIP(hipMemcpyAsync((uint32_t*)(recv + (size_t)o.rank * f.bytes + f.bgr_part) + gsk::kFootSticky,
                              o.d_sticky, 4, hipMemcpyDeviceToDevice, m.comm_stream));
      }
    }
  }
  if (!g->threaded || !g->rccl)
    for (Member& m : g->mem)
      if ((rc = member_gathered(g, m, f)) != GS_OK) return rc;
  Member& m0 = g->mem[0];
  if ((rc = set_dev(m0.device)) != GS_OK) return rc;
  si.used = true;
  si.gather_timed = f.timed;
  si.frame = g->frame;
  si.bounds = g->bounds;
  si.pad_rows = f.pad;
  si.bgr_part = f.bgr_part;
  si.bytes = f.bytes;
  // the footers of this frame for the re-balancing kRebalanceEvery / 2 frames on
  if (g->rebalance && g->world > 1 && g->frame % kRebalanceEvery == kRebalanceEvery / 2) {
    if ((rc = copy_footers(g, i, g->h_snap, m0.comm_stream, true)) != GS_OK) return rc;
    GS_HIP(hipEventRecord(g->ev_snap, m0.comm_stream));
    g->snap_bounds = g->bounds;
    g->snap_pending = true;
  }
  g->last_slot = i;
  g->last_read = false;
  g->frame += 1;
  return GS_OK;
}

int ensure_capacity(Group* g) {
  // after an overflow: every band renderer of every rank gets the same new
  // capacity, from the gathered footers (the longest band list of the last
  // frame; the next frames may move the bands) and at least twice the old
  // one (the overflow may have come from an earlier in-flight frame)
  const uint64_t need = g->need_pairs + g->need_pairs / 4 + 1024;
  if (g->need_pairs > 0xFFFFFFF0ull || g->pair_cap >= 0xFFFFFFF0ull) {
    set_error("gs_render: a band's pair count exceeds 2^32");
    return GS_EOVERFLOW;
  }
  g->pair_cap = std::min<uint64_t>(std::max<uint64_t>(need, 2 * g->pair_cap), 0xFFFFFFF0ull);
  for (Member& m : g->mem) {
    int rc = set_dev(m.device);
    if (rc != GS_OK) return rc;
    for (gs_renderer* c : m.slot) {
      if (c->pair_cap >= g->pair_cap) continue;
      GS_HIP(hipStreamSynchronize(c->stream));
      if ((rc = gsr::alloc_pairs(c, g->pair_cap)) != GS_OK) return rc;
    }
  }
  return GS_OK;
}

void release(Group* g) {
  stop_workers(g);
  for (Member& m : g->mem) {
    (void)hipSetDevice(m.device);
    if (m.comm_stream) (void)hipStreamSynchronize(m.comm_stream);
    for (gs_renderer* c : m.slot) gsr::destroy(c);
    m.slot.clear();
    if (m.comm) (void)rccl().CommDestroy(m.comm);
    if (m.d_recv) (void)hipFree(m.d_recv);
    if (m.d_sticky) (void)hipFree(m.d_sticky);
    for (hipEvent_t e : m.ev_render)
      if (e) (void)hipEventDestroy(e);
    for (auto* v : {&m.ev_gathered, &m.ev_t0, &m.ev_t1, &m.ev_t2})
      for (hipEvent_t e : *v)
        if (e) (void)hipEventDestroy(e);
    if (m.comm_stream) (void)hipStreamDestroy(m.comm_stream);
  }
  if (!g->mem.empty()) (void)hipSetDevice(g->mem[0].device);
  if (g->ev_snap) (void)hipEventDestroy(g->ev_snap);
  if (g->h_snap) (void)hipHostFree(g->h_snap);
  if (g->h_last) (void)hipHostFree(g->h_last);
  g->mem.clear();
}

}  // namespace

int create(const gs_gaussian3d* gs, size_t n, const gs_config* cfg, const gs_comm_id* id, int rank,
           int world, gs_renderer** out) {
  if (!out || !cfg || (n > 0 && !gs)) {
    set_error("gs_create: null argument");
    return GS_EINVAL;
  }
  *out = nullptr;
  const bool mp = id != nullptr;
  const int G = mp ? world : (int)cfg->num_gpus;
  if (cfg->flags & GS_FLAG_LATTICE) {
    set_error("gs_create: the lattice emulator (GS_FLAG_LATTICE) runs on one device, not in a row-band group");
    return GS_EINVAL;
  }
  if (G < 1 || (!mp && G > GS_MAX_GPUS) || (mp && (rank < 0 || rank >= world)) || cfg->tile_height == 0 ||
      cfg->tile_width == 0 || cfg->width == 0 || cfg->height == 0) {
    set_error("gs_create: invalid row-band group (num_gpus / rank / world)");
    return GS_EINVAL;
  }
  const int tiles_y = (int)((cfg->height + cfg->tile_height - 1) / cfg->tile_height);
  if (tiles_y < G) {
    set_error("gs_create: fewer tile rows than bands");
    return GS_EINVAL;
  }
  Group* g = new Group();
  auto fail = [&](int rc) {
    release(g);
    delete g;
    return rc;
  };
  g->cfg = *cfg;
  g->n = n;
  g->world = G;
  g->multi_process = mp;
  g->F = std::max(1, std::min(kMaxInFlight, (int)cfg->frames_in_flight));
  g->rebalance = (cfg->flags & GS_FLAG_NO_REBALANCE) == 0;
  g->profile = (cfg->flags & GS_FLAG_PROFILE) != 0;
  g->W = (int)cfg->width;
  g->H = (int)cfg->height;
  g->tw = (int)cfg->tile_width;
  g->th = (int)cfg->tile_height;
  g->tiles_x = (int)((cfg->width + cfg->tile_width - 1) / cfg->tile_width);
  g->tiles_y = tiles_y;
  g->T = g->tiles_x * g->tiles_y;
  g->foot_words = 16 + (size_t)g->T;
  g->slot_cap = align256(align256((size_t)g->tiles_y * g->th * g->W * 3) + g->foot_words * 4);
  for (int i = 0; i < 16; ++i) g->view[i] = g->proj[i] = (i % 5 == 0) ? 1.0f : 0.0f;

  // members: the bands this process renders
  std::vector<int> devs;
  if (mp) {
    int dev = cfg->device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return fail(gsr::hip_fail(hipGetDevice(&dev), "hipGetDevice"));
    devs.push_back(dev);
  } else {
    for (int k = 0; k < G; ++k) devs.push_back(cfg->device_ids[k]);
  }
  bool dup = false;
  for (size_t a = 0; a < devs.size(); ++a)
    for (size_t b = a + 1; b < devs.size(); ++b) dup = dup || devs[a] == devs[b];
  g->rccl = mp || !(dup || (cfg->flags & GS_FLAG_GATHER_COPY));
  if (mp && (cfg->flags & GS_FLAG_GATHER_COPY)) {
    set_error("gs_create_rank: the copy gather needs every band in one process");
    return fail(GS_EINVAL);
  }
  g->mem.resize(devs.size());
  for (size_t k = 0; k < devs.size(); ++k) {
    g->mem[k].device = devs[k];
    g->mem[k].rank = mp ? rank : (int)k;
  }

  // the initial split: equal work per tile (nearly equal rows); later frames
  // re-balance from the gathered histograms
  g->bounds.assign((size_t)G + 1, 0u);
  {
    std::vector<double> ones((size_t)tiles_y, 1.0);
    balanced_bands(ones.data(), tiles_y, G, g->bounds.data());
  }
  g->sinfo.assign((size_t)g->F, SlotInfo{});

  // band renderers: sized for the whole frame (any split fits), band cull on
  gs_config cc = *cfg;
  cc.num_gpus = 0;
  cc.frames_in_flight = 0;
  cc.band_index = 0;
  cc.band_count = 1;
  cc.band_row_begin = 0;
  cc.band_row_end = (uint32_t)tiles_y;
  cc.band_pad_rows = (uint32_t)tiles_y;
  cc.flags = (cfg->flags | GS_FLAG_BAND_CULL) & ~(GS_FLAG_BAND_INTERLEAVED | GS_FLAG_NO_REBALANCE |
                                                   GS_FLAG_GATHER_COPY | GS_FLAG_PROFILE);
  int rc = GS_OK;
  for (size_t k = 0; k < g->mem.size(); ++k) {
    Member& m = g->mem[k];
    cc.device = m.device;
    const gs_renderer* share = nullptr;  // one scene copy per device
    for (size_t j = 0; j <= k && !share; ++j)
      if (g->mem[j].device == m.device && !g->mem[j].slot.empty()) share = g->mem[j].slot[0];
    for (int s = 0; s < g->F; ++s) {
      gs_config c2 = cc;
      if (k == 0 && s == 0 && g->profile) c2.flags |= GS_FLAG_PROFILE;
      gs_renderer* c = nullptr;
      if ((rc = gsr::create(gs, n, &c2, share, &c)) != GS_OK) return fail(rc);
      m.slot.push_back(c);
      if (!share) share = c;
    }
    if ((rc = set_dev(m.device)) != GS_OK) return fail(rc);
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&m.comm_stream, hipStreamNonBlocking)) != hipSuccess)
      return fail(gsr::hip_fail(e, "hipStreamCreate(comm)"));
    if ((e = hipMalloc(&m.d_recv, (size_t)g->F * g->world * g->slot_cap)) != hipSuccess)
      return fail(gsr::hip_fail(e, "hipMalloc(all-gather recv)"));
    if ((e = hipMemset(m.d_recv, 0, (size_t)g->F * g->world * g->slot_cap)) != hipSuccess)
      return fail(gsr::hip_fail(e, "hipMemset(all-gather recv)"));
    if ((e = hipMalloc(&m.d_sticky, 256)) != hipSuccess) return fail(gsr::hip_fail(e, "hipMalloc(sticky)"));
    if ((e = hipMemset(m.d_sticky, 0, 256)) != hipSuccess) return fail(gsr::hip_fail(e, "hipMemset(sticky)"));
    for (gs_renderer* c : m.slot) c->buf.group_sticky = m.d_sticky;
    m.ev_render.assign((size_t)g->F, nullptr);
    m.ev_gathered.assign((size_t)g->F, nullptr);
    for (int s = 0; s < g->F; ++s) {
      if ((e = hipEventCreateWithFlags(&m.ev_render[s], hipEventDisableTiming)) != hipSuccess ||
          (e = hipEventCreateWithFlags(&m.ev_gathered[s], hipEventDisableTiming)) != hipSuccess)
        return fail(gsr::hip_fail(e, "hipEventCreate"));
    }
    if (g->profile) {  // per-member band / gather timing
      for (auto* v : {&m.ev_t0, &m.ev_t1, &m.ev_t2}) {
        v->assign((size_t)g->F, nullptr);
        for (int s = 0; s < g->F; ++s)
          if ((e = hipEventCreate(&(*v)[s])) != hipSuccess) return fail(gsr::hip_fail(e, "hipEventCreate"));
      }
    }
  }
  if ((rc = set_dev(g->mem[0].device)) != GS_OK) return fail(rc);
  {
    hipError_t e;
    if ((e = hipEventCreateWithFlags(&g->ev_snap, hipEventDisableTiming)) != hipSuccess)
      return fail(gsr::hip_fail(e, "hipEventCreate"));
    const size_t fb = (size_t)g->world * g->foot_words * 4;
    if ((e = hipHostMalloc((void**)&g->h_snap, fb, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void**)&g->h_last, fb, hipHostMallocDefault)) != hipSuccess)
      return fail(gsr::hip_fail(e, "hipHostMalloc(footers)"));
    std::memset(g->h_snap, 0, fb);
    std::memset(g->h_last, 0, fb);
  }

  // communicators
  if (g->rccl) {
    if ((rc = rccl_check()) != GS_OK) return fail(rc);
    if (mp) {
      ncclUniqueId uid;
      static_assert(sizeof(uid) == sizeof(id->bytes), "ncclUniqueId is 128 bytes");
      std::memcpy(&uid, id->bytes, sizeof(uid));
      if ((rc = set_dev(g->mem[0].device)) != GS_OK) return fail(rc);
      ncclResult_t nr = rccl().CommInitRank(&g->mem[0].comm, world, uid, rank);
      if (nr != ncclSuccess) return fail(nccl_fail(nr, "ncclCommInitRank"));
    } else {
      std::vector<ncclComm_t> comms(devs.size());
      ncclResult_t nr = rccl().CommInitAll(comms.data(), (int)devs.size(), devs.data());
      if (nr != ncclSuccess) return fail(nccl_fail(nr, "ncclCommInitAll"));
      for (size_t k = 0; k < devs.size(); ++k) g->mem[k].comm = comms[k];
    }
    int cnt = -1;
    if (rccl().CommCount && rccl().CommCount(g->mem[0].comm, &cnt) == ncclSuccess) g->comm_ranks = cnt;
  }
  // one enqueue thread per member past the first
  {
    g->threaded = g->mem.size() > 1;
    if (g->threaded)
      for (size_t k = 1; k < g->mem.size(); ++k) g->workers.emplace_back(worker_main, g, (int)k);
  }

  {
    gs_renderer* c0 = g->mem[0].slot[0];
    g->pair_cap = c0->pair_cap;  // the same on every rank (same configuration and scene size)
    g->stats.n_gaussians = n;
    g->stats.n_tiles = (uint32_t)g->T;
    g->stats.tiles_x = (uint32_t)g->tiles_x;
    g->stats.tiles_y = (uint32_t)g->tiles_y;
    g->stats.band_y0 = 0;
    g->stats.band_rows = (uint32_t)g->H;
    g->stats.band_stride = 1;
    g->stats.bin_global = (uint32_t)c0->bin_global;
    g->hist.assign((size_t)g->T, 0u);
  }
  gs_renderer* h = new gs_renderer();
  h->cfg = *cfg;
  h->n = n;
  h->device = g->mem[0].device;
  h->grp = g;
  *out = h;
  return GS_OK;
}

void destroy(Group* g) {
  if (!g) return;
  release(g);
  delete g;
}

int set_view(Group* g, const float* rm) {
  std::memcpy(g->view, rm, sizeof(g->view));
  return GS_OK;
}

int set_projection(Group* g, const float* rm) {
  std::memcpy(g->proj, rm, sizeof(g->proj));
  return GS_OK;
}

int set_focal(Group* g, float fov, float sd) {
  g->fov = fov;
  g->sd = sd;
  return GS_OK;
}

int render_async(Group* g) { return enqueue(g); }

// Waits for every frame of this rank, then reads the last frame's footers
// (its stats and histogram) once.  The status is decided from those gathered
// bytes only -- the same on every rank -- never from a rank-local flag: a
// band's overflow in an earlier in-flight frame reaches the last frame's
// footer through its GPU's sticky word.  Readbacks call this too; it changes
// neither the split nor the sticky words, so a readback on some ranks only
// cannot make the ranks diverge.
int wait_frames(Group* g) {
  int rc = GS_OK;
  for (Member& m : g->mem) {
    if ((rc = set_dev(m.device)) != GS_OK) return rc;
    GS_HIP(hipStreamSynchronize(m.comm_stream));
    for (gs_renderer* c : m.slot) {
      rc = gsr::finish_frame(c);  // (a local overflow is in the footers already)
      if (rc != GS_OK && rc != GS_EOVERFLOW) return rc;
    }
  }
  if (g->last_slot >= 0 && !g->last_read) {
    if ((rc = set_dev(g->mem[0].device)) != GS_OK) return rc;
    if ((rc = copy_footers(g, g->last_slot, g->h_last, nullptr, false)) != GS_OK) return rc;
    if (g->rccl && g->world == 1) {
      // (one rank: its sticky word is read here, not copied into every
      // frame's footer -- member_gather_rccl)
      uint32_t sticky = 0;
      GS_HIP(hipMemcpy(&sticky, g->mem[0].d_sticky, 4, hipMemcpyDeviceToHost));
      g->h_last[gsk::kFootSticky] = sticky;
    }
    g->last_status = parse_footers(g, g->h_last, g->sinfo[g->last_slot].bounds, true, false);
    g->last_read = true;
  }
  for (int i = 0; i < g->F; ++i)  // every frame is done: its timings
    if ((rc = harvest_timing(g, i, true)) != GS_OK) return rc;
  if (g->last_status == GS_EOVERFLOW) {
    set_error("pair list overflow: a band of a frame since the last gs_sync binned more pairs than its capacity");
    return GS_EOVERFLOW;
  }
  return GS_OK;
}

// gs_sync: collective (every rank calls it after the same frames).  The
// status of the frames since the last gs_sync, then the sticky words start
// over (on every rank at the same frame).
int sync(Group* g) {
  const int st = wait_frames(g);
  if (st != GS_OK && st != GS_EOVERFLOW) return st;
  for (Member& m : g->mem) {
    int rc = set_dev(m.device);
    if (rc != GS_OK) return rc;
    GS_HIP(hipMemsetAsync(m.d_sticky, 0, 4, m.comm_stream));
    GS_HIP(hipStreamSynchronize(m.comm_stream));
  }
  if (st == GS_EOVERFLOW)
    set_error("pair list overflow: a band of a frame since the last gs_sync binned more pairs than its capacity");
  return st;
}

// gs_render: collective.  Every rank decides from the same footers whether
// to grow and render again, and re-balances the split from its frame.
int render(Group* g) {
  for (int attempt = 0; attempt < 8; ++attempt) {
    int rc = enqueue(g);
    if (rc != GS_OK) return rc;
    rc = sync(g);
    if (rc == GS_OK) {
      if (g->rebalance && g->world > 1)
        parse_footers(g, g->h_last, g->sinfo[g->last_slot].bounds, false, true);
      return GS_OK;
    }
    if (rc != GS_EOVERFLOW) return rc;
    // every rank saw the same footers: all of them grow and render the frame again
    if ((rc = ensure_capacity(g)) != GS_OK) return rc;
  }
  set_error("gs_render: capacity growth did not converge");
  return GS_EOVERFLOW;
}

int get_stream(Group* g, void** s) {
  // the stream the last frame completes on: the communication stream, or a
  // one-rank world's render stream of that frame
  const Member& m0 = g->mem[0];
  *s = (g->rccl && g->world == 1 && g->last_slot >= 0) ? (void*)m0.slot[g->last_slot]->stream
                                                       : (void*)m0.comm_stream;
  return GS_OK;
}

int read_bgr8(Group* g, uint8_t* dst, size_t bytes) {
  const size_t need = (size_t)g->H * g->W * 3;
  if (bytes < need) {
    set_error("gs_read_bgr8: destination too small");
    return GS_EINVAL;
  }
  int rc = wait_frames(g);
  if (rc != GS_OK) return rc;
  if (g->last_slot < 0) {
    set_error("gs_read_bgr8: no frame rendered yet");
    return GS_EINVAL;
  }
  const SlotInfo& si = g->sinfo[g->last_slot];
  const Member& m0 = g->mem[0];
  if ((rc = set_dev(m0.device)) != GS_OK) return rc;
  const uint8_t* recv = m0.d_recv + (size_t)g->last_slot * g->world * g->slot_cap;
  for (int r = 0; r < g->world; ++r) {  // drop each band's padding
    const int y0 = (int)si.bounds[r] * g->th, y1 = std::min(g->H, (int)si.bounds[r + 1] * g->th);
    if (y1 > y0)
      GS_HIP(hipMemcpy(dst + (size_t)y0 * g->W * 3, recv + (size_t)r * si.bytes, (size_t)(y1 - y0) * g->W * 3,
                       hipMemcpyDeviceToHost));
  }
  return GS_OK;
}

int read_rgba32f(Group* g, float* dst, size_t n_floats, int layout) {
  if (g->multi_process && g->world > 1) {
    set_error("gs_read_rgba32f: a rank of a multi-process group holds only its band's RGBA f32 "
              "(the all-gather moves BGR8)");
    return GS_EINVAL;
  }
  if (layout != GS_LAYOUT_ROW_MAJOR && layout != GS_LAYOUT_REF_TILE_MAJOR) return GS_EINVAL;
  const size_t W = (size_t)g->W, H = (size_t)g->H;
  const size_t need = layout == GS_LAYOUT_ROW_MAJOR ? H * W * 4 : (size_t)g->T * g->tw * g->th * 4;
  if (n_floats < need) {
    set_error("gs_read_rgba32f: destination too small");
    return GS_EINVAL;
  }
  int rc = wait_frames(g);
  if (rc != GS_OK) return rc;
  if (g->last_slot < 0) {
    set_error("gs_read_rgba32f: no frame rendered yet");
    return GS_EINVAL;
  }
  std::vector<float> tmp;
  float* rm = dst;
  if (layout != GS_LAYOUT_ROW_MAJOR) {
    tmp.resize(H * W * 4);
    rm = tmp.data();
  }
  for (Member& m : g->mem) {
    gs_renderer* c = m.slot[g->last_slot];
    if ((rc = gsr::read_rgba32f(c, rm + (size_t)c->band_py0 * W * 4, (size_t)c->band_rows * W * 4,
                                GS_LAYOUT_ROW_MAJOR)) != GS_OK)
      return rc;
  }
  if (layout != GS_LAYOUT_ROW_MAJOR) gsr::retile(rm, H, W, g->tw, g->th, g->tiles_x, g->T, dst);
  return GS_OK;
}

int read_tile_histogram(Group* g, uint32_t* dst, size_t n) {
  std::lock_guard<std::mutex> lk(g->hist_mu);
  if (n < g->hist.size()) {
    set_error("gs_read_tile_histogram: destination too small");
    return GS_EINVAL;
  }
  std::copy(g->hist.begin(), g->hist.end(), dst);
  return GS_OK;
}

int get_stats(Group* g, gs_frame_stats* st) {
  std::lock_guard<std::mutex> lk(g->hist_mu);
  *st = g->stats;
  // the profiled band renderer's own counts (this rank's band), and the
  // kernels its frames launch (the footers carry no paths)
  st->paths = gsr::frame_paths(g->mem[0].slot[0]);
  st->blend_records = g->mem[0].slot[0]->stats.blend_records;
  st->blend_cont_records = g->mem[0].slot[0]->stats.blend_cont_records;
  st->cont_keys = g->mem[0].slot[0]->stats.cont_keys;
  st->cont_lists = g->mem[0].slot[0]->stats.cont_lists;
  st->cont_max = g->mem[0].slot[0]->stats.cont_max;
  st->prefix_overflows = g->mem[0].slot[0]->stats.prefix_overflows;
  st->cont_full_sorts = g->mem[0].slot[0]->stats.cont_full_sorts;
  st->big_pairs = g->mem[0].slot[0]->stats.big_pairs;
  st->big_prefix_keys = g->mem[0].slot[0]->stats.big_prefix_keys;
  st->big_window_keys = g->mem[0].slot[0]->stats.big_window_keys;
  uint64_t cap = ~0ull;
  for (Member& m : g->mem)
    for (gs_renderer* c : m.slot) cap = std::min<uint64_t>(cap, c->pair_cap);
  st->pair_capacity = cap;
  return GS_OK;
}

int read_bins(Group* g, uint64_t* tile_start, size_t n_start, uint32_t* list, size_t n_list) {
  if (g->multi_process && g->world > 1) {
    set_error("gs_read_bins: a rank of a multi-process group holds only its band's lists");
    return GS_EINVAL;
  }
  int rc = wait_frames(g);
  if (rc != GS_OK) return rc;
  if (g->last_slot < 0) {
    set_error("gs_read_bins: no frame rendered yet");
    return GS_EINVAL;
  }
  if (n_start < (size_t)g->T + 1) {
    set_error("gs_read_bins: destination too small");
    return GS_EINVAL;
  }
  uint64_t off = 0;
  size_t t_base = 0;
  for (Member& m : g->mem) {  // ranks in band order
    gs_renderer* c = m.slot[g->last_slot];
    const size_t nt = (size_t)c->n_tiles;
    if (n_list < off + c->stats.n_pairs) {
      set_error("gs_read_bins: destination too small");
      return GS_EINVAL;
    }
    std::vector<uint64_t> ts(nt + 1);
    if ((rc = gsr::read_bins(c, ts.data(), nt + 1, list + off, n_list - off)) != GS_OK) return rc;
    for (size_t j = 0; j < nt; ++j) tile_start[t_base + j] = off + ts[j];
    t_base += nt;
    off += ts[nt];
  }
  tile_start[t_base] = off;
  return GS_OK;
}

int read_projected(Group* g, float* dst, size_t n_floats) {
  int rc = wait_frames(g);
  if (rc != GS_OK) return rc;
  if (g->last_slot < 0) {
    set_error("gs_read_projected: no frame rendered yet");
    return GS_EINVAL;
  }
  if ((rc = set_dev(g->mem[0].device)) != GS_OK) return rc;
  return gsr::read_projected(g->mem[0].slot[g->last_slot], dst, n_floats);
}

int kernel_times(Group* g, double* avg_ms, uint64_t* launches, int n) {
  if (!g->profile) {
    set_error("gs_kernel_times: group created without GS_FLAG_PROFILE");
    return GS_EINVAL;
  }
  gs_renderer* c = g->mem[0].slot[0];
  int rc = set_dev(c->device);
  if (rc != GS_OK) return rc;
  for (auto& s : c->ring)
    if ((rc = gsr::profile_harvest(c, s)) != GS_OK) return rc;
  for (int k = 0; k < n && k < GS_K_COUNT; ++k) {
    if (k == GS_K_GATHER) {
      avg_ms[k] = g->g_n ? g->g_ms / (double)g->g_n : 0.0;
      if (launches) launches[k] = g->g_n;
    } else {
      avg_ms[k] = c->k_launches[k] ? c->k_ms[k] / (double)c->k_launches[k] : 0.0;
      if (launches) launches[k] = c->k_launches[k];
    }
  }
  return GS_OK;
}

int reset_kernel_times(Group* g) {
  int rc = wait_frames(g);
  if (rc != GS_OK && rc != GS_EOVERFLOW) return rc;
  gs_renderer* c = g->mem[0].slot[0];
  if (c->profile) {
    if ((rc = set_dev(c->device)) != GS_OK) return rc;
    for (auto& s : c->ring)
      if ((rc = gsr::profile_harvest(c, s)) != GS_OK) return rc;
    for (int k = 0; k < GS_K_COUNT; ++k) {
      c->k_ms[k] = 0.0;
      c->k_launches[k] = 0;
    }
  }
  g->g_ms = 0.0;
  g->g_n = 0;
  for (Member& m : g->mem) {
    m.band_ms = m.gather_ms = 0.0;
    m.timed_n = 0;
  }
  return GS_OK;
}

int set_profile_interval(Group* g, uint32_t every) {
  g->profile_every = every;
  for (Member& m : g->mem)
    for (gs_renderer* c : m.slot) {
      c->profile_every = every;
      c->frame_seq = 0;
    }
  return GS_OK;
}

int set_sh(Group* g, const float* f_dc, const float* f_rest, size_t n, int degree) {
  int rc = wait_frames(g);
  if (rc != GS_OK && rc != GS_EOVERFLOW) return rc;
  // one copy of the coefficients per device: the first band renderer on it
  // uploads, the others (frames in flight, emulated bands) share it
  std::vector<const gs_renderer*> first;
  for (Member& m : g->mem)
    for (gs_renderer* c : m.slot) {
      const gs_renderer* share = nullptr;
      for (const gs_renderer* o : first)
        if (o->device == c->device) share = o;
      if ((rc = gsr::set_sh(c, f_dc, f_rest, n, degree, share)) != GS_OK) {
        // a renderer that shares another's copy may now point at a copy its
        // owner replaced: every sharer drops its pointer (DC colour again)
        for (Member& mm : g->mem)
          for (gs_renderer* o : mm.slot)
            if (o->d_sh && !o->owns_sh) {
              o->d_sh = nullptr;
              o->buf.sh = nullptr;
              o->sh_degree = -1;
            }
        return rc;
      }
      if (!share) first.push_back(c);
    }
  return GS_OK;
}

int info(Group* g, gs_group_info* out) {
  std::memset(out, 0, sizeof(*out));
  out->world = (uint32_t)g->world;
  out->local_bands = (uint32_t)g->mem.size();
  out->comm_ranks = g->rccl ? g->comm_ranks : -1;
  out->multi_process = g->multi_process ? 1u : 0u;
  out->threaded = g->threaded ? 1u : 0u;
  out->frames_in_flight = (uint32_t)g->F;
  out->frames = g->frame;
  out->rebalances = g->rebalances;
  const std::vector<uint32_t>& b = g->last_slot >= 0 ? g->sinfo[g->last_slot].bounds : g->bounds;
  for (size_t k = 0; k < b.size() && k <= GS_MAX_GPUS; ++k) out->bounds[k] = b[k];
  for (size_t k = 0; k < g->mem.size() && k < GS_MAX_GPUS; ++k) {
    const Member& m = g->mem[k];
    out->band_rank[k] = m.rank;
    out->device[k] = m.device;
    out->band_ms[k] = m.timed_n ? m.band_ms / (double)m.timed_n : 0.0;
    out->gather_ms[k] = m.timed_n ? m.gather_ms / (double)m.timed_n : 0.0;
  }
  out->timed_frames = g->mem.empty() ? 0 : g->mem[0].timed_n;
  return GS_OK;
}

int bands(Group* g, uint32_t* bounds, size_t n) {
  const std::vector<uint32_t>& b = g->last_slot >= 0 ? g->sinfo[g->last_slot].bounds : g->bounds;
  if (n < b.size()) {
    set_error("gs_group_bands: destination too small");
    return GS_EINVAL;
  }
  std::copy(b.begin(), b.end(), bounds);
  return GS_OK;
}

}  // namespace gsg

extern "C" int gs_group_decide(const uint32_t* footers, size_t foot_words, uint32_t world, uint32_t tiles_x,
                               uint32_t tiles_y, const uint32_t* frame_bounds, const uint32_t* cur_bounds,
                               int rebalance, uint32_t* next_bounds, uint64_t* need_pairs) {
  if (!footers || !frame_bounds || !cur_bounds || world == 0 || tiles_y < world || foot_words < 16) {
    set_error("gs_group_decide: invalid arguments");
    return GS_EINVAL;
  }
  for (uint32_t r = 0; r < world; ++r)
    if (frame_bounds[r] >= frame_bounds[r + 1] || cur_bounds[r] >= cur_bounds[r + 1] ||
        16 + (size_t)(frame_bounds[r + 1] - frame_bounds[r]) * tiles_x > foot_words) {
      set_error("gs_group_decide: bounds are not a split of the tile rows that fits the footers");
      return GS_EINVAL;
    }
  if (frame_bounds[0] != 0 || cur_bounds[0] != 0 || frame_bounds[world] != tiles_y || cur_bounds[world] != tiles_y) {
    set_error("gs_group_decide: bounds must cover tile rows [0, tiles_y)");
    return GS_EINVAL;
  }
  return gsg::decide(footers, foot_words, (int)world, (int)tiles_x, (int)tiles_y, frame_bounds, cur_bounds,
                     rebalance != 0, true, next_bounds, need_pairs, nullptr, nullptr);
}

extern "C" int gs_group_get_info(gs_renderer* r, gs_group_info* out) {
  if (!r || !out) return GS_EINVAL;
  if (!r->grp) {
    set_error("gs_group_get_info: not a row-band group");
    return GS_EINVAL;
  }
  return gsg::info(r->grp, out);
}

extern "C" int gs_comm_id_create(gs_comm_id* out) {
  if (!out) return GS_EINVAL;
  int rc = gsg::rccl_check();
  if (rc != GS_OK) return rc;
  ncclUniqueId uid;
  ncclResult_t r = gsg::rccl().GetUniqueId(&uid);
  if (r != ncclSuccess) {
    set_error(std::string("ncclGetUniqueId: ") + gsg::rccl().GetErrorString(r));
    return GS_EDEVICE;
  }
  std::memcpy(out->bytes, &uid, sizeof(out->bytes));
  return GS_OK;
}
