// gs_lattice.hip -- the lattice-migration emulator (SURVEY §8 f4,
// GS_FLAG_LATTICE): the reference's multi-frame transport of the Gaussians
// over the 4-neighbour channel lattice of IPU tiles, one frame per launch,
// reproducing its transient (non-converged) frames.
//
// The reference runs one GSplat codelet per IPU tile (codelets.cpp:143-641):
// it reads four in-channels, keeps the records whose mean it contains, sends
// halo copies and in-transit records one hop on (readInput :507-586,
// renderInternal :437-505), quicksorts its z-buffer (:295-356) and blends its
// pixels (renderTile :358-421); a Poplar exchange then copies every
// out-channel into the neighbour's in-channel (edge_builder.cpp:15-84).
//
// Here one 64-lane workgroup emulates one IPU tile.  The per-record math
// (projection, EWA covariance, radius, tile geometry) runs lane-parallel over
// 64 records at a time; the order-dependent bookkeeping -- which slot a record
// lands in, which channel fills first, the short-circuiting sends -- runs in
// the reference's record order, one record at a time, each insert a
// wave-wide scan of the destination's gids (mirrored in LDS).  The exchange is
// a parity swap: frame f writes out-channel set f & 1 and reads the
// neighbours' set (f - 1) & 1 as its in-channels.  The quicksort runs in one
// lane over (z, position) pairs in LDS and permutes the z-buffer entries
// after.  The blend stages 64 z-buffer entries at a time in LDS; every lane
// blends its pixels over them.
//
// Arithmetic: the same fp32 operations, in the same order, as the CPU oracle
// (oracle/gs_oracle.cpp, or_lattice_*) and as the frame path's projection
// (gs_kernels.hip project_one): frames, histograms and slot contents are
// bit-identical to it.
#include "gs_kernels.hpp"
#include "gs_math.hpp"

namespace gsk {
namespace {

// enum direction (ipu_geometry.hpp:94-100)
constexpr int kLeft = 0, kRight = 1, kUp = 2, kDown = 3, kNone = 4;

// float -> unsigned of a negative / NaN / huge value: saturated (the reference
// converts out of range; see oracle/gs_oracle.h)
__device__ __forceinline__ uint32_t lat_u32(float v) {
  if (!(v > 0.0f)) return 0u;
  if (v >= 4294967296.0f) return 0xFFFFFFFFu;
  return (uint32_t)v;
}

struct LB {
  float x0, y0, x1, y1;
};

// TiledFramebuffer::getTileBounds (tile_config.hpp:57-71)
__device__ __forceinline__ LB lat_bounds(const LatticeParams& lp, uint32_t tid) {
  const float div = __builtin_floorf((float)tid / lp.across);
  const float mod = (float)tid - div * lp.across;
  LB b;
  b.x0 = __builtin_floorf(mod * lp.tw);
  b.y0 = __builtin_floorf(div * lp.th);
  b.x1 = b.x0 + lp.tw;
  b.y1 = b.y0 + lp.th;
  return b;
}

// Bounds2f::centroid (ipu_geometry.hpp:109-111)
__device__ __forceinline__ void lat_centroid(const LB& b, float& cx, float& cy) {
  cx = (b.x1 + b.x0) * 0.5f;
  cy = (b.y1 + b.y0) * 0.5f;
}

// getNearbyTile (tile_config.hpp:73-86)
__device__ __forceinline__ uint32_t lat_nearby(const LatticeParams& lp, uint32_t tid, int from) {
  if (from == kLeft) return tid - 1u;
  if (from == kRight) return tid + 1u;
  if (from == kUp) return lat_u32((float)tid - lp.across);
  return lat_u32((float)tid + lp.across);
}

// Bounds2f::contains (ipu_geometry.hpp:163-165)
__device__ __forceinline__ bool lat_contains(const LB& b, float x, float y) {
  return __builtin_ceilf(x) >= b.x0 && __builtin_floorf(x) < b.x1 && __builtin_ceilf(y) >= b.y0 &&
         __builtin_floorf(y) < b.y1;
}

// the centroid of pixCoordToTile(y, x)'s tile (tile_config.hpp:43-54)
__device__ __forceinline__ void lat_dest(const LatticeParams& lp, float vx, float vy, float& cx, float& cy) {
  const float r = __builtin_rintf(vy), c = __builtin_rintf(vx);
  const float tc = __builtin_floorf(c / lp.tw);
  const float tr = __builtin_floorf(r / lp.th);
  lat_centroid(lat_bounds(lp, lat_u32(tr * lp.across + tc)), cx, cy);
}

__device__ __forceinline__ float lat_manhattan(float ax, float ay, float bx, float by) {
  return __builtin_fabsf(ax - bx) + __builtin_fabsf(ay - by);
}

// getBestDirection (tile_config.hpp:92-110): y first
__device__ __forceinline__ int lat_best_dir(float sx, float sy, float dx, float dy) {
  if (lat_manhattan(sx, sy, dx, dy) == 0.0f) return kNone;
  if (sy < dy) return kDown;
  if (sy > dy) return kUp;
  if (sx < dx) return kRight;
  if (sx > dx) return kLeft;
  return kNone;
}

// Bounds2f::clip's flags (ipu_geometry.hpp:133-139) as bits 1 << direction
__device__ __forceinline__ uint32_t lat_clip(float bx0, float by0, float bx1, float by1, const LB& tb) {
  uint32_t d = 0;
  if (__builtin_floorf(bx0) < tb.x0) d |= 1u << kLeft;
  if (__builtin_floorf(by0) < tb.y0) d |= 1u << kUp;
  if (__builtin_ceilf(bx1) >= tb.x1) d |= 1u << kRight;
  if (__builtin_ceilf(by1) >= tb.y1) d |= 1u << kDown;
  return d;
}

struct LatP {
  float vx, vy, z, a, b, c, radius;
  bool within;
};

// The per-record math of readInput / renderInternal (codelets.cpp:460-470,
// 537-551, 576-578): the frame path's projection (project_one), op for op.
__device__ __forceinline__ void lat_project(const LatticeParams& lp, const float4* rec, LatP& p) {
  const float4 mean = rec[0], rot = rec[2], sg = rec[3];
  const float* m = lp.mvp;
  const float cx = mv_row(m, 0, mean.x, mean.y, mean.z, mean.w);
  const float cy = mv_row(m, 1, mean.x, mean.y, mean.z, mean.w);
  const float cz = mv_row(m, 2, mean.x, mean.y, mean.z, mean.w);
  const float cw = mv_row(m, 3, mean.x, mean.y, mean.z, mean.w);
  const float s = 0.5f / cw;
  float vx = cx * s, vy = cy * s;
  vx = vx + 0.5f;
  vy = vy + 0.5f;
  vx = vx * lp.W;
  vy = vy * lp.H;
  vx = vx + 0.0f;
  vy = vy + 0.0f;
  float tx = mv_row(m, 0, mean.x, mean.y, mean.z, 1.0f);
  float ty = mv_row(m, 1, mean.x, mean.y, mean.z, 1.0f);
  const float tz = mv_row(m, 2, mean.x, mean.y, mean.z, 1.0f);
  const float lim = 1.3f * lp.tanfov;
  const float txtz = tx / tz;
  const float tytz = ty / tz;
  tx = smin(lim, smax(-lim, txtz)) * tz;
  ty = smin(lim, smax(-lim, tytz)) * tz;
  M3 J;
  J.m[0][0] = lp.focal_x / tz;
  J.m[0][1] = 0.0f;
  J.m[0][2] = -(lp.focal_x * tx) / (tz * tz);
  J.m[1][0] = 0.0f;
  J.m[1][1] = lp.focal_y / tz;
  J.m[1][2] = -(lp.focal_y * ty) / (tz * tz);
  J.m[2][0] = 0.0f;
  J.m[2][1] = 0.0f;
  J.m[2][2] = 0.0f;
  M3 W;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) W.m[c][r] = m[c * 4 + r];
  const M3 T = m3_mul(W, J);
  const M3 C3 = cov3d(rot, sg.x / lp.scale_div, sg.y / lp.scale_div, sg.z / lp.scale_div);
  const M3 cov = m3_mul(m3_mul(m3_t(T), m3_t(C3)), T);
  const float a = cov.m[0][0] + 0.3f;
  const float bb = cov.m[0][1];
  const float c = cov.m[1][1] + 0.3f;
  const float det = a * c - bb * bb;
  const float mid = 0.5f * (a + c);
  const float l1 = mid + __builtin_sqrtf(smax(0.1f, mid * mid - det));
  const float l2 = mid - __builtin_sqrtf(smax(0.1f, mid * mid - det));
  const float radius = __builtin_ceilf(3.0f * __builtin_sqrtf(smax(l1, l2)));
  const float minx = vx - radius, miny = vy - radius;
  const float maxx = vx + radius, maxy = vy + radius;
  const float ddx = maxx - minx, ddy = maxy - miny;
  p.vx = vx;
  p.vy = vy;
  p.z = cz;
  p.a = a;
  p.b = bb;
  p.c = c;
  p.radius = radius;
  p.within = __builtin_sqrtf(ddx * ddx + ddy * ddy) < lp.guard_thr;
}

// insert (codelets.cpp:41-59), wave-uniform: a slot already holding the gid
// -> -2, no empty slot (gid == 0) -> -1, else the first empty slot
__device__ __forceinline__ int lat_find(const float* gids, int n, float gid, int lane) {
  int first = -1;
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int i = b0 + lane;
    const float v = i < n ? gids[i] : -1.0f;
    if (ballot64(i < n && v == gid)) return -2;
    const unsigned long long f = ballot64(i < n && v == 0.0f);
    if (first < 0 && f) first = b0 + __builtin_ctzll(f);
  }
  return first;
}

// insert the staged record into a slot array (gids mirrored in LDS)
__device__ __forceinline__ bool lat_insert(float* gids, int n, float4* slots, const float4* rec, int lane) {
  const float gid = rec[3].w;
  const int s = lat_find(gids, n, gid, lane);
  if (s == -2) return true;
  if (s < 0) return false;
  if (lane < 4) slots[(size_t)s * 4 + lane] = rec[lane];
  if (lane == 0) gids[s] = gid;
  __syncthreads();
  return true;
}

constexpr int kLatChanSlots = kLatChan;

// the emulator's per-frame kernel: one workgroup of one wave per IPU tile
__global__ __launch_bounds__(64) void gs_lattice_kernel(LatticeParams lp, LatticeBufs lb) {
  __shared__ float s_vgid[kLatMaxSlots];       // gid of every vertsIn slot
  __shared__ float s_ogid[4 * kLatChanSlots];  // gid of every out-channel slot
  __shared__ float4 s_rec[64][4];              // a batch of records
  __shared__ uint32_t s_act[64];               // their actions
  __shared__ float s_key[kLatMaxSlots];        // quicksort: z of the entries
  __shared__ uint16_t s_pos[kLatMaxSlots];     //   and their positions
  __shared__ int s_stk[kLatMaxSlots + 2];      //   explicit (l, h) stack
  __shared__ float s_ent[64][10];              // blend: staged z-buffer entries

  const int t = blockIdx.x;
  const int lane = threadIdx.x;
  const int T = lp.n_tiles;
  const bool last = t == T - 1;
  const size_t base = (size_t)t * (size_t)(lp.gpt + kLatExtra);
  const int nvs = lp.gpt + kLatExtra + (last ? lp.rem : 0);
  const int nz = last ? lp.gpt + lp.rem : lp.gpt + kLatExtra;
  float4* vs = lb.slots + base * 4;
  float4* zb = lb.zbuf + base * 3;
  float4* zs = lb.zscratch + base * 3;
  const int par = lp.parity;
  float4* out = lb.chan + (((size_t)par * T + t) * 4) * kLatChanSlots * 4;
  uint32_t dropped = 0, send_failed = 0, overrun = 0;

  // clearOutBuffers (codelets.cpp:588-602): evict every out-channel slot
  for (int k = lane; k < 4 * kLatChanSlots; k += 64) {
    s_ogid[k] = 0.0f;
    out[(size_t)k * 4 + 3].w = 0.0f;
  }
  for (int i = lane; i < nvs; i += 64) s_vgid[i] = vs[(size_t)i * 4 + 3].w;
  __syncthreads();

  const LB tb = lat_bounds(lp, (uint32_t)t);
  float tcx, tcy;
  lat_centroid(tb, tcx, tcy);

  // sendOnce (codelets.cpp:214-225) of staged record j
  auto send_once = [&](int j, int dir) -> bool {
    if (dir == kNone) return false;
    const bool ok = lat_insert(s_ogid + dir * kLatChanSlots, kLatChanSlots, out + (size_t)dir * kLatChanSlots * 4,
                               s_rec[j], lane);
    if (!ok) ++send_failed;
    return ok;
  };

  // ---- readInput of the four in-channels (codelets.cpp:507-586, order :630-633)
  const LB self = tb;
  const bool bl = self.x0 < 1.0f, bu = self.y0 < 1.0f;  // checkImageBoundaries (tile_config.hpp:116-126)
  const bool br = self.x1 > (float)(lp.width - 1), bd = self.y1 > (float)(lp.height - 1);
  for (int oi = 0; oi < 4; ++oi) {
    const int from = oi == 0 ? kRight : oi == 1 ? kLeft : oi == 2 ? kUp : kDown;
    // the out-channel the exchange copied here (edge_builder.cpp:35-84)
    int st = t, sd = from;
    if (from == kRight && !br) { st = t + 1; sd = kLeft; }
    if (from == kLeft && !bl) { st = t - 1; sd = kRight; }
    if (from == kUp && !bu) { st = t - lp.tiles_x; sd = kDown; }
    if (from == kDown && !bd) { st = t + lp.tiles_x; sd = kUp; }
    const float4* in = lb.chan + (((size_t)(par ^ 1) * T + st) * 4 + sd) * kLatChanSlots * 4;
    float pcx, pcy;
    lat_centroid(lat_bounds(lp, lat_nearby(lp, (uint32_t)t, from)), pcx, pcy);
    for (int b0 = 0; b0 < kLatChanSlots; b0 += 64) {
      const int k = b0 + lane;
      uint32_t act = 0;
      if (k < kLatChanSlots) {
        float4 r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = in[(size_t)k * 4 + q];
#pragma unroll
        for (int q = 0; q < 4; ++q) s_rec[lane][q] = r[q];
        if (!(r[3].w <= 0.0f)) {
          LatP p;
          lat_project(lp, r, p);
          act = 1;  // keep it (insert into vertsIn)
          if (!lat_contains(tb, p.vx, p.vy)) {
            float dcx, dcy;
            lat_dest(lp, p.vx, p.vy, dcx, dcy);
            if (lat_manhattan(tcx, tcy, dcx, dcy) < lat_manhattan(pcx, pcy, dcx, dcy)) {
              act = 2 | ((uint32_t)lat_best_dir(tcx, tcy, dcx, dcy) << 4);  // in transit
            } else if (p.within) {
              act = 3 | (lat_clip(p.vx - p.radius, p.vy - p.radius, p.vx + p.radius, p.vy + p.radius, tb) << 8);
            }
          }
        }
      }
      s_act[lane] = act;
      __syncthreads();
      const int cnt = min(64, kLatChanSlots - b0);
      for (int j = 0; j < cnt; ++j) {
        const uint32_t a = s_act[j];
        const uint32_t code = a & 15u;
        if (!code) continue;
        if (code == 2) send_once(j, (int)((a >> 4) & 15u));
        if (code == 3) {  // protocol (codelets.cpp:251-293)
          const uint32_t s = a >> 8;
          const bool su = s & (1u << kUp), sdn = s & (1u << kDown), sl = s & (1u << kLeft), sr = s & (1u << kRight);
          if (from == kRight && sl) {
            bool ok = send_once(j, kLeft);
            if (sdn) ok = ok && send_once(j, kDown);
            if (su) ok = ok && send_once(j, kUp);
          } else if (from == kLeft && sr) {
            bool ok = send_once(j, kRight);
            if (sdn) ok = ok && send_once(j, kDown);
            if (su) ok = ok && send_once(j, kUp);
          } else if (from == kUp && sdn) {
            send_once(j, kDown);
          } else if (from == kDown && su) {
            send_once(j, kUp);
          } else if (s) {
            bool ok = true;
            if (su && from != kUp) ok = ok && send_once(j, kUp);
            if (sdn && from != kDown) ok = ok && send_once(j, kDown);
          }
        }
        if (!lat_insert(s_vgid, nvs, vs, s_rec[j], lane)) ++dropped;
      }
      __syncthreads();
    }
  }

  // ---- renderInternal (codelets.cpp:437-505)
  int to_render = 0;
  for (int b0 = 0; b0 < nvs; b0 += 64) {
    const int i = b0 + lane;
    uint32_t act = 0;
    bool rend = false;
    LatP p;
    float4 r[4];
    if (i < nvs && !(s_vgid[i] <= 0.0f)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) r[q] = vs[(size_t)i * 4 + q];
#pragma unroll
      for (int q = 0; q < 4; ++q) s_rec[lane][q] = r[q];
      lat_project(lp, r, p);
      if (lat_contains(tb, p.vx, p.vy)) {
        // send (codelets.cpp:194-212) with the clip flags (none outside the guard band)
        const uint32_t d =
            p.within ? lat_clip(p.vx - p.radius, p.vy - p.radius, p.vx + p.radius, p.vy + p.radius, tb) : 0u;
        act = 1 | (d << 8);
      } else {
        float dcx, dcy;
        lat_dest(lp, p.vx, p.vy, dcx, dcy);
        act = 2 | ((uint32_t)lat_best_dir(tcx, tcy, dcx, dcy) << 4);
      }
      rend = p.within && p.z < 0.0f;
    }
    // the z-buffer entries, in slot order (insertAt :493-497)
    const unsigned long long m = ballot64(rend);
    const int pos = to_render + (int)__builtin_popcountll(m & ((1ull << lane) - 1ull));
    if (rend) {
      if (pos < nz) {
        zb[(size_t)pos * 3 + 0] = r[1];  // colour
        zb[(size_t)pos * 3 + 1] = make_float4(p.a, p.b, p.c, p.z);
        zb[(size_t)pos * 3 + 2] = make_float4(p.vx, p.vy, 0.0f, 0.0f);
      }
    }
    overrun += (uint32_t)__builtin_popcountll(ballot64(rend && pos >= nz));
    to_render += (int)__builtin_popcountll(m);
    s_act[lane] = act;
    __syncthreads();
    const int cnt = min(64, nvs - b0);
    for (int j = 0; j < cnt; ++j) {
      const uint32_t a = s_act[j];
      const uint32_t code = a & 15u;
      if (!code) continue;
      if (code == 1) {
        const uint32_t d = a >> 8;
        bool sent = true;
        if (d & (1u << kRight)) sent = sent && send_once(j, kRight);
        if (d & (1u << kLeft)) sent = sent && send_once(j, kLeft);
        if (d & (1u << kUp)) sent = sent && send_once(j, kUp);
        if (d & (1u << kDown)) sent = sent && send_once(j, kDown);
      } else if (send_once(j, (int)((a >> 4) & 15u))) {
        // evicted; a failed send puts it right back (the slot is unchanged)
        if (lane == 0) {
          s_vgid[b0 + j] = 0.0f;
          vs[(size_t)(b0 + j) * 4 + 3].w = 0.0f;
        }
      }
    }
    __syncthreads();
  }

  // ---- sortBuffer (codelets.cpp:346-356): [0, L] inclusive unless L >= nz - 1
  const int L = to_render;
  if (L >= 1 && L < nz - 1) {
    for (int k = lane; k <= L; k += 64) {
      s_key[k] = zb[(size_t)k * 3 + 1].w;
      s_pos[k] = (uint16_t)k;
    }
    __syncthreads();
    if (lane == 0) {  // iterativeQuickSort / partition (codelets.cpp:303-344)
      int top = -1;
      s_stk[++top] = 0;
      s_stk[++top] = L;
      while (top >= 0) {
        const int h = s_stk[top--];
        const int l = s_stk[top--];
        const float pivot = s_key[h];
        int ii = l - 1;
        for (int j = l; j <= h - 1; ++j) {
          const float kj = s_key[j];
          if (kj <= pivot) {
            ++ii;
            const float ki = s_key[ii];
            const uint16_t pi_ = s_pos[ii];
            s_key[ii] = kj;
            s_pos[ii] = s_pos[j];
            s_key[j] = ki;
            s_pos[j] = pi_;
          }
        }
        {
          const float ki = s_key[ii + 1];
          const uint16_t pi_ = s_pos[ii + 1];
          s_key[ii + 1] = s_key[h];
          s_pos[ii + 1] = s_pos[h];
          s_key[h] = ki;
          s_pos[h] = pi_;
        }
        const int pv = ii + 1;
        if (pv - 1 > l) {
          s_stk[++top] = l;
          s_stk[++top] = pv - 1;
        }
        if (pv + 1 < h) {
          s_stk[++top] = pv + 1;
          s_stk[++top] = h;
        }
      }
    }
    __syncthreads();
    for (int k = lane; k <= L; k += 64)
#pragma unroll
      for (int q = 0; q < 3; ++q) zs[(size_t)k * 3 + q] = zb[(size_t)k * 3 + q];
    __syncthreads();
    for (int k = lane; k <= L; k += 64) {
      const size_t src = s_pos[k];
#pragma unroll
      for (int q = 0; q < 3; ++q) zb[(size_t)k * 3 + q] = zs[src * 3 + q];
    }
    __syncthreads();
  }

  // ---- renderTile (codelets.cpp:358-421) into the zeroed tile framebuffer
  const int tw = lp.tile_w, npx = lp.tile_w * lp.tile_h;
  for (int pg = 0; pg < npx; pg += 64) {
    const int px = pg + lane;
    const int lx = px % tw, ly = px / tw;
    const float pfx = tb.x0 + (float)lx, pfy = tb.y0 + (float)ly;
    float T_ = 1.0f, c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
    bool done = px >= npx;
    for (int e0 = 0; e0 < L; e0 += 64) {
      const int j = e0 + lane;
      if (j < L) {
        float4 col = make_float4(0.f, 0.f, 0.f, 0.f), cv = col, mn = col;
        if (j < nz) {  // past the z-buffer: an empty record
          col = zb[(size_t)j * 3 + 0];
          cv = zb[(size_t)j * 3 + 1];
          mn = zb[(size_t)j * 3 + 2];
        }
        // ComputeConicOpacity (ipu_geometry.hpp:278-286)
        const float det = cv.x * cv.z - cv.y * cv.y;
        float k0 = 0.0f, k1 = 0.0f, k2 = 0.0f, op = 0.0f;
        if (!(det == 0.0f)) {
          const float inv = 1.0f / det;
          k0 = cv.z * inv;
          k1 = -cv.y * inv;
          k2 = cv.x * inv;
          op = col.w;
        }
        float* e = s_ent[lane];
        e[0] = mn.x;
        e[1] = mn.y;
        e[2] = k0;
        e[3] = k1;
        e[4] = k2;
        e[5] = op;
        e[6] = col.x;
        e[7] = col.y;
        e[8] = col.z;
        e[9] = col.w;
      }
      __syncthreads();
      const int cnt = min(64, L - e0);
      for (int q = 0; q < cnt && !done; ++q) {
        const float* e = s_ent[q];
        const float op = e[5];
        if (op == 0.0f) continue;
        const float dx = e[0] - pfx, dy = e[1] - pfy;
        const float power = -0.5f * (e[2] * dx * dx + e[4] * dy * dy) - e[3] * dx * dy;
        if (power > 0.0f) continue;
        const float v = op * gs_expf(power);
        const float alpha = (v < 0.99f) ? v : 0.99f;
        if (alpha < 1.0f / 255.0f) continue;
        const float test_T = T_ * (1.0f - alpha);
        if (test_T < 0.0001f) {
          done = true;
          break;
        }
        c0 = c0 + (e[6] * alpha) * T_;
        c1 = c1 + (e[7] * alpha) * T_;
        c2 = c2 + (e[8] * alpha) * T_;
        c3 = c3 + (e[9] * alpha) * T_;
        T_ = test_T;
      }
      __syncthreads();
    }
    if (px < npx) {
      const size_t x = (size_t)tb.x0 + (size_t)lx, y = (size_t)tb.y0 + (size_t)ly;
      const float o0 = 0.0f + c0, o1 = 0.0f + c1, o2 = 0.0f + c2, o3 = 0.0f + c3;
      if (lp.write_rgba) lb.rgba[y * (size_t)lp.width + x] = make_float4(o0, o1, o2, o3);
      uint8_t* dst = lb.bgr + y * (size_t)lp.bgr_pitch + 3 * x;
      dst[0] = to_u8(o2);  // RGBA2BGR
      dst[1] = to_u8(o1);
      dst[2] = to_u8(o0);
    }
  }
  if (lane == 0) {
    if (L > 0) lb.splatted[t] = (uint32_t)L;  // splatted[0] = toRender (codelets.cpp:501-504)
    uint32_t* ts = lb.tile_stat + (size_t)t * 4;
    ts[0] = (uint32_t)L;
    ts[1] = dropped;
    ts[2] = send_failed;
    ts[3] = overrun;
  }
}

// The frame's counters and histogram into the renderer's mapped host mirror
// (counters[16] + splatted[T]): 2 / 5,6 / 10,11 = sum of the tiles' render
// lists, 4 = the longest, 12 = dropped vertsIn inserts, 13 = failed channel
// inserts, 14 = z-buffer overruns.
__global__ __launch_bounds__(256) void gs_lattice_finish_kernel(LatticeParams lp, LatticeBufs lb) {
  __shared__ unsigned long long s_sum[4][4];
  __shared__ uint32_t s_max[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  unsigned long long sum[4] = {0, 0, 0, 0};
  uint32_t mx = 0;
  for (int t = tid; t < lp.n_tiles; t += 256) {
    const uint32_t* ts = lb.tile_stat + (size_t)t * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) sum[q] += ts[q];
    const uint32_t sp = lb.splatted[t];
    mx = max(mx, sp);
    lb.host_counters[16 + t] = sp;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned long long v = sum[q];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_sum[w][q] = v;
  }
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
  if (lane == 0) s_max[w] = mx;
  __syncthreads();
  if (tid < 16) {
    unsigned long long tot[4] = {0, 0, 0, 0};
    uint32_t m = 0;
    for (int k = 0; k < 4; ++k) {
      for (int q = 0; q < 4; ++q) tot[q] += s_sum[k][q];
      m = max(m, s_max[k]);
    }
    uint32_t v = 0;
    switch (tid) {
      case 2: v = (uint32_t)tot[0]; break;
      case 4: v = m; break;
      case 5: case 10: v = (uint32_t)tot[0]; break;
      case 6: case 11: v = (uint32_t)(tot[0] >> 32); break;
      case 12: v = (uint32_t)tot[1]; break;
      case 13: v = (uint32_t)tot[2]; break;
      case 14: v = (uint32_t)tot[3]; break;
      default: v = 0;
    }
    lb.host_counters[tid] = v;
  }
}

}  // namespace

void launch_lattice(const LatticeParams& lp, const LatticeBufs& lb, hipStream_t s) {
  hipLaunchKernelGGL(gs_lattice_kernel, dim3((unsigned)lp.n_tiles), dim3(64), 0, s, lp, lb);
  hipLaunchKernelGGL(gs_lattice_finish_kernel, dim3(1), dim3(256), 0, s, lp, lb);
}

}  // namespace gsk
