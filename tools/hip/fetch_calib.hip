// fetch_calib.hip -- calibration of the PMC counter FETCH_SIZE for the access
// widths the blend uses ("calibrate FETCH_SIZE for the blend's
// 16-B and 32-B index gathers on a known byte count").  Each kernel reads a
// known number of distinct bytes exactly once from a buffer far larger than
// the L2s (so every byte comes from HBM once); rocprofv3 --pmc FETCH_SIZE of
// each launch over those bytes is the factor the PMC reports for that access
// pattern:
//   stream16   one float4 per lane, lane-consecutive            (the guide's streaming case)
//   gather32   two float4 per index (a 32-B record), indices a random permutation
//   gather16   one float4 per index (a 16-B colour), random permutation
//   gather4    one u32 per index, random permutation
//   runs32     32-B records, indices in runs of 8 consecutive records (the
//              blend's Morton-local records: neighbours share cache lines)
// and, for WRITE_SIZE (its own --pmc pass), 16-B lane-consecutive stores:
//   store16    plain global_store_dwordx4
//   store16nt  the same stores non-temporal (the blend's RGBA pixels)
//
//   hipcc --offload-arch=gfx950 -O3 tools/hip/fetch_calib.hip -o tools/hip/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d <dir> -o calib --output-format csv -- tools/hip/fetch_calib
// The program prints one line per kernel: name, launches, bytes per launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

__global__ void stream16(const float4* __restrict__ src, float* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (i < n) {
    const float4 v = src[i];
    acc = v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[0] = acc;  // keeps the loads; never true for the zero-filled input
}

__global__ void gather32(const float4* __restrict__ rec, const uint32_t* __restrict__ idx, float* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (i < n) {
    const uint32_t g = idx[i];
    const float4 a = rec[2 * (size_t)g], b = rec[2 * (size_t)g + 1];
    acc = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
  }
  if (acc == 12345.f) out[0] = acc;
}

__global__ void gather16(const float4* __restrict__ col, const uint32_t* __restrict__ idx, float* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (i < n) {
    const float4 a = col[idx[i]];
    acc = a.x + a.y + a.z + a.w;
  }
  if (acc == 12345.f) out[0] = acc;
}

__global__ void gather4(const uint32_t* __restrict__ w, const uint32_t* __restrict__ idx, float* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  if (i < n) acc = w[idx[i]];
  if (acc == 12345u) out[0] = (float)acc;
}

__global__ void store16(float4* __restrict__ dst, size_t n, float v) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = make_float4(v, v, v, v);
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));
__global__ void store16nt(float4* __restrict__ dst, size_t n, float v) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const f32x4_t w = {v, v, v, v};
  if (i < n) __builtin_nontemporal_store(w, reinterpret_cast<f32x4_t*>(dst + i));
}

int main() {
  const size_t n = (size_t)1 << 24;  // 16 M items: 256 MB of 16-B, 512 MB of 32-B -- far past the L2s
  float4 *d_a = nullptr, *d_b = nullptr;
  uint32_t *d_idx = nullptr, *d_runs = nullptr, *d_w = nullptr;
  float* d_out = nullptr;
  CK(hipMalloc(&d_a, n * 16));
  CK(hipMalloc(&d_b, n * 32));
  CK(hipMalloc(&d_w, n * 4));
  CK(hipMalloc(&d_idx, n * 4));
  CK(hipMalloc(&d_runs, n * 4));
  CK(hipMalloc(&d_out, 64));
  CK(hipMemset(d_a, 0, n * 16));
  CK(hipMemset(d_b, 0, n * 32));
  CK(hipMemset(d_w, 0, n * 4));
  std::vector<uint32_t> perm(n), runs(n);
  std::iota(perm.begin(), perm.end(), 0u);
  std::mt19937_64 rng(7);
  std::shuffle(perm.begin(), perm.end(), rng);
  // runs of 8 consecutive records, the runs in random order
  std::vector<uint32_t> starts(n / 8);
  std::iota(starts.begin(), starts.end(), 0u);
  std::shuffle(starts.begin(), starts.end(), rng);
  for (size_t r = 0; r < n / 8; ++r)
    for (size_t k = 0; k < 8; ++k) runs[r * 8 + k] = starts[r] * 8 + (uint32_t)k;
  CK(hipMemcpy(d_idx, perm.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_runs, runs.data(), n * 4, hipMemcpyHostToDevice));
  const unsigned grid = (unsigned)((n + 255) / 256);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) {
    stream16<<<grid, 256>>>(d_a, d_out, n);
    gather32<<<grid, 256>>>(d_b, d_idx, d_out, n);
    gather16<<<grid, 256>>>(d_a, d_idx, d_out, n);
    gather4<<<grid, 256>>>(d_w, d_idx, d_out, n);
    gather32<<<grid, 256>>>(d_b, d_runs, d_out, n);  // (second gather32 launch of each rep: the runs pattern)
    store16<<<grid, 256>>>(d_a, n, 1.0f);
    store16nt<<<grid, 256>>>(d_a, n, 2.0f);
  }
  CK(hipDeviceSynchronize());
  // the bytes each launch reads (the index arrays: 4 B per item, streamed)
  std::printf("stream16 %d launches, %zu bytes per launch (data)\n", reps, n * 16);
  std::printf("gather32 %d launches, %zu bytes per launch (data) + %zu (indices)  [odd launches: random, even: runs of 8]\n",
              2 * reps, n * 32, n * 4);
  std::printf("gather16 %d launches, %zu bytes per launch (data) + %zu (indices)\n", reps, n * 16, n * 4);
  std::printf("store16 / store16nt %d launches each, %zu bytes per launch (written)\n", reps, n * 16);
  std::printf("gather4 %d launches, %zu bytes per launch (data) + %zu (indices)\n", reps, n * 4, n * 4);
  (void)hipFree(d_a);
  (void)hipFree(d_b);
  (void)hipFree(d_w);
  (void)hipFree(d_idx);
  (void)hipFree(d_runs);
  (void)hipFree(d_out);
  return 0;
}
