// Host launch cost on this box: N plain kernel launches per "frame" against
// one hipGraphLaunch of the same N kernels captured once (the frame's
// parameters in a device buffer refreshed by one small kernel per frame).
//   hipcc --offload-arch=gfx950 -O2 tools/hip/launch_bench.hip -o /tmp/launch_bench
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

struct Params { float m[64]; int n; };

__global__ void k_work(const Params* p, float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += p->m[0];
}
__global__ void k_byval(Params p, float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += p.m[0];
}
__global__ void k_set(Params p, Params* dst) {
  if (threadIdx.x == 0) *dst = p;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 8, F = 2000;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Params* dp; float* out;
  CK(hipMalloc(&dp, sizeof(Params)));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(out, 0, 4));
  Params hp{};
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  // warm
  for (int i = 0; i < 100; ++i) k_byval<<<1024, 256, 0, s>>>(hp, out);
  CK(hipStreamSynchronize(s));
  // (a) N by-value launches per frame
  auto t0 = now();
  for (int f = 0; f < F; ++f) {
    hp.m[0] = (float)f;
    for (int k = 0; k < N; ++k) k_byval<<<1024, 256, 0, s>>>(hp, out);
  }
  auto t1 = now();
  CK(hipStreamSynchronize(s));
  auto t2 = now();
  printf("plain launches: host %.2f us/frame (%.2f us/launch), wall %.2f us/frame\n", us(t0, t1) / F, us(t0, t1) / F / N, us(t0, t2) / F);
  // (b) graph of N pointer-arg kernels, params refreshed by one by-value kernel
  hipGraph_t g;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < N; ++k) k_work<<<1024, 256, 0, s>>>(dp, out);
  CK(hipStreamEndCapture(s, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 50; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  t0 = now();
  for (int f = 0; f < F; ++f) {
    hp.m[0] = (float)f;
    k_set<<<1, 64, 0, s>>>(hp, dp);
    CK(hipGraphLaunch(ge, s));
  }
  t1 = now();
  CK(hipStreamSynchronize(s));
  t2 = now();
  printf("set kernel + graph launch: host %.2f us/frame, wall %.2f us/frame\n", us(t0, t1) / F, us(t0, t2) / F);
  // (c) graph alone
  t0 = now();
  for (int f = 0; f < F; ++f) CK(hipGraphLaunch(ge, s));
  t1 = now();
  CK(hipStreamSynchronize(s));
  t2 = now();
  printf("graph launch only: host %.2f us/frame, wall %.2f us/frame\n", us(t0, t1) / F, us(t0, t2) / F);
  // (d) N pointer-arg launches (small kernarg)
  t0 = now();
  for (int f = 0; f < F; ++f)
    for (int k = 0; k < N; ++k) k_work<<<1024, 256, 0, s>>>(dp, out);
  t1 = now();
  CK(hipStreamSynchronize(s));
  t2 = now();
  printf("pointer-arg launches: host %.2f us/frame (%.2f us/launch), wall %.2f us/frame\n", us(t0, t1) / F, us(t0, t1) / F / N, us(t0, t2) / F);
  // (e) S streams, each replaying its own graph of N kernels (one frame per
  // stream in flight): does the GPU overlap the streams' dependent chains?
  for (int S : {1, 2, 3, 4, 6}) {
    hipStream_t ss[8];
    hipGraphExec_t gx[8];
    for (int i = 0; i < S; ++i) {
      CK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
      hipGraph_t gi;
      CK(hipStreamBeginCapture(ss[i], hipStreamCaptureModeThreadLocal));
      for (int k = 0; k < N; ++k) k_work<<<1024, 256, 0, ss[i]>>>(dp, out);
      CK(hipStreamEndCapture(ss[i], &gi));
      CK(hipGraphInstantiate(&gx[i], gi, nullptr, nullptr, 0));
      for (int w = 0; w < 20; ++w) CK(hipGraphLaunch(gx[i], ss[i]));
    }
    CK(hipDeviceSynchronize());
    t0 = now();
    for (int f = 0; f < F; ++f) CK(hipGraphLaunch(gx[f % S], ss[f % S]));
    t1 = now();
    CK(hipDeviceSynchronize());
    t2 = now();
    printf("%d streams x graph of %d: host %.2f us/frame, wall %.2f us/frame\n", S, N, us(t0, t1) / F, us(t0, t2) / F);
  }
  return 0;
}
