# Sensitivity probe (never shipped): one synthetic kernel added to every
# frame after the emit, to read which resource the pipelined frame pays for.
#   PROBE=valu  ~20 us alone of independent fp32 mul/add chains, no memory
#   PROBE=mem   a grid-stride read of the pair buffers (up to 100 MB), no math
#   PROBE=lat   one 64-lane wave that waits ~20 us (s_sleep), no resources
import os

kind = os.environ["PROBE"]
k = open("gs_kernels.hip").read()
probe = r'''
namespace {
__global__ __launch_bounds__(256) void gs_probe_valu_kernel(FrameParams fp, Buffers b) {
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (float)threadIdx.x * 1e-3f + (float)j;
  for (int it = 0; it < 100; ++it)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = a[j] * 0.999f + 0.25f;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += a[j];
  if (fp.n < 0 && s == 1.0f) b.counters[15] = 1u;  // (never: keeps the chains)
}
__global__ __launch_bounds__(256) void gs_probe_mem_kernel(FrameParams fp, Buffers b) {
  const size_t words = min((size_t)fp.pair_cap * 2, (size_t)100 << 20) / 4;  // uint4 of pairs + pairs_alt
  const uint4* p = reinterpret_cast<const uint4*>(b.pairs);
  const uint4* q = reinterpret_cast<const uint4*>(b.pairs_alt);
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (size_t)gridDim.x * 256) {
    const uint4 v = p[i];
    const uint4 w = q ? q[i] : v;
    acc ^= v.x ^ v.y ^ v.z ^ v.w ^ w.x ^ w.w;
  }
  if (fp.n < 0 && acc == 7u) b.counters[15] = 1u;  // (never)
}
__global__ __launch_bounds__(64) void gs_probe_lat_kernel(FrameParams fp, Buffers b) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < 2000ull) __builtin_amdgcn_s_sleep(8);  // 20 us at 100 MHz
  if (fp.n < 0) b.counters[15] = 1u;  // (never)
}
}  // namespace
void launch_probe_x(const FrameParams& fp, const Buffers& b, hipStream_t s) {
  %s
}
'''
call = {"valu": "gs_probe_valu_kernel<<<4096, 256, 0, s>>>(fp, b);",
        "mem": "gs_probe_mem_kernel<<<4096, 256, 0, s>>>(fp, b);",
        "lat": "gs_probe_lat_kernel<<<1, 64, 0, s>>>(fp, b);"}[kind]
tail = "}  // namespace gsk\n"
i = k.rindex(tail)
k = k[:i] + probe % call + k[i:]
open("gs_kernels.hip", "w").write(k)

r = open("gs_renderer.hip").read()
line = "  gsk::launch_emit(fp, r->buf, s);\n"
i = r.index("int enqueue_frame(")
j = r.index(line, i) + len(line)
r = r[:j] + "  gsk::launch_probe_x(fp, r->buf, s);\n" + r[j:]
i = r.index("namespace gsr {")
r = r[:i] + "namespace gsk { void launch_probe_x(const FrameParams&, const Buffers&, hipStream_t); }\n" + r[i:]
open("gs_renderer.hip", "w").write(r)
