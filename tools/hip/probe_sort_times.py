"""Edit script for tools/build_variant_from.sh (run inside csrc/): a probe build
in which every gs_sort_tiles workgroup writes (start, end, list length, class)
of its own run (s_memrealtime, 100 MHz) into rgba[blockIdx.x], and the blend
is not launched (so the framebuffer keeps them).  tools/sort_times.py reads
them back.  Not a product build."""
p = "gs_kernels.hip"
s = open(p).read()
old = """__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_sort_tiles_kernel(FrameParams fp, Buffers b) {
  sort_tiles<256>(fp, b);
}"""
new = """__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_sort_tiles_kernel(FrameParams fp, Buffers b) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  sort_tiles<256>(fp, b);
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    const uint32_t n_med = b.counters[7];
    uint32_t L = 0u, cls = 1u;
    if (blockIdx.x < n_med) {
      uint32_t st;
      tile_segment(fp, b, (int)b.medium_tiles[blockIdx.x], st, L);
      cls = 2u;
    }
    b.rgba[blockIdx.x] = make_float4(__uint_as_float((uint32_t)t0), __uint_as_float((uint32_t)t1),
                                     __uint_as_float(L), __uint_as_float(cls));
  }
}"""
assert old in s
s = s.replace(old, new)
# sort_tiles returns early on several paths: make them fall through to the stamp
open(p, "w").write(s)
r = "gs_renderer.hip"
s = open(r).read()
old = """  gsk::launch_blend(fb, r->buf, s);"""
assert old in s
s = s.replace(old, """  if (!std::getenv("GSPLAT_SKIP_BLEND")) gsk::launch_blend(fb, r->buf, s);""")
open(r, "w").write(s)
