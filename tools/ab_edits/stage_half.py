# A/B: the projection's record staging in two rounds of 32 records per wave
# (4 KB of LDS per workgroup instead of 8 KB).
p = "gs_kernels.hip"
s = open(p).read()
a = """    __shared__ float4 s_rec[4][128];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float4 r2[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    if (i < fp.n) rendered = project_one<P2>(fp, b, i, rect, crect, r2);
    float4* const sw = s_rec[wave];
    sw[2 * lane] = r2[0];
    sw[2 * lane + 1] = r2[1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int i0 = blk * 256 + wave * 64;  // the wave's first Gaussian
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 64 * h + lane;  // float4 k of the wave's records: record i0 + k / 2
      if (i0 + (k >> 1) < fp.n) store_stream(b.rec + 2 * (size_t)i0 + k, sw[k]);
    }
"""
b_ = """    __shared__ float4 s_rec[4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float4 r2[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    if (i < fp.n) rendered = project_one<P2>(fp, b, i, rect, crect, r2);
    float4* const sw = s_rec[wave];
    const int i0 = blk * 256 + wave * 64;  // the wave's first Gaussian
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // records 32 h .. 32 h + 31 of the wave
      if ((lane >> 5) == h) {
        sw[2 * (lane & 31)] = r2[0];
        sw[2 * (lane & 31) + 1] = r2[1];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (i0 + 32 * h + (lane >> 1) < fp.n) store_stream(b.rec + 2 * (size_t)(i0 + 32 * h) + lane, sw[lane]);
      __builtin_amdgcn_wave_barrier();
    }
"""
assert s.count(a) == 1
s = s.replace(a, b_)
open(p, "w").write(s)
