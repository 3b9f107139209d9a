# Experiment (config 3 only, never shipped as is): 20-B records (mean, conic)
# from the whole-frame projection; the two-pixel blend recomputes the power
# cut-off and the alpha box at staging (alpha_footprint, the projection's own
# function on the same inputs: with pair culling every binned record has
# k3 == the colour's opacity).  Other blends still expect 32-B records, so
# only 16x16 whole frames without big lists are valid with this build.
p = "gs_kernels.hip"
s = open(p).read()
rep = [
("""    float4* const sw = s_rec[wave];
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
""", """    float* const sf = reinterpret_cast<float*>(s_rec[wave]);
    sf[5 * lane + 0] = r2[0].x;
    sf[5 * lane + 1] = r2[0].y;
    sf[5 * lane + 2] = r2[0].z;
    sf[5 * lane + 3] = r2[0].w;
    sf[5 * lane + 4] = r2[1].x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int i0 = blk * 256 + wave * 64;  // the wave's first Gaussian
#pragma unroll
    for (int h = 0; h < 5; ++h) {
      const int k = 64 * h + lane;  // float k of the wave's 20-B records: record i0 + k / 5
      if (i0 + k / 5 < fp.n)
        __builtin_nontemporal_store(sf[k], reinterpret_cast<float*>(b.rec) + 5 * (size_t)i0 + k);
    }
"""),
("""  auto load_rec = [&](uint32_t g, float4& r0, float4& r1, float4& r2) {
    const float4* qq = b.rec + 2 * (size_t)g;
    r0 = qq[0];
    const float4 t = qq[1];    // k1 pcut boxx boxy
    const float4 c = ccol[g];  // r g b opacity
    r1 = make_float4(t.x, t.y, c.x, c.y);
    r2 = make_float4(c.z, c.w, t.z, t.w);
  };
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0;
  uint32_t g_cur = load_idx(lane);""", """  auto load_rec = [&](uint32_t g, float4& r0, float4& r1, float4& r2) {
    const float* qq = reinterpret_cast<const float*>(b.rec) + 5 * (size_t)g;
    r0 = make_float4(qq[0], qq[1], qq[2], qq[3]);
    const float k1 = qq[4];
    const float4 c = ccol[g];  // r g b opacity
    float pcut;
    uint32_t b01, b23;
    alpha_footprint(r0.x, r0.y, r0.z, k1, r0.w, c.w, fp, pcut, b01, b23);
    r1 = make_float4(k1, pcut, c.x, c.y);
    r2 = make_float4(c.z, c.w, __uint_as_float(b01), __uint_as_float(b23));
  };
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0;
  uint32_t g_cur = load_idx(lane);"""),
]
for a, b_ in rep:
    assert s.count(a) >= 1, a[:60]
    i = s.rindex(a)  # (the two-pixel blend's load_rec is the file's last)
    s = s[:i] + b_ + s[i + len(a):]
open(p, "w").write(s)
