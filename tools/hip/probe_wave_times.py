"""Edit script for tools/build_variant_from.sh (run inside csrc/): a probe build
in which every blend wave writes (start, end, batches staged, 0) as raw u32
(s_memrealtime, 100 MHz) into the RGBA f32 pixel of its lane 0 after the
frame's own store; tools/wave_times.py reads them back.  Not a product build."""
p = "gs_kernels.hip"
s = open(p).read()
old = """  const int wave = GS_BLEND_WPG == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wid = blk * GS_BLEND_WPG + wave;"""
new = """  const unsigned long long probe_t0 = __builtin_amdgcn_s_memrealtime();
  const int wave = GS_BLEND_WPG == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wid = blk * GS_BLEND_WPG + wave;"""
assert old in s
s = s.replace(old, new)
old = """  blend_count_store(fp, b, wid, staged);
  if (valid) store_pixel(fp, b, px, tyb * fp.tile_h + ly, q);
}"""
new = """  blend_count_store(fp, b, wid, staged);
  if (valid) store_pixel(fp, b, px, tyb * fp.tile_h + ly, q);
  const unsigned long long probe_t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0 && valid && fp.write_rgba)
    b.rgba[(size_t)(tyb * fp.tile_h + ly) * fp.width + px] =
        make_float4(__uint_as_float((uint32_t)probe_t0), __uint_as_float((uint32_t)probe_t1),
                    __uint_as_float(staged / 64u), 0.0f);
}"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
