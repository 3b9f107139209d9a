# A/B: the streaming RGBA stores on whole frames only (row bands plain).
p = "gs_kernels.hip"
s = open(p).read()
a = "  if (fp.write_rgba) store_stream(b.rgba + (size_t)row * fp.width + px, make_float4(o0, o1, o2, o3));\n"
assert s.count(a) == 1
s = s.replace(a, """  if (fp.write_rgba) {
    if (fp.band_cull)
      b.rgba[(size_t)row * fp.width + px] = make_float4(o0, o1, o2, o3);
    else
      store_stream(b.rgba + (size_t)row * fp.width + px, make_float4(o0, o1, o2, o3));
  }
""")
open(p, "w").write(s)
