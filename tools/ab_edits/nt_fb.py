# Non-temporal accesses (A/B variants; environment flags choose them):
#   NT_RGBA   the RGBA f32 pixels the blend writes once per frame
#   NT_BGR    the BGR8 bytes likewise
#   NT_SCENE  the projection's once-per-frame scene reads (mean + opacity,
#             the cached covariances)
# so that once-touched bytes do not displace the records and lists of the
# frames in flight.
import os

p = "gs_kernels.hip"
s = open(p).read()
if os.environ.get("NT_RGBA"):
    old = "  if (fp.write_rgba) b.rgba[(size_t)row * fp.width + px] = make_float4(o0, o1, o2, o3);\n"
    new = """  typedef float v4f __attribute__((ext_vector_type(4)));
  if (fp.write_rgba) {
    v4f v = {o0, o1, o2, o3};
    __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(b.rgba + (size_t)row * fp.width + px));
  }
"""
    assert s.count(old) == 1
    s = s.replace(old, new)
if os.environ.get("NT_BGR"):
    old = """  dst[0] = to_u8(o2);  // RGBA2BGR
  dst[1] = to_u8(o1);
  dst[2] = to_u8(o0);"""
    new = """  __builtin_nontemporal_store(to_u8(o2), dst);  // RGBA2BGR
  __builtin_nontemporal_store(to_u8(o1), dst + 1);
  __builtin_nontemporal_store(to_u8(o0), dst + 2);"""
    assert s.count(old) == 1
    s = s.replace(old, new)
if os.environ.get("NT_SCENE"):
    old2 = "    const float4 mo = b.mean_op[i];\n"
    assert s.count(old2) == 1
    s = s.replace(old2, "    typedef float v4f __attribute__((ext_vector_type(4)));\n"
                  "    const v4f mv = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(b.mean_op + i));\n"
                  "    const float4 mo = make_float4(mv.x, mv.y, mv.z, mv.w);\n")
    old3 = "      for (int k = 0; k < 9; ++k) c3[k] = b.cov3[k * nn + i];\n"
    assert s.count(old3) == 2
    s = s.replace(old3, "      for (int k = 0; k < 9; ++k) c3[k] = __builtin_nontemporal_load(b.cov3 + k * nn + i);\n")
    old4 = "    sg = make_float4(0.f, 0.f, 0.f, b.cov3[9 * nn + i]);\n"
    assert s.count(old4) == 1
    s = s.replace(old4, "    sg = make_float4(0.f, 0.f, 0.f, __builtin_nontemporal_load(b.cov3 + 9 * nn + i));\n")
open(p, "w").write(s)
