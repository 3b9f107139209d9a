# tools/build_variant.sh edit (runs inside the copied csrc/): the GS_LANES
# counting build of tools/blend_lanes.py -- the same sources with the blend's
# lane counters compiled in.
p = "gs_kernels.hpp"
s = open(p).read()
old = "#ifndef GS_LANES\n#define GS_LANES 0\n#endif"
assert old in s
open(p, "w").write(s.replace(old, "#define GS_LANES 1"))
