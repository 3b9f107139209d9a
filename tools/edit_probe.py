# tools/build_variant.sh probe tools/edit_probe.py: the timeline probe build
# (GS_PROBE=1; run with GSPLAT_PROBE_FILE=<path>, read with tools/probe_timeline.py)
p = "gs_kernels.hpp"
s = open(p).read()
s = s.replace("#ifndef GS_PROBE\n#define GS_PROBE 0\n#endif", "#define GS_PROBE 1", 1)
open(p, "w").write(s)
