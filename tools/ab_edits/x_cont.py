# Sensitivity probe (never shipped; its frames are wrong where a lazy list
# outlives its prefix): config 5 without the continuation's pass 2
# (CONT=p1) or without the continuation at all (CONT=none), to bound what
# shortening that chain could give.
import os
p = "gs_kernels.hip"
s = open(p).read()
if os.environ["CONT"] == "none":
    a = "  if (waves == 0 || !fp.lazy) return;\n"
    assert s.count(a) == 1
    s = s.replace(a, "  if (waves == 0 || !fp.lazy || waves > 0) return;\n")
else:
    a = "  FrameParams f2 = fp;\n  f2.big_pass = 2;\n"
    assert s.count(a) == 1
    s = s.replace(a, "  if (waves > 0) return;\n" + a)
open(p, "w").write(s)
