# A/B: whole-frame binning chunks of at least CHUNK Gaussians (default 4096):
# a smaller chunk x tile matrix (count writes it, the column scan reads and
# rewrites it, the emit reads it) against fewer count / emit workgroups.
import os
p = "gs_renderer.hip"
s = open(p).read()
a = "    size_t cs = std::max<size_t>(4096, (n + 255) / 256);\n"
assert s.count(a) == 1
s = s.replace(a, "    size_t cs = std::max<size_t>(%s, (n + 255) / 256);\n" % os.environ["CHUNK"])
open(p, "w").write(s)
