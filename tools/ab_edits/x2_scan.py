# Sensitivity probe (never shipped): the multi-workgroup tile scan launched
# twice per frame (it rewrites the same starts, queues and counters).
p = "gs_kernels.hip"
s = open(p).read()
line = "    gs_scan_multi_kernel<<<(fp.n_tiles + 63) / 64, 256, 0, s>>>(fp, b);\n"
assert s.count(line) == 1
s = s.replace(line, line + line)
open(p, "w").write(s)
