# Sensitivity probe (never shipped): the chunk count launched twice per frame
# (it rewrites the same chunk rows before the column scan).
p = "gs_kernels.hip"
s = open(p).read()
line = "    gs_count_kernel<<<fp.n_chunks, 1024, lds, s>>>(fp, b);\n"
assert s.count(line) == 1
s = s.replace(line, line + line)
open(p, "w").write(s)
