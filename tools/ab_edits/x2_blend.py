# Sensitivity probe (never shipped): the blend stage launched twice per frame
# (idempotent: the second launch rewrites the same outputs), to read the
# stage's marginal cost in the pipelined frame.
p = "gs_renderer.hip"
s = open(p).read()
line = "  gsk::launch_blend(fb, r->buf, s);\n"
i = s.index("int enqueue_frame(")
j = s.index(line, i)
s = s[:j] + line + s[j:]
open(p, "w").write(s)
