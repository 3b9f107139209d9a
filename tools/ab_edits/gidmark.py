# A/B: the covariance cache without its gid plane: an empty slot (gid <= 0)
# is marked by a negative Sigma[2][2] (a live one's is a sum of squares,
# >= +0 or NaN), so the whole-frame projection streams 52 instead of 56 B
# per Gaussian.
p = "gs_kernels.hip"
s = open(p).read()
rep = [
    ("    sg = make_float4(0.f, 0.f, 0.f, load_stream(b.cov3 + 9 * nn + i));\n",
     "    sg = make_float4(0.f, 0.f, 0.f, 1.0f);  // (liveness: the sign of Sigma[2][2], below)\n", 1),
    ("      for (int k = 0; k < 9; ++k) c3[k] = load_stream(b.cov3 + k * nn + i);\n    } else {\n",
     "      for (int k = 0; k < 9; ++k) c3[k] = load_stream(b.cov3 + k * nn + i);\n      if (c3[8] < 0.0f) sg.w = 0.0f;\n    } else {\n", 1),
    ("  b.cov3[9 * nn + i] = sg.w;\n  if (sg.w <= 0.0f) return;  // (an empty slot: the projection skips it)\n",
     "  if (sg.w <= 0.0f) {  // (an empty slot: the projection skips it)\n    b.cov3[8 * nn + i] = -1.0f;\n    return;\n  }\n", 1),
]
for a, b_, n in rep:
    assert s.count(a) == n, a
    s = s.replace(a, b_)
open(p, "w").write(s)
