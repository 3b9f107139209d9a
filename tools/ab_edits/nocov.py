# A/B: no covariance cache (the projection computes ComputeCov3D from the
# rotation and scales again), those reads streamed on whole frames.
p = "gs_renderer.hip"
s = open(p).read()
a = "  fp.cov_cache = r->d_cov ? 1 : 0;\n"
assert s.count(a) == 1
s = s.replace(a, "  fp.cov_cache = 0;\n")
open(p, "w").write(s)
p = "gs_kernels.hip"
s = open(p).read()
rep = [("    sg = b.scale_gid[i];\n", "    sg = fp.band_cull ? b.scale_gid[i] : load_stream(b.scale_gid + i);\n", 1),
       ("    } else {\n      rot = b.rot[i];\n", "    } else {\n      rot = load_stream(b.rot + i);\n", 1)]
for a, b_, n in rep:
    assert s.count(a) == n, a
    s = s.replace(a, b_)
open(p, "w").write(s)
