# A/B: the projection's 32-B records (read back by the blend's gathers after
# the binning and the sort) written as streaming stores.
p = "gs_kernels.hip"
s = open(p).read()
a = """      rec[0] = rec0;
      rec[1] = make_float4(k1, pcut, __uint_as_float(b01), __uint_as_float(b23));
"""
b_ = """      store_stream(rec, rec0);
      store_stream(rec + 1, make_float4(k1, pcut, __uint_as_float(b01), __uint_as_float(b23)));
"""
assert s.count(a) == 1
s = s.replace(a, b_)
open(p, "w").write(s)
