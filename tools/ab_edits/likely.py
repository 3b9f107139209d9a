s = open("gs_kernels.hip").read()
a = s.count("if (__builtin_expect(upda, 0))")
s = s.replace("if (__builtin_expect(upda, 0))", "if (upda)").replace("if (__builtin_expect(updb, 0))", "if (updb)")
assert a == 1
open("gs_kernels.hip", "w").write(s)
