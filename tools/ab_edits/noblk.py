s = open("gs_renderer.hip").read()
old = "fp.block_list = fp.band_cull;"
assert old in s
open("gs_renderer.hip", "w").write(s.replace(old, "fp.block_list = 0;"))
