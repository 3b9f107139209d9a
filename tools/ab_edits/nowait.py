s = open("gs_group.hip").read()
old = '''    if (f.prev >= 0) GS_HIP(hipStreamWaitEvent(rs, m.ev_render[f.prev], 0));
    gsk::launch_copy_word'''
assert old in s
s = s.replace(old, "    gsk::launch_copy_word")
open("gs_group.hip", "w").write(s)
