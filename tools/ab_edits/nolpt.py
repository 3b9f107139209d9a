# px2 blend in plain tile order (no LPT, no seg table): the XCD variant's control
r = open("gs_renderer.hip").read()
r = r.replace('''  if (fp.blend_px2) fp.blend_lpt = 1;''', '''  if (fp.blend_px2) fp.blend_lpt = 0;''')
old = '''  fp.blend_seg = (fp.blend_px2 && !fp.big_separate) ? 1 : 0;'''
assert old in r
r = r.replace(old, '''  fp.blend_seg = 0;''')
open("gs_renderer.hip", "w").write(r)
