# px2 blend: tile order (no LPT, no seg table), each XCD (WG b -> b % 8) a
# contiguous band of tiles (L2 locality of the records neighbouring tiles share)
s = open("gs_kernels.hip").read()
old = '''__device__ __forceinline__ void blend_wave_px2(const FrameParams& fp, const Buffers& b, int wid, float4 (*st)[64]) {
  const int slot = wid >> 1, half = wid & 1;
  if (slot >= fp.n_tiles) return;
  int tile;
  uint32_t s, L;
  if (fp.blend_seg) {'''
new = '''__device__ __forceinline__ void blend_wave_px2(const FrameParams& fp, const Buffers& b, int wid, float4 (*st)[64]) {
  const int slot0 = wid >> 1, half = wid & 1;
  const int R2 = (((fp.n_tiles + 7) / 8) + 1) & ~1;
  const int bwg = slot0 >> 1, xcd = bwg & 7, li = 2 * (bwg >> 3) + (slot0 & 1);
  const int slot = xcd * R2 + li;
  if (li >= R2 || slot >= fp.n_tiles) return;
  int tile;
  uint32_t s, L;
  if (fp.blend_seg) {'''
assert old in s
s = s.replace(old, new)
old = '''    const unsigned g2 = (unsigned)((2L * fp.n_tiles + GS_PX2_WPG - 1) / GS_PX2_WPG);'''
new = '''    const unsigned g2 = (unsigned)(4 * ((((fp.n_tiles + 7) / 8) + 1) & ~1));'''
assert old in s
s = s.replace(old, new)
open("gs_kernels.hip", "w").write(s)
r = open("gs_renderer.hip").read()
old = '''  if (fp.blend_px2) fp.blend_lpt = 1;'''
assert old in r
r = r.replace(old, '''  if (fp.blend_px2) fp.blend_lpt = 0;''')
open("gs_renderer.hip", "w").write(r)
r = open("gs_renderer.hip").read()
old = '''  fp.blend_seg = (fp.blend_px2 && !fp.big_separate) ? 1 : 0;'''
assert old in r
r = r.replace(old, '''  fp.blend_seg = 0;''')
open("gs_renderer.hip", "w").write(r)
