# px2 blend: 8x4-tile blocks, block k on XCD k % 8 (WG b -> XCD b % 8), the
# tiles of a block on one XCD (L2 locality of shared records), blocks spread
# over the XCDs (balance); no LPT, no seg table
s = open("gs_kernels.hip").read()
old = '''__device__ __forceinline__ void blend_wave_px2(const FrameParams& fp, const Buffers& b, int wid, float4 (*st)[64]) {
  const int slot = wid >> 1, half = wid & 1;
  if (slot >= fp.n_tiles) return;
  int tile;
  uint32_t s, L;
  if (fp.blend_seg) {'''
new = '''__device__ __forceinline__ void blend_wave_px2(const FrameParams& fp, const Buffers& b, int wid, float4 (*st)[64]) {
  const int slot0 = wid >> 1, half = wid & 1;
  const int bwg = slot0 >> 1, xcd = bwg & 7, li = bwg >> 3;
  const int nbx = (fp.tiles_x + 7) / 8, nby = (fp.band_nrows + 3) / 4;
  const int kb = xcd + 8 * (li >> 4), tt = 2 * (li & 15) + (slot0 & 1);
  if (kb >= nbx * nby) return;
  const int ttx = (kb % nbx) * 8 + (tt & 7), tty = (kb / nbx) * 4 + (tt >> 3);
  if (ttx >= fp.tiles_x || tty >= fp.band_nrows) return;
  const int slot = tty * fp.tiles_x + ttx;
  int tile;
  uint32_t s, L;
  if (fp.blend_seg) {'''
assert old in s
s = s.replace(old, new)
old = '''    const unsigned g2 = (unsigned)((2L * fp.n_tiles + GS_PX2_WPG - 1) / GS_PX2_WPG);'''
new = '''    const int nbk = ((fp.tiles_x + 7) / 8) * ((fp.band_nrows + 3) / 4);
    const unsigned g2 = (unsigned)(8 * ((nbk + 7) / 8) * 16);'''
assert old in s
s = s.replace(old, new)
open("gs_kernels.hip", "w").write(s)
r = open("gs_renderer.hip").read()
r = r.replace('''  if (fp.blend_px2) fp.blend_lpt = 1;''', '''  if (fp.blend_px2) fp.blend_lpt = 0;''')
old = '''  fp.blend_seg = (fp.blend_px2 && !fp.big_separate) ? 1 : 0;'''
assert old in r
r = r.replace(old, '''  fp.blend_seg = 0;''')
open("gs_renderer.hip", "w").write(r)
