exec(open("/tmp/abedit/blk.py").read())
s = open("gs_kernels.hip").read()
old = '''  const int kb = xcd + 8 * (li >> 4), tt = 2 * (li & 15) + (slot0 & 1);
  if (kb >= nbx * nby) return;'''
new = '''  const int kslot = xcd + 8 * (li >> 4), tt = 2 * (li & 15) + (slot0 & 1);
  if (kslot >= nbx * nby) return;
  const int kb = (int)((const uint32_t*)b.blend_seg)[kslot];  // the blocks, heaviest first'''
assert old in s
s = s.replace(old, new)
old = '''template <bool HWEXP>
__global__ __launch_bounds__(64 * GS_PX2_WPG) void gs_blend_px2_kernel(FrameParams fp, Buffers b) {'''
new = '''// the px2 blend's 8x4-tile blocks, heaviest first (their binned pairs),
// into blend_seg's words
__global__ __launch_bounds__(1024) void gs_blend_order_kernel(FrameParams fp, Buffers b) {
  __shared__ uint32_t w[1024];
  const int nbx = (fp.tiles_x + 7) / 8, nby = (fp.band_nrows + 3) / 4, nb = nbx * nby;
  uint32_t* order = (uint32_t*)b.blend_seg;
  const int k = threadIdx.x;
  if (nb > 1024) {
    for (int i = k; i < nb; i += 1024) order[i] = (uint32_t)i;
    return;
  }
  uint32_t wk = 0;
  if (k < nb) {
    const int bx = (k % nbx) * 8, by = (k / nbx) * 4;
    for (int t = 0; t < 32; ++t) {
      const int tx = bx + (t & 7), ty = by + (t >> 3);
      if (tx < fp.tiles_x && ty < fp.band_nrows) {
        const int tile = ty * fp.tiles_x + tx;
        wk += b.tile_start[tile + 1] - b.tile_start[tile];
      }
    }
  }
  w[k] = wk;
  __syncthreads();
  if (k < nb) {
    int rank = 0;
    for (int j = 0; j < nb; ++j) {
      const uint32_t wj = w[j];
      rank += (wj > wk || (wj == wk && j < k)) ? 1 : 0;
    }
    order[rank] = (uint32_t)k;
  }
}

template <bool HWEXP>
__global__ __launch_bounds__(64 * GS_PX2_WPG) void gs_blend_px2_kernel(FrameParams fp, Buffers b) {'''
assert old in s
s = s.replace(old, new)
old = '''    const int nbk = ((fp.tiles_x + 7) / 8) * ((fp.band_nrows + 3) / 4);
    const unsigned g2 = (unsigned)(8 * ((nbk + 7) / 8) * 16);'''
new = '''    const int nbk = ((fp.tiles_x + 7) / 8) * ((fp.band_nrows + 3) / 4);
    const unsigned g2 = (unsigned)(8 * ((nbk + 7) / 8) * 16);
    gs_blend_order_kernel<<<1, 1024, 0, s>>>(fp, b);'''
assert old in s
s = s.replace(old, new)
open("gs_kernels.hip", "w").write(s)
