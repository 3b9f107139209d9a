# A/B: the tile sort as two launches -- big + medium lists (16.6-KB LDS
# workgroups), then the small lists with only the waves' tie slices in LDS
# (8 KB), so that the small lists' workgroups fit beside the other frames'.
p = "gs_kernels.hip"
s = open(p).read()
rep = [
("""template <int NT>
__device__ __forceinline__ void sort_tiles(const FrameParams& fp, const Buffers& b) {
  constexpr int NW = NT / 64;
  // the radix path's histograms alias the merge path's key buffer (a
  // workgroup takes one path)
  constexpr int kRadixWords = 8 * 256 + 256 + NW * 256;
  constexpr int kWords = 2 * kSortLdsCap > kRadixWords ? 2 * kSortLdsCap : kRadixWords;
""", """template <int NT, int PART = 0>
__device__ __forceinline__ void sort_tiles(const FrameParams& fp, const Buffers& b) {
  constexpr int NW = NT / 64;
  // the radix path's histograms alias the merge path's key buffer (a
  // workgroup takes one path)
  constexpr int kRadixWords = 8 * 256 + 256 + NW * 256;
  constexpr int kWords = PART == 2 ? 2 * NW * kSortRegCap
                                   : (2 * kSortLdsCap > kRadixWords ? 2 * kSortLdsCap : kRadixWords);
"""),
("""  if (blockIdx.x < n_big) {  // the longest lists first
    const uint32_t t = b.big_tiles[blockIdx.x];""", """  if constexpr (PART == 2) {
    const uint32_t n_med = b.counters[7], n_small = b.counters[9];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t k = blockIdx.x * (uint32_t)NW + (uint32_t)wave;
    if (k >= n_small) return;
    const int lane = threadIdx.x & 63;
    uint32_t s, L;
    const uint32_t t = b.small_tiles[k];
    tile_segment(fp, b, (int)t, s, L);
    put_seg(n_big + n_med + k, t, s, L);
    wave_sort_list(b, b.pairs + s, s, L, lane, keys + wave * kSortRegCap);
    return;
  } else {
  if (blockIdx.x < n_big) {  // the longest lists first
    const uint32_t t = b.big_tiles[blockIdx.x];"""),
("""      merge_sort_tile<NT, 2, kOutInput, kSrcRekey>(b, s, L, keys);
    }
    return;
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t k = (item - n_med) * (uint32_t)NW + (uint32_t)wave;""", """      merge_sort_tile<NT, 2, kOutInput, kSrcRekey>(b, s, L, keys);
    }
    return;
  }
  if constexpr (PART == 1) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t k = (item - n_med) * (uint32_t)NW + (uint32_t)wave;"""),
("""  unsigned long long* const slice = keys + wave * kSortRegCap;
  wave_sort_list(b, b.pairs + s, s, L, lane, slice);
}
""", """  unsigned long long* const slice = keys + wave * kSortRegCap;
  wave_sort_list(b, b.pairs + s, s, L, lane, slice);
  }
}
"""),
("""  sort_tiles<256>(fp, b);
}
""", """  sort_tiles<256>(fp, b);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_sort_tiles_bm_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrSortTiles);
  sort_tiles<256, 1>(fp, b);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void gs_sort_tiles_small_kernel(FrameParams fp, Buffers b) {
  GS_PROBE_SCOPE(kPrSortTiles);
  sort_tiles<256, 2>(fp, b);
}
"""),
("""  gs_sort_tiles_kernel<<<fp.n_tiles + (fp.n_tiles + 3) / 4, 256, 0, s>>>(fp, b);
""", """  gs_sort_tiles_bm_kernel<<<fp.n_tiles, 256, 0, s>>>(fp, b);
  gs_sort_tiles_small_kernel<<<(fp.n_tiles + 3) / 4, 256, 0, s>>>(fp, b);
"""),
]
for a, b_ in rep:
    assert s.count(a) == 1, a[:70]
    s = s.replace(a, b_)
open(p, "w").write(s)
