# A/B: the two-pixel blend's BGR8 bytes through the wave's idle LDS and out
# as whole dwords (two store instructions per wave instead of six byte
# stores per lane), for tiles wholly inside the image and 4-B aligned rows.
p = "gs_kernels.hip"
s = open(p).read()
a = """  if (va) store_bgr(fp, b, px, tyb * fp.tile_h + ly, qa);
  if (vb) store_bgr(fp, b, px + 1, tyb * fp.tile_h + ly, qb);
}
"""
b_ = """  const bool dw = tile_x0 + 16 <= fp.width && ((uintptr_t)b.bgr & 3u) == 0u && (fp.bgr_pitch & 3) == 0;
  if (dw) {
    uint8_t* const sb = reinterpret_cast<uint8_t*>(&st[2][0]);  // 8 rows x 48 B (st[2] is idle)
    const float4 oa = pixel_rgba(qa), ob = pixel_rgba(qb);
    uint8_t* const d = sb + row * 48 + 3 * lx;
    d[0] = to_u8(oa.z);  // RGBA2BGR
    d[1] = to_u8(oa.y);
    d[2] = to_u8(oa.x);
    d[3] = to_u8(ob.z);
    d[4] = to_u8(ob.y);
    d[5] = to_u8(ob.x);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 64 * h + lane;  // dword k of the half tile's 96: row k / 12, dword k % 12
      if (k < 96) {
        const int r = k / 12, c = k - 12 * r;
        if (tile_y0 + 8 * half + r < fp.height)
          *reinterpret_cast<uint32_t*>(b.bgr + (size_t)(tyb * fp.tile_h + 8 * half + r) * fp.bgr_pitch +
                                       3 * (size_t)tile_x0 + 4 * c) = reinterpret_cast<const uint32_t*>(sb)[k];
      }
    }
  } else {
    if (va) store_bgr(fp, b, px, tyb * fp.tile_h + ly, qa);
    if (vb) store_bgr(fp, b, px + 1, tyb * fp.tile_h + ly, qb);
  }
}
"""
assert s.count(a) == 1
s = s.replace(a, b_)
open(p, "w").write(s)
