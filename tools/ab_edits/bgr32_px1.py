# A/B: the one-pixel blend's BGR8 bytes (8x8 quad blocks, BQW = 4: config
# 5's whole frames, the row bands' in-blend sort, the continuation) through
# the wave's idle LDS and out as whole dwords (one store instruction per wave
# instead of three byte stores per lane), for blocks wholly inside the image
# and 4-B aligned rows.
p = "gs_kernels.hip"
s = open(p).read()
a = """  if (fp.blend_cont && lane == 0) b.cont_flag[4 * jb + chunk] = 0u;  // this wave is done
  blend_count_store(fp, b, wid, staged);
  if (valid) store_pixel(fp, b, px, tyb * fp.tile_h + ly, q);
}
"""
b_ = """  if (fp.blend_cont && lane == 0) b.cont_flag[4 * jb + chunk] = 0u;  // this wave is done
  blend_count_store(fp, b, wid, staged);
  if constexpr (BQW == 4) {
    const bool dw = nq_wave == 16 && q_x + 8 <= fp.tile_w && q_y + 8 <= fp.tile_h &&
                    tile_x0 + q_x + 8 <= fp.width && ((uintptr_t)b.bgr & 3u) == 0u && (fp.bgr_pitch & 3) == 0;
    if (dw) {
      if (fp.write_rgba && valid) store_stream(b.rgba + (size_t)(tyb * fp.tile_h + ly) * fp.width + px, pixel_rgba(q));
      uint8_t* const sb = reinterpret_cast<uint8_t*>(&st[0][0]);  // 8 rows x 24 B (the staging is idle)
      __builtin_amdgcn_wave_barrier();
      const float4 o = pixel_rgba(q);
      uint8_t* const d = sb + (ly - q_y) * 24 + 3 * (lx - q_x);
      d[0] = to_u8(o.z);  // RGBA2BGR
      d[1] = to_u8(o.y);
      d[2] = to_u8(o.x);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < 48) {  // dword lane of the block's 48: row lane / 6, dword lane % 6
        const int r = lane / 6, c = lane - 6 * r;
        if (tile_y0 + q_y + r < fp.height)
          *reinterpret_cast<uint32_t*>(b.bgr + (size_t)(tyb * fp.tile_h + q_y + r) * fp.bgr_pitch +
                                       3 * (size_t)(tile_x0 + q_x) + 4 * c) = reinterpret_cast<const uint32_t*>(sb)[lane];
      }
      return;
    }
  }
  if (valid) store_pixel(fp, b, px, tyb * fp.tile_h + ly, q);
}
"""
assert s.count(a) == 1
s = s.replace(a, b_)
open(p, "w").write(s)
