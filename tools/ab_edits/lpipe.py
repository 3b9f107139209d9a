# px2 record loop with the next record's LDS reads issued before the current
# record's arithmetic (two register sets, loop unrolled by two)
s = open("gs_kernels.hip").read()
i = s.find("template <int EXP>\n__device__ __forceinline__ void blend_records_px2(")
j = s.find("// wid = (tile slot) * 2 + half; st: the wave's LDS staging of one batch")
assert i > 0 and j > i
new = r'''template <int EXP>
__device__ __forceinline__ bool px2_step(Px& qa, Px& qb, const float4& a0, const float4& a1, const float4& a2) {
  const float h0 = a0.z, h2 = a0.w, k1 = a1.x;
  const float dy = a0.y - qa.p.y;
  const float h2dd = h2 * dy * dy;
  const float dxa = a0.x - qa.p.x, dxb = a0.x - qb.p.x;
  const float pa = (h0 * dxa * dxa + h2dd) - k1 * dxa * dy;
  const float pb = (h0 * dxb * dxb + h2dd) - k1 * dxb * dy;
  const float ea = EXP == kExpHw ? gs_expf_hw(pa) : (EXP == kExpInRange ? gs_expf_inrange(pa) : gs_expf(pa));
  const float eb = EXP == kExpHw ? gs_expf_hw(pb) : (EXP == kExpInRange ? gs_expf_inrange(pb) : gs_expf(pb));
  const float pcut = a1.y, op = a2.y;
  const float va = op * ea, vb = op * eb;
  const float ala = (va < 0.99f) ? va : 0.99f, alb = (vb < 0.99f) ? vb : 0.99f;
  const float tta = qa.T * (1.0f - ala), ttb = qb.T * (1.0f - alb);
  asm volatile("" ::"v"(ala), "v"(alb), "v"(tta), "v"(ttb));
  const bool hita = !qa.done && !(pa > 0.0f) && !(pa < pcut) && !(ala < 1.0f / 255.0f);
  const bool hitb = !qb.done && !(pb > 0.0f) && !(pb < pcut) && !(alb < 1.0f / 255.0f);
  const bool brka = hita && tta < 0.0001f, brkb = hitb && ttb < 0.0001f;
  const bool upda = hita && !brka, updb = hitb && !brkb;
  if (upda) {
    qa.c01.x = qa.c01.x + (a1.z * ala) * qa.T;
    qa.c01.y = qa.c01.y + (a1.w * ala) * qa.T;
    qa.c23.x = qa.c23.x + (a2.x * ala) * qa.T;
    qa.c23.y = qa.c23.y + (op * ala) * qa.T;
    qa.T = tta;
  }
  if (updb) {
    qb.c01.x = qb.c01.x + (a1.z * alb) * qb.T;
    qb.c01.y = qb.c01.y + (a1.w * alb) * qb.T;
    qb.c23.x = qb.c23.x + (a2.x * alb) * qb.T;
    qb.c23.y = qb.c23.y + (op * alb) * qb.T;
    qb.T = ttb;
  }
  qa.done = qa.done || brka;
  qb.done = qb.done || brkb;
  return qa.done && qb.done;
}

template <int EXP>
__device__ __forceinline__ void blend_records_px2(Px& qa, Px& qb, float4 (*st)[64], uint32_t w, uint32_t h) {
  unsigned long long m = ((unsigned long long)h << 32) | w;
  if (!m) return;
  int j = __builtin_ctzll(m);
  float4 a0 = st[0][j], a1 = st[1][j], a2 = st[2][j];
  while (true) {
    m &= m - 1ull;
    j = m ? __builtin_ctzll(m) : j;
    const float4 b0 = st[0][j], b1 = st[1][j], b2 = st[2][j];  // the next record's reads, issued first
    if (px2_step<EXP>(qa, qb, a0, a1, a2) || !m) break;
    m &= m - 1ull;
    j = m ? __builtin_ctzll(m) : j;
    a0 = st[0][j];
    a1 = st[1][j];
    a2 = st[2][j];
    if (px2_step<EXP>(qa, qb, b0, b1, b2) || !m) break;
  }
}

'''
s = s[:i] + new + s[j:]
open("gs_kernels.hip", "w").write(s)
