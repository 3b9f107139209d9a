# gs_expf2_inrange: rint by the 1.5 * 2^23 addition, 2^k from the sum's bits
s = open("gs_kernels.hip").read()
old = '''  const float ka = __builtin_rintf(xa * 1.44269502162933349609f), kb = __builtin_rintf(xb * 1.44269502162933349609f);
  const f32x2 k = f32x2{ka, kb};'''
new = '''  const float ma = xa * 1.44269502162933349609f + 12582912.0f, mb = xb * 1.44269502162933349609f + 12582912.0f;
  const float ka = ma - 12582912.0f, kb = mb - 12582912.0f;
  const f32x2 k = f32x2{ka, kb};'''
assert old in s
s = s.replace(old, new)
old = '''  return f32x2{__builtin_amdgcn_ldexpf(p.x + 1.0f, (int)ka), __builtin_amdgcn_ldexpf(p.y + 1.0f, (int)kb)};'''
new = '''  return f32x2{(p.x + 1.0f) * __uint_as_float((__float_as_uint(ma) + (127u - 0x4B400000u)) << 23),
               (p.y + 1.0f) * __uint_as_float((__float_as_uint(mb) + (127u - 0x4B400000u)) << 23)};'''
assert old in s
s = s.replace(old, new)
open("gs_kernels.hip", "w").write(s)
