# A/B: non-temporal loads at the last reader of per-frame intermediates
# (the count's rectangles, the emit's culled rectangles and depth keys, the
# tile sort's pairs), on top of the shipped streaming scene reads / RGBA stores.
p = "gs_kernels.hip"
s = open(p).read()
rep = [
    ("          rr[k] = rect8_unpack(live[k] ? reinterpret_cast<const uint32_t*>(b.rect)[i] : 0x00010001u);\n",
     "          rr[k] = rect8_unpack(live[k] ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(b.rect) + i) : 0x00010001u);\n", 1),
    ("          r[k] = rect8_unpack(live[k] ? reinterpret_cast<const uint32_t*>(b.crect)[i] : 0x00010001u);\n",
     "          r[k] = rect8_unpack(live[k] ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(b.crect) + i) : 0x00010001u);\n", 1),
    ("        dk[k] = live[k] ? b.depth_key[i] : 0u;\n",
     "        dk[k] = live[k] ? __builtin_nontemporal_load(b.depth_key + i) : 0u;\n", 1),
    ("    v[e] = i < L ? src[i] : ~0ull;\n", "    v[e] = i < L ? __builtin_nontemporal_load(src + i) : ~0ull;\n", 1),
    ("      else v[e] = i < L ? b.pairs[s + i] : ~0ull;\n", "      else v[e] = i < L ? __builtin_nontemporal_load(b.pairs + s + i) : ~0ull;\n", 1),
]
for a, b_, n in rep:
    assert s.count(a) == n, a
    s = s.replace(a, b_)
open(p, "w").write(s)
