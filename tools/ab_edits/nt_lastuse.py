# A/B: streaming loads at the last reader of one per-frame intermediate
# (environment: NTL=list | pairs | emit): the blend's list entries, the tile
# sort's pairs, the emit's culled rectangles and depth keys.
import os
p = "gs_kernels.hip"
s = open(p).read()
kind = os.environ["NTL"]
if kind == "list":
    rep = [("__HIP_MEMORY_SCOPE_AGENT) : list[k];", "__HIP_MEMORY_SCOPE_AGENT) : __builtin_nontemporal_load(list + k);", 1)]
elif kind == "pairs":
    rep = [("    v[e] = i < L ? src[i] : ~0ull;\n", "    v[e] = i < L ? __builtin_nontemporal_load(src + i) : ~0ull;\n", 1),
           ("      else v[e] = i < L ? b.pairs[s + i] : ~0ull;\n", "      else v[e] = i < L ? __builtin_nontemporal_load(b.pairs + s + i) : ~0ull;\n", 1)]
else:
    rep = [("          r[k] = rect8_unpack(live[k] ? reinterpret_cast<const uint32_t*>(b.crect)[i] : 0x00010001u);\n",
            "          r[k] = rect8_unpack(live[k] ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(b.crect) + i) : 0x00010001u);\n", 1),
           ("        dk[k] = live[k] ? b.depth_key[i] : 0u;\n",
            "        dk[k] = live[k] ? __builtin_nontemporal_load(b.depth_key + i) : 0u;\n", 1)]
for a, b_, n in rep:
    assert s.count(a) == n, a
    s = s.replace(a, b_)
open(p, "w").write(s)
