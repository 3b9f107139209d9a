"""VALU cycles per instruction of the frame kernels' hot loops (CPU; gfx950
ISA from hipcc, per-instruction SIMD costs measured on the MI355X by
tools/hip/valu_rate.hip).

The MI355X SIMD does not issue every VALU instruction at one rate
(tools/hip/valu_rate.hip, eight waves per SIMD, profiles/r06_probe/
valu_rate_operands.json): the FP32 add / sub / mul / fma family and the
plain moves and bitwise ops take ~2.1-2.5 SIMD cycles per wave64 instruction
when every source is a VGPR, an inline constant or a literal (a v_fma_f32 of
three VGPRs 2.46, the MI355X_MICROARCH.md "2 cyc" row) and ~4.1-4.2 when a
source is an SGPR (the round-5 benchmark's form, v_fma_f32 v8, s3, v8, v1:
4.17) or the same VGPR bank is read twice (v_fmac_f32 of one register twice:
4.14); min / max / compares / conversions / rndne / ldexp / ffbl / shifts /
cndmask / integer multiplies and every v_pk_* ~4.1-4.2 whatever the sources
(a packed FMA does two lanes' worth); v_exp / v_sqrt / v_rcp ~8.1.  So
SQ_INSTS_VALU alone does not say how busy the VALU pipe is.  This tool weighs each kernel's innermost loop -- the blocks LLVM
annotates "in Loop: Header=... Depth=<max>", the loop with the most VALU
instructions -- by those costs and writes

  {kernel short name: {"cpi": cycles / instruction, "loop_valu": n,
                       "loop_cycles": c, "source": ...}}

to profiles/valu_cpi.json, which bench.py uses for the roofline's
`valu_issue_frac` (SQ_INSTS_VALU x cpi over 1 024 SIMDs x 2.4 GHz x the
launch time).  Static: one pass through the loop body with every branch
taken (the blend's two update blocks included).

  python tools/valu_cpi.py [--rates profiles/r06_probe/valu_rate_operands.json] [--out profiles/valu_cpi.json]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gaussian_splat_ipu_amd", "csrc", "gs_kernels.hip")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "--cuda-device-only", "-S"]

# kernel short name (bench / rocprof) -> mangled symbol prefix
KERNELS = {
    "gs_blend_px2": "_ZN3gsk12_GLOBAL__N_119gs_blend_px2_kernelILb0EEEvNS_11FrameParamsENS_7BuffersE",
    "gs_blend": "_ZN3gsk12_GLOBAL__N_115gs_blend_kernelILi4ELb0EEEvNS_11FrameParamsENS_7BuffersE",
    "gs_blend_sort": "_ZN3gsk12_GLOBAL__N_120gs_blend_sort_kernelILb0EEEvNS_11FrameParamsENS_7BuffersE",
    "gs_blend_direct": "_ZN3gsk12_GLOBAL__N_122gs_blend_direct_kernelILb0EEEvNS_11FrameParamsENS_7BuffersE",
    "gs_blend_cont": "_ZN3gsk12_GLOBAL__N_120gs_blend_cont_kernelILb0EEEvNS_11FrameParamsENS_7BuffersE",
}


# the FP32 add / mul / fma family and plain moves / bitwise / u32 adds: full
# rate (2.1-2.5 cycles) unless a source is an SGPR or two sources share a VGPR
# bank (reg % 4), then 4.1-4.2
FAST = {"v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_fma_f32", "v_fmac_f32", "v_fmamk_f32",
        "v_fmaak_f32", "v_mov_b32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_add_u32", "v_sub_u32",
        "v_subrev_u32", "v_not_b32"}


def rates(path):
    """op -> cycles: the eight-waves-per-SIMD entries of a valu_rate run, plus
    the operand-kind rows ("fast": a FAST op with VGPR / constant sources,
    "fast_sgpr": with an SGPR source)."""
    out = {}
    for e in json.load(open(path)):
        if e.get("waves_per_simd") != 8 or e.get("chains") != 8:
            continue
        c = e.get("simd_cycles_per_inst", e.get("simd_cycles_per_inst_at_2.4GHz"))
        if e["op"] == "v_cndmask_b32" and c > 8:
            continue  # (a first run read a VALU-written vcc: its hazard, not the instruction's rate)
        out[e["op"]] = c
    fast = [out[k] for k in ("bv_v_mul_f32_vgpr", "bv_v_add_f32_vgpr", "bv_v_fma_f32_vgpr", "bv_v_mul_f32_inline",
                             "bv_v_mul_f32_literal", "v_mul_f32", "v_add_u32", "v_and_b32", "v_mov_b32") if k in out]
    slow = [out[k] for k in ("bi_v_fma_f32", "bi_v_mul_f32", "bi_v_add_f32") if k in out]
    out["fast"] = sum(fast) / len(fast) if fast else 2.0
    out["fast_sgpr"] = sum(slow) / len(slow) if slow else 4.0
    return out


def sources(line):
    """The source operands of an ISA line (everything after the destination;
    a VOPC compare's vcc / SGPR-pair destination included as written)."""
    t = line.strip().split(None, 1)
    if len(t) < 2:
        return []
    ops = [o.strip() for o in t[1].split(",")]
    return ops[1:]


def vbank(o):
    m = re.fullmatch(r"v(\d+)", o) or re.fullmatch(r"v\[(\d+):\d+\]", o)
    return int(m.group(1)) % 4 if m else None


def cost(op, table, line=""):
    base = re.sub(r"_e(32|64|64_dpp|32_dpp|_sdwa)$", "", op)
    if base in FAST:
        src = sources(line)
        sg = any(re.match(r"^-?\|?s(\d+|\[)", o) for o in src)
        banks = [vbank(o.lstrip("-|")) for o in src]
        banks = [b for b in banks if b is not None]
        clash = len(banks) != len(set(banks))
        return (table["fast_sgpr"] if (sg or clash) else table["fast"]), True
    if base in table:
        return table[base], True
    for alias, to in (("v_cvt_u32_f32", "v_cvt_i32_f32"), ("v_cvt_f32_i32", "v_cvt_f32_u32"),
                      ("v_lshrrev_b32", "v_lshlrev_b32"), ("v_ashrrev_i32", "v_lshlrev_b32"),
                      ("v_min_i32", "v_min_u32"), ("v_max_u32", "v_min_u32"), ("v_max_i32", "v_min_u32"),
                      ("v_bfe_i32", "v_bfe_u32"), ("v_mov_b64", "v_lshl_add_u64"), ("v_subbrev_co_u32", "v_add_u32")):
        if base == alias and to in table:
            return table[to], True
    if base.startswith("v_cmp"):
        return table.get("v_cmp_lt_f32", 4.0), True
    if base.startswith("v_pk_"):
        return table.get("v_pk_fma_f32", 4.0), True
    return 4.0, False  # unmeasured: the 4-cycle class


def hot_loop(body):
    """The innermost loop with the most VALU instructions: its instructions."""
    blocks, cur, label, info = [], [], None, ""
    for line in body.splitlines():
        m = re.match(r"^(\.LBB\d+_\d+):\s*(;.*)?$", line)
        m2 = re.match(r"^; %bb\.\d+:\s*(;.*)?$", line.strip()) if not m else None
        if m or m2:
            blocks.append((label, info, cur))
            label = m.group(1) if m else None
            info = (m.group(2) if m else m2.group(1)) or ""
            cur = []
            continue
        if line.strip().startswith(";") and cur == [] and "Loop" in line:
            info += " " + line.strip()
            continue
        cur.append(line)
    blocks.append((label, info, cur))
    loops = {}
    for label, info, ins in blocks:
        m = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", info)
        h = re.search(r"Loop Header: Depth=(\d+)", info)
        if m:
            key, d = "BB" + m.group(1), int(m.group(2))
        elif h and label:
            key, d = label.lstrip(".L"), int(h.group(1))  # .LBB24_49 -> BB24_49
        else:
            continue
        loops.setdefault((key, d), []).extend(ins)
    if not loops:
        return None, 0
    dmax = max(d for _, d in loops)
    cand = [(k, v) for k, v in loops.items() if k[1] == dmax]
    # the blends instantiate their record loop per exponential: the in-range
    # one (v_ldexp_f32; every batch whose records all have pcut >= -80, i.e.
    # nearly all) rather than the clamped one of the rare other batches
    inr = [kv for kv in cand if any(l.strip().startswith("v_ldexp_f32") for l in kv[1])]
    best = max(inr or cand, key=lambda kv: sum(1 for l in kv[1] if l.strip().startswith("v_")))
    return best[1], dmax


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default=os.path.join(ROOT, "profiles", "r06_probe", "valu_rate_operands.json"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "valu_cpi.json"))
    ap.add_argument("--isa", default=None, help="an existing gs_kernels.hip ISA listing (else hipcc makes one)")
    a = ap.parse_args()
    table = rates(a.rates)
    isa = a.isa
    if isa is None:
        fd, isa = tempfile.mkstemp(suffix=".s")
        os.close(fd)
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, SRC, "-o", isa], check=True)
    s = open(isa).read()
    out = {}
    for short, sym in KERNELS.items():
        i = s.find(sym + ":")
        if i < 0:
            print(f"{short}: not in the listing", file=sys.stderr)
            continue
        body = s[i:s.find(".Lfunc_end", i)]
        ins, depth = hot_loop(body)
        if not ins:
            continue
        n = cyc = 0
        unmeasured = set()
        for line in ins:
            t = line.strip().split()
            if not t or not t[0].startswith("v_"):
                continue
            c, known = cost(t[0], table, line)
            n += 1
            cyc += c
            if not known:
                unmeasured.add(t[0])
        out[short] = {"cpi": round(cyc / n, 3), "loop_valu": n, "loop_cycles": round(cyc, 1), "loop_depth": depth,
                      "unmeasured_ops_at_4": sorted(unmeasured),
                      "source": "gs_kernels.hip hot loop, static (every block once), "
                                f"costs {os.path.relpath(a.rates, ROOT)}"}
        print(short, out[short])
    json.dump(out, open(a.out, "w"), indent=1)
    if a.isa is None:
        os.unlink(isa)


if __name__ == "__main__":
    main()
