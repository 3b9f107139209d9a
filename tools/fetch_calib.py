"""FETCH_SIZE calibration (tools/hip/fetch_calib.hip): the factor between the
PMC counter and the bytes each access pattern really reads from HBM.

    hipcc --offload-arch=gfx950 -O3 tools/hip/fetch_calib.hip -o tools/hip/fetch_calib
    rocprofv3 --pmc FETCH_SIZE -d <dir> -o calib --output-format csv -- tools/hip/fetch_calib
    rocprofv3 --pmc WRITE_SIZE -d <dir>w -o calib --output-format csv -- tools/hip/fetch_calib
    python tools/fetch_calib.py <dir> [--json out.json]

Per kernel (gather32 split into its random-order and runs-of-8 launches by
dispatch order): FETCH_SIZE x 1024 over the bytes read (data + indices).
"""
import argparse
import collections
import csv
import glob
import json
import os

N = 1 << 24
BYTES = {  # data + streamed indices per launch (fetch_calib.hip)
    "stream16": N * 16,
    "gather32_random": N * 32 + N * 4,
    "gather32_runs8": N * 32 + N * 4,
    "gather16": N * 16 + N * 4,
    "gather4": N * 4 + N * 4,
    "store16": N * 16,
    "store16nt": N * 16,
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = []
    wacc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == "WRITE_SIZE":
                    if "store16" in r["Kernel_Name"]:
                        k = "store16nt" if "store16nt" in r["Kernel_Name"] else "store16"
                        wacc[k].append(float(r["Counter_Value"]) * 1024)
                    continue
                if r["Counter_Name"] != "FETCH_SIZE":
                    continue
                did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(rows))
                rows.append((did, r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    acc = collections.defaultdict(list)
    n32 = 0
    for _, name, v in rows:
        base = name.split("(")[0].split()[-1] if "(" in name else name
        for k in ("stream16", "gather32", "gather16", "gather4"):
            if k in base:
                if k == "gather32":
                    k = "gather32_random" if n32 % 2 == 0 else "gather32_runs8"
                    n32 += 1
                acc[k].append(v * 1024)
                break
    out = {}
    for k, vs in acc.items():
        vs = vs[1:] if len(vs) > 1 else vs  # (the first launch of each warms the TLB)
        mean = sum(vs) / len(vs)
        out[k] = {"launches": len(vs), "fetch_bytes": mean, "true_bytes": BYTES[k], "fetch_over_true": mean / BYTES[k]}
        print(f"{k:16s} FETCH_SIZE {mean / 1e6:9.1f} MB  true {BYTES[k] / 1e6:9.1f} MB  ratio {mean / BYTES[k]:.3f}")
    for k, vs in wacc.items():
        vs = vs[1:] if len(vs) > 1 else vs
        mean = sum(vs) / len(vs)
        out[k] = {"launches": len(vs), "write_bytes": mean, "true_bytes": BYTES[k], "write_over_true": mean / BYTES[k]}
        print(f"{k:16s} WRITE_SIZE {mean / 1e6:9.1f} MB  true {BYTES[k] / 1e6:9.1f} MB  ratio {mean / BYTES[k]:.3f}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
