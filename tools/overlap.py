#!/usr/bin/env python3
"""Kernel concurrency of the pipelined bench (frames in flight), from a
rocprofv3 --kernel-trace CSV.

    python tools/overlap.py gpurun_out/ov/<...>_kernel_trace.csv

The window is the middle 60 % of the blend launches (with --steps in the
hundreds that is the timed region).  Reports, per kernel: launches per frame,
average duration while overlapped, and the share of the window during which at
least one instance runs; plus the window's frame period, the union busy
fraction (any gs_ kernel running) and the average number of kernels running.
"""
import csv
import sys
from collections import defaultdict


def short(name):
    for p in ("void ", "gsk::", "(anonymous namespace)::"):
        name = name.replace(p, "")
    return name.split("(")[0].split("<")[0].replace("_kernel", "")


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if not k.startswith("gs_"):
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    blends = [r for r in rows if r[2] == "gs_blend"]
    nb = len(blends)
    lo, hi = blends[nb // 5][0], blends[(4 * nb) // 5][0]
    win = [r for r in rows if lo <= r[0] < hi]
    frames = sum(1 for r in win if r[2] == "gs_blend")
    span = hi - lo
    per = defaultdict(list)
    for s, e, k in win:
        per[k].append(e - s)
    # union of busy intervals, overall and per kernel
    def union(iv):
        tot, cur_s, cur_e = 0, None, None
        for s, e in sorted(iv):
            e = min(e, hi)
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        return tot

    busy = union([(s, e) for s, e, _ in win])
    print(f"window {span / 1e3:.1f} us, {frames} frames, period {span / frames / 1e3:.2f} us/frame")
    print(f"busy (any kernel) {busy / span:.3f}, mean kernels running {sum(e - s for s, e, _ in win) / span:.2f}")
    print(f"{'kernel':22s} {'per frame':>9s} {'avg us':>8s} {'sum us/frame':>12s} {'running frac':>12s}")
    for k, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        u = union([(s, e) for s, e, kk in win if kk == k])
        print(f"{k:22s} {len(d) / frames:9.2f} {sum(d) / len(d) / 1e3:8.2f} {sum(d) / frames / 1e3:12.2f} {u / span:12.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
