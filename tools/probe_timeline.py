"""Kernel timeline of a probe build (bash tools/build_x.sh probe "-DGS_PROBE=1"): per frame and
kernel, the first wave's start and the last wave's end on the GPU's 100 MHz
wall clock -- without a profiler in the process, so frames in flight overlap
as they do in the bench.

    GSPLAT_LIB=tmp_ab/probe/libgsplat.so GSPLAT_PROBE_FILE=/tmp/p.bin \\
        python tools/band_emulate.py --balanced --bands 8 --only-band 3 --inflight 3
    python tools/probe_timeline.py /tmp/p.bin [--json out.json]

Reports, over the middle of the run (warm-up and the emulator's profiled
frames left out): the frame period, each kernel's median duration and the
median gap from the previous kernel of its frame (launch latency), the frame
latency, the fraction of time any kernel runs and the mean number running,
and for each kernel how often the same kernel of the next frame starts before
it has ended (frames overlapping, or queued behind each other).
"""
import argparse
import json
import statistics as stats
import struct

import numpy as np

NAMES = ["project", "agg_scan", "agg_emit", "count", "colscan", "scan_multi", "emit_chunk", "sort_tiles",
         "blend", "blend_cont", "scan", "emit", "big"]
TICK_US = 0.01  # 100 MHz


def read(path):
    out = []
    with open(path, "rb") as f:
        while True:
            h = f.read(16)
            if len(h) < 16:
                break
            magic, dev, nf, K = struct.unpack("<4i", h)
            if magic != 0x52505347:
                raise SystemExit(f"{path}: bad record header")
            a = np.frombuffer(f.read(nf * K * 16), dtype=np.uint64).reshape(nf, K, 2)
            out.append((dev, a))
    return out


def frames_of(recs):
    fr = []  # (renderer, frame, {kernel: (t0, t1)})
    for ri, (_, a) in enumerate(recs):
        for fi in range(a.shape[0]):
            ks = {}
            for k in range(a.shape[1]):
                s, e = int(a[fi, k, 0]), int(a[fi, k, 1])
                if s != 0xFFFFFFFFFFFFFFFF and e >= s:
                    ks[k] = (s, e)
            if ks:
                fr.append((ri, fi, ks))
    fr.sort(key=lambda x: min(v[0] for v in x[2].values()))
    return fr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--json")
    ap.add_argument("--keep", type=float, default=0.6, help="middle fraction of the frames analysed")
    a = ap.parse_args()
    fr = frames_of(read(a.path))
    n = len(fr)
    lo = int(n * (1 - a.keep) / 2)
    win = fr[lo:lo + max(1, int(n * a.keep))]
    starts = [min(v[0] for v in ks.values()) for _, _, ks in win]
    ends = [max(v[1] for v in ks.values()) for _, _, ks in win]
    # (frames of F streams start in bursts: the mean spacing, not the median)
    period = (starts[-1] - starts[0]) / (len(starts) - 1) * TICK_US if len(starts) > 1 else None
    latency = stats.median([e - s for s, e in zip(starts, ends)]) * TICK_US
    dur, gap = {}, {}
    for _, _, ks in win:
        order = sorted(ks.items(), key=lambda kv: kv[1][0])
        prev_end = None
        for k, (s, e) in order:
            dur.setdefault(k, []).append((e - s) * TICK_US)
            if prev_end is not None:
                gap.setdefault(k, []).append((s - prev_end) * TICK_US)
            prev_end = max(prev_end or 0, e)
    # time any kernel runs, mean kernels running (over the window)
    ev = []
    for _, _, ks in win:
        for s, e in ks.values():
            ev.append((s, 1))
            ev.append((e, -1))
    ev.sort()
    t0w, t1w = starts[0], ends[-1]
    busy = area = 0
    cur, last = 0, ev[0][0]
    for t, d in ev:
        if cur > 0:
            busy += t - last
        area += cur * (t - last)
        cur += d
        last = t
    span = max(1, t1w - t0w)
    # the same kernel of consecutive frames: overlapping, or the next one
    # starting only after this one ended
    same = {}
    for (_, _, a_), (_, _, b_) in zip(win, win[1:]):
        for k in set(a_) & set(b_):
            same.setdefault(k, []).append(b_[k][0] < a_[k][1])
    rep = {
        "frames": len(win),
        "period_us": round(period, 2) if period else None,
        "frame_latency_us": round(latency, 2),
        "busy_frac": round(busy / span, 3),
        "mean_kernels_running": round(area / span, 2),
        "kernels": {
            NAMES[k] if k < len(NAMES) else str(k): {
                "median_us": round(stats.median(v), 2),
                "median_gap_before_us": round(stats.median(gap[k]), 2) if gap.get(k) else None,
                "overlaps_next_frames_same_kernel": round(sum(same.get(k, [])) / max(1, len(same.get(k, []))), 3),
            }
            for k, v in sorted(dur.items())
        },
    }
    print(f"{rep['frames']} frames: period {rep['period_us']} us, frame latency {rep['frame_latency_us']} us, "
          f"busy {rep['busy_frac']}, mean kernels running {rep['mean_kernels_running']}")
    print(f"{'kernel':12s} {'median us':>10s} {'gap before':>11s} {'overlaps next':>14s}")
    for k, v in rep["kernels"].items():
        print(f"{k:12s} {v['median_us']:10.2f} {str(v['median_gap_before_us']):>11s} "
              f"{v['overlaps_next_frames_same_kernel']:14.3f}")
    if a.json:
        json.dump(rep, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
