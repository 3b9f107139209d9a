"""Blend work census of the current kernel's structure (CPU, oracle data).

For a sample of 16x16 tiles of the bench scene: each 8x8 blend wave walks the
tile's binned list in batches of 64; a lane's batch mask holds the records
whose integer alpha box contains its pixel; it walks them two per iteration
until its pixel saturates.  Counts, per wave and summed:
  iters      wave iterations (max over live lanes of ceil(bits / 2))
  batches    batches staged (the mask build runs once per batch)
  evals      lane-record evaluations that do work (bits walked)
  util       evals / (2 * 64 * iters)
and the split of idle lane-iterations into "mask exhausted while others
continue" and "pixel saturated".  Alternative structures are costed on the
same data (see --help).

  python tools/blend_census.py [--n 1000000] [--tiles 300]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussian_splat_ipu_amd import camera, scene  # noqa: E402
from oracle import oracle  # noqa: E402


def boxes(m, c, o):
    """pcut and the integer alpha box (x0, x1, y0, y1) as gs_kernels.hip's
    alpha_footprint (float64 here: a census, not parity)."""
    a, b, cc = c[:, 0].astype(np.float64), c[:, 1].astype(np.float64), c[:, 2].astype(np.float64)
    op = o.astype(np.float64)
    ln = np.log(np.maximum(255.0 * op, 1e-30))
    pc = -ln - 0.05
    pcut = pc - (ln * 1e-5 + 1e-5)
    det = a * cc - b * b
    ok = (op >= 1 / 255.0) & (a > 0) & (cc > 0) & (det > 1e-3 * a * cc)
    R = -2.0 * pcut
    with np.errstate(invalid="ignore", divide="ignore"):
        ex = np.sqrt(np.maximum(R * cc / det, 0)) * 1.001
        ey = np.sqrt(np.maximum(R * a / det, 0)) * 1.001
    x0 = np.where(ok, np.ceil(m[:, 0] - ex), -1e9)
    x1 = np.where(ok, np.floor(m[:, 0] + ex), 1e9)
    y0 = np.where(ok, np.ceil(m[:, 1] - ey), -1e9)
    y1 = np.where(ok, np.floor(m[:, 1] + ey), 1e9)
    empty = op < 1 / 255.0
    x0 = np.where(empty, 1e9, x0)
    return pcut, x0, x1, y0, y1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--tiles", type=int, default=300)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    W, H, TW = 1920, 1080, 16
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=a.n, seed=1, sh_degree=0)))
    view, proj = camera.headless(bb, W, H)
    fr = oracle.make_frame(view, proj, W, H, TW, TW, camera.FOV_DEFAULT, 1.0)
    p = oracle.project(g, fr, 8)
    ts, lst = oracle.bin_lists(p, fr, 8)
    T = ts.size - 1
    tx_n = -(-W // TW)
    op = oracle._g(g)[:, 7]
    pcut_all, bx0, bx1, by0, by1 = boxes(p["mean2d"], p["conic"], op)
    rng = np.random.default_rng(a.seed)
    lens = np.diff(ts)
    pick = np.unique(np.concatenate([rng.choice(T, a.tiles // 2, replace=False),
                                     rng.choice(T, a.tiles // 2, p=lens / lens.sum())]))
    acc = dict(iters=0, iters1=0, batches=0, evals=0, idle_mask=0, idle_sat=0, staged=0, binned=0,
               dense=0, ref=0, hits=0, empty_batches=0)
    live_hist = np.zeros(65, np.int64)  # wave iterations by live lanes at batch start
    tail_evals = np.zeros(65, np.int64)
    for t in pick:
        ids = lst[ts[t]:ts[t + 1]]
        tx, ty = t % tx_n, t // tx_n
        X0, Y0 = tx * TW, ty * TW
        acc["ref"] += ids.size
        # pair cull: the binned list keeps the records whose box meets the tile
        keep = ~((bx0[ids] > X0 + TW - 1) | (bx1[ids] < X0) | (by0[ids] > Y0 + TW - 1) | (by1[ids] < Y0))
        ids = ids[keep]
        acc["binned"] += ids.size
        if ids.size == 0:
            continue
        m = p["mean2d"][ids].astype(np.float32)
        c = p["conic"][ids].astype(np.float32)
        o = op[ids].astype(np.float32)
        for wy in (0, 8):
            for wx in (0, 8):
                ys, xs = np.mgrid[Y0 + wy:Y0 + wy + 8, X0 + wx:X0 + wx + 8]
                px = xs.reshape(-1).astype(np.float32)
                py = ys.reshape(-1).astype(np.float32)
                inb = ((bx0[ids][:, None] <= px[None]) & (bx1[ids][:, None] >= px[None]) &
                       (by0[ids][:, None] <= py[None]) & (by1[ids][:, None] >= py[None]))  # [rec, lane]
                dx = m[:, 0:1] - px[None]
                dy = m[:, 1:2] - py[None]
                power = np.float32(-0.5) * (c[:, 0:1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy
                alpha = np.minimum(np.float32(0.99), o[:, None] * np.exp(power))
                hit = (power <= 0) & (alpha >= np.float32(1 / 255.0)) & (o[:, None] != 0)
                Tt = np.ones(64, np.float32)
                done = np.zeros(64, bool)
                for base in range(0, ids.size, 64):
                    if done.all():
                        break
                    acc["batches"] += 1
                    acc["staged"] += min(64, ids.size - base)
                    nlive = int((~done).sum())
                    k = np.zeros(64, np.int64)  # bits walked per lane in this batch
                    for r in range(base, min(base + 64, ids.size)):
                        live = ~done & inb[r]
                        k += live
                        h = live & hit[r]
                        acc["hits"] += int(h.sum())
                        tT = Tt * (np.float32(1) - alpha[r])
                        brk = h & (tT < np.float32(1e-4))
                        Tt = np.where(h & ~brk, tT, Tt)
                        done |= brk
                    if k.max() == 0:
                        acc["empty_batches"] += 1  # no live lane has a record of this batch
                    it = int(np.max((k + 1) // 2))
                    acc["iters"] += it
                    live_hist[nlive] += it
                    tail_evals[nlive] += int(k.sum())
                    acc["iters1"] += int(np.max(k))
                    acc["evals"] += int(k.sum())
                    acc["dense"] += int(-(-k.sum() // 64))
                    # idle lane-iterations: lanes whose bits ran out (split by
                    # whether the pixel is done at batch end)
                    idle = it - (k + 1) // 2
                    acc["idle_sat"] += int(idle[done].sum())
                    acc["idle_mask"] += int(idle[~done].sum())
    scale = T / pick.size
    it, b, e = acc["iters"], acc["batches"], acc["evals"]
    print(f"tiles sampled {pick.size} of {T}; ref pairs {acc['ref']} binned {acc['binned']} staged {acc['staged']}")
    print(f"wave iterations {it}  batches {b}  lane evals {e}  util {e / (2 * 64 * max(it, 1)):.3f}")
    tot_idle = acc["idle_sat"] + acc["idle_mask"]
    print(f"idle lane-iterations: mask exhausted {acc['idle_mask'] / max(tot_idle, 1):.3f}, "
          f"saturated {acc['idle_sat'] / max(tot_idle, 1):.3f}")
    print(f"one record per iteration: {acc['iters1']} iterations; perfectly dense batches: {acc['dense']} "
          f"iterations of 64 lane-records")
    cum = np.cumsum(live_hist)
    cev = np.cumsum(tail_evals)
    for thr in (4, 8, 16, 24, 32, 48):
        print(f"  iterations with <= {thr:2d} live lanes at batch start: {cum[thr] / max(it, 1):.3f} "
              f"(their lane evals: {cev[thr] / max(e, 1):.3f} of all)")
    print(f"batches in which no live lane has a record: {acc['empty_batches']} of {b} ({acc['empty_batches'] / max(b, 1):.3f})")
    print(f"hits (power in range, alpha >= 1/255) among lane evals: {acc['hits'] / max(e, 1):.3f}")
    print(f"whole frame (scaled): iters {it * scale:.0f} batches {b * scale:.0f} evals {e * scale:.0f}")


if __name__ == "__main__":
    main()
