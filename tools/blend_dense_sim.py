"""Cost model of a two-phase blend (CPU, oracle data): per batch, rounds of
up to K records per lane; phase A evaluates every (pixel, record) pair of the
round densely across the wave's 64 lanes (power, exp, alpha, the skip tests,
the premultiplied colour), phase B walks each lane's pairs in list order and
does only the state update (T, colour, the break).  Against the current
one-walk blend (every lane evaluates its own records, the wave iterates to its
slowest lane).

VALU per wave-iteration are the estimates of the ISA listing (old walk ~56;
A ~50 per dense pass, B ~14, A0 ~6 per record to compact the lanes' indices,
~20 per round for the prefix scan and bookkeeping).

  python tools/blend_dense_sim.py [--tiles 200] [--k 4,8,16]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussian_splat_ipu_amd import camera, scene  # noqa: E402
from oracle import oracle  # noqa: E402
from blend_census import boxes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--tiles", type=int, default=200)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--k", default="2,4,8,16,64")
    ap.add_argument("--c-old", type=float, default=56.0)
    ap.add_argument("--c-a", type=float, default=50.0)
    ap.add_argument("--c-b", type=float, default=14.0)
    ap.add_argument("--c-a0", type=float, default=6.0)
    ap.add_argument("--c-round", type=float, default=20.0)
    a = ap.parse_args()
    Ks = [int(x) for x in a.k.split(",")]
    W, H, TW = 1920, 1080, 16
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=a.n, seed=1, sh_degree=0)))
    view, proj = camera.headless(bb, W, H)
    fr = oracle.make_frame(view, proj, W, H, TW, TW, camera.FOV_DEFAULT, 1.0)
    p = oracle.project(g, fr, 8)
    ts, lst = oracle.bin_lists(p, fr, 8)
    T = ts.size - 1
    tx_n = -(-W // TW)
    op = oracle._g(g)[:, 7]
    _, bx0, bx1, by0, by1 = boxes(p["mean2d"], p["conic"], op)
    rng = np.random.default_rng(a.seed)
    lens = np.diff(ts)
    pick = np.unique(np.concatenate([rng.choice(T, a.tiles // 2, replace=False),
                                     rng.choice(T, a.tiles // 2, p=lens / lens.sum())]))
    old_iters = 0
    batches = 0
    st = {K: dict(rounds=0, a_iters=0, b_iters=0, pairs=0, useful=0) for K in Ks}
    for t in pick:
        ids = lst[ts[t]:ts[t + 1]]
        tx, ty = t % tx_n, t // tx_n
        X0, Y0 = tx * TW, ty * TW
        keep = ~((bx0[ids] > X0 + TW - 1) | (bx1[ids] < X0) | (by0[ids] > Y0 + TW - 1) | (by1[ids] < Y0))
        ids = ids[keep]
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
                # the record at which each lane saturates (index into ids), or
                # ids.size; the lane's walked records are inb before it
                Tt = np.ones(64, np.float32)
                sat = np.full(64, ids.size, np.int64)
                for r in range(ids.size):
                    h = hit[r] & (sat == ids.size) & inb[r]
                    tT = Tt * (np.float32(1) - alpha[r])
                    brk = h & (tT < np.float32(1e-4))
                    Tt = np.where(h & ~brk, tT, Tt)
                    sat = np.where(brk, r, sat)
                for base in range(0, ids.size, 64):
                    live0 = sat >= base
                    if not live0.any():
                        break
                    batches += 1
                    hi = min(base + 64, ids.size)
                    bits = inb[base:hi] & live0[None]  # [rec, lane] at batch start
                    # old: a lane walks its bits up to and including its saturating record
                    walked = bits & (np.arange(base, hi)[:, None] <= sat[None])
                    old_iters += int(walked.sum(0).max())
                    for K in Ks:
                        s = st[K]
                        # rounds: each lane takes its next <= K bits (if still live)
                        pos = [list(np.nonzero(bits[:, l])[0] + base) for l in range(64)]
                        ptr = np.zeros(64, np.int64)
                        done = ~live0.copy()
                        while True:
                            take = np.zeros(64, np.int64)
                            bmax = 0
                            for l in range(64):
                                if done[l]:
                                    continue
                                rem = len(pos[l]) - ptr[l]
                                if rem <= 0:
                                    continue
                                cl = min(K, rem)
                                take[l] = cl
                                recs = pos[l][ptr[l]:ptr[l] + cl]
                                # B walks until saturation
                                w = sum(1 for r in recs if r <= sat[l])
                                s["useful"] += w
                                bmax = max(bmax, w)
                                if any(r >= sat[l] for r in recs):
                                    done[l] = True
                                ptr[l] += cl
                            S = int(take.sum())
                            if S == 0:
                                break
                            s["rounds"] += 1
                            s["pairs"] += S
                            s["a_iters"] += -(-S // 64)
                            s["b_iters"] += bmax
    scale = T / pick.size
    old = a.c_old * old_iters
    print(f"tiles {pick.size}; batches {batches}; old one-record iterations {old_iters} -> VALU {old:.0f}")
    for K in Ks:
        s = st[K]
        new = (a.c_round * s["rounds"] + a.c_a0 * s["b_iters"] + a.c_a * s["a_iters"] + a.c_b * s["b_iters"])
        print(f"K={K:3d}: rounds {s['rounds']} pairs {s['pairs']} (useful {s['useful']}) dense iters {s['a_iters']} "
              f"B iters {s['b_iters']} -> VALU {new:.0f} ({new / old:.3f} of old)")
    print(f"scale to frame x{scale:.1f}")


if __name__ == "__main__":
    main()
