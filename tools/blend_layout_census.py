"""Blend layout census (CPU, oracle data): how much walking, staging and
masked-off work each lane layout of the 16x16-tile blend costs on the bench
scene, to choose the layout before building it.

Layouts (a wave walks its tile's depth-sorted list in batches of 64; a lane
walks, in list order, the batch's records whose integer alpha box meets any
of its pixels, until all of its pixels have saturated; the wave stages the
next batch until every lane is done):
  px1  4 waves per tile, an 8x8 block each, one pixel per lane
  px2  2 waves per tile, a 16x8 half each, a horizontal pixel pair per lane
  px4  1 wave per tile, a 2x2 pixel quad per lane
  px4h 1 wave per tile, a 4x1 pixel run per lane
Per layout, summed over the sampled tiles and scaled to the frame:
  iters    wave record-steps (per batch: the most records any lane walked)
  staged   records staged (each wave its own copy)
  evals    pixel-record evaluations the lanes run (every pixel of a walking
           lane, live or not) and the useful ones (the pixel's box holds the
           record and the pixel is still live)
  tail     the heaviest tile's longest wave, in record-steps
  python tools/blend_layout_census.py [--tiles 400]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussian_splat_ipu_amd import camera, scene  # noqa: E402
from oracle import oracle  # noqa: E402
from blend_census import boxes  # noqa: E402

TW = 16
# lane -> list of tile-local pixel indices (y * 16 + x), per wave
LAYOUTS = {}


def _layout_px1():
    waves = []
    for by in (0, 8):
        for bx in (0, 8):
            waves.append([[(by + l // 8) * TW + bx + l % 8] for l in range(64)])
    return waves


def _layout_px2():
    return [[[(8 * h + l // 8) * TW + 2 * (l % 8), (8 * h + l // 8) * TW + 2 * (l % 8) + 1] for l in range(64)]
            for h in (0, 1)]


def _layout_px4():
    out = []
    for l in range(64):
        x, y = 2 * (l % 8), 2 * (l // 8)
        out.append([y * TW + x, y * TW + x + 1, (y + 1) * TW + x, (y + 1) * TW + x + 1])
    return [out]


def _layout_px4h():
    return [[[(l // 4) * TW + 4 * (l % 4) + k for k in range(4)] for l in range(64)]]


LAYOUTS = {"px1": _layout_px1(), "px2": _layout_px2(), "px4": _layout_px4(), "px4h": _layout_px4h()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--tiles", type=int, default=400)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch", type=int, default=64, help="records staged per batch (a lane walks its whole batch mask)")
    ap.add_argument("--layouts", default="px1,px2,px4,px4h")
    ap.add_argument("--mask", choices=["box", "ellipse", "rows"], default="box",
                    help="a lane's records: the integer alpha box meets a pixel (the kernels), or the pixel "
                         "lies in the record's pcut ellipse (an ideal per-pixel mask), or 'rows': the "
                         "ellipse's x-extent over groups of --row-group pixel rows")
    ap.add_argument("--row-group", type=int, default=4)
    ap.add_argument("--window", type=lambda t: [int(x) for x in t.split(",")], default=[],
                    help="also cost windows of K staged batches (comma list), lanes running ahead within it")
    ap.add_argument("--no-lane-exit", action="store_true",
                    help="lanes stop only at batch boundaries (no per-record saturation exit)")
    a = ap.parse_args()
    B = a.batch
    lay = {k: LAYOUTS[k] for k in a.layouts.split(",")}
    W, H = 1920, 1080
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
                                     rng.choice(T, a.tiles // 2, p=lens / lens.sum()),
                                     [int(np.argmax(lens))]]))
    acc = {k: dict(iters=0, staged=0, evals=0, useful=0, batches=0, tail=0) for k in lay}
    for t in pick:
        ids = lst[ts[t]:ts[t + 1]]
        tx, ty = t % tx_n, t // tx_n
        X0, Y0 = tx * TW, ty * TW
        keep = ~((bx0[ids] > X0 + TW - 1) | (bx1[ids] < X0) | (by0[ids] > Y0 + TW - 1) | (by1[ids] < Y0))
        ids = ids[keep]
        L = ids.size
        if L == 0:
            continue
        ys, xs = np.mgrid[Y0:Y0 + TW, X0:X0 + TW]
        px = xs.reshape(-1).astype(np.float64)
        py = ys.reshape(-1).astype(np.float64)
        valid = (px < W) & (py < H)
        inb = ((bx0[ids][:, None] <= px[None]) & (bx1[ids][:, None] >= px[None]) &
               (by0[ids][:, None] <= py[None]) & (by1[ids][:, None] >= py[None]) & valid[None])  # [L, 256]
        m = p["mean2d"][ids].astype(np.float64)
        c = p["conic"][ids].astype(np.float64)
        o = op[ids].astype(np.float64)
        dx = m[:, 0:1] - px[None]
        dy = m[:, 1:2] - py[None]
        power = -0.5 * (c[:, 0:1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy
        alpha = np.minimum(0.99, o[:, None] * np.exp(power))
        hit = inb & (power <= 0) & (alpha >= 1 / 255.0) & (o[:, None] != 0)
        # the record at which each pixel breaks (T' < 1e-4), L if never
        om = np.where(hit, 1.0 - alpha, 1.0)
        Tc = np.cumprod(om, axis=0)
        brk = hit & (Tc < 1e-4)
        done_at = np.where(brk.any(axis=0), np.argmax(brk, axis=0), L)  # last record walked
        done_at = np.where(valid, done_at, -1)
        rec = np.arange(L)[:, None]
        live = inb & (rec <= done_at[None])  # useful evaluations: box holds it, pixel live
        msk = inb & (power >= pcut_all[ids][:, None]) if a.mask == "ellipse" else inb
        if a.mask == "rows":
            ell = (inb & (power >= pcut_all[ids][:, None])).reshape(L, TW, TW)  # [L, y, x]
            G = a.row_group
            eg = ell.reshape(L, TW // G, G, TW).any(axis=2)  # [L, groups, x]: x in the extent of some row
            xs_ = np.arange(TW)
            lo = np.where(eg.any(axis=2), np.argmax(eg, axis=2), TW)
            hi = np.where(eg.any(axis=2), TW - 1 - np.argmax(eg[:, :, ::-1], axis=2), -1)
            inx = (xs_[None, None, :] >= lo[:, :, None]) & (xs_[None, None, :] <= hi[:, :, None])  # [L, groups, x]
            msk = inb & np.repeat(inx, G, axis=1).reshape(L, TW * TW)
        for name, waves in lay.items():
            A = acc[name]
            for lanes in waves:
                P = np.array(lanes)  # [64, k]
                k = P.shape[1]
                lane_end = done_at[P].max(axis=1)  # the lane walks until its last pixel breaks
                union = msk[:, P].any(axis=2)  # [L, 64]
                if a.no_lane_exit:
                    # live at the batch start: the lane walks its whole batch mask
                    bstart = (rec // B) * B
                    walk = union & (bstart <= lane_end[None])
                else:
                    walk = union & (rec <= lane_end[None])
                # (no batch barrier: every lane walks the whole list at its own
                # pace -- the wave's steps are its slowest lane's total)
                A.setdefault("free", 0)
                A["free"] += int(walk.sum(axis=0).max()) if L else 0
                # a window of K staged batches: each step, every lane with a record
                # left in the window takes one; when no lane has one left in the
                # window's first batch, the window slides (the next batch staged)
                relw = np.nonzero(union.any(axis=1))[0]
                for K, wk, key in [(K, walk, f"win{K}") for K in a.window] + \
                                  [(K, walk[relw], f"cwin{K}") for K in a.window]:
                    A.setdefault(key, 0)
                    nb = -(-wk.shape[0] // B)
                    cnt = np.zeros((nb, wk.shape[1]), np.int64)
                    for bb in range(nb):
                        cnt[bb] = wk[bb * B:(bb + 1) * B].sum(axis=0)
                    rem = cnt.copy()
                    steps = 0
                    w = 0
                    while w < nb:
                        if not rem[w].any():
                            w += 1
                            continue
                        # one step: each lane takes its earliest remaining record in [w, w+K)
                        hi = min(nb, w + K)
                        sub = rem[w:hi]
                        has = sub.any(axis=0)
                        first = np.argmax(sub > 0, axis=0)
                        lanes = np.nonzero(has)[0]
                        rem[w + first[lanes], lanes] -= 1
                        steps += 1
                    A[key] += steps
                wave_iters = 0
                for base in range(0, L, B):
                    if base > lane_end.max():
                        break
                    A["batches"] += 1
                    A["staged"] += min(B, L - base)
                    w = walk[base:base + B]
                    it = int(w.sum(axis=0).max())
                    wave_iters += it
                    A["evals"] += int(w.sum()) * k
                A["iters"] += wave_iters
                A["tail"] = max(A["tail"], wave_iters)
                # compacted staging (round 6): the wave stages only the records
                # whose box meets one of its pixels, in list order, 64 a batch
                rel = np.nonzero(union.any(axis=1))[0]
                wc = walk[rel]
                endc = np.searchsorted(rel, lane_end.max(), side="right")  # records up to the wave's end
                for k_, key in (("cmp_iters", "cmp_iters"), ("cmp_batches", "cmp_batches"), ("cmp_staged", "cmp_staged")):
                    A.setdefault(key, 0)
                for base in range(0, int(endc), B):
                    w = wc[base:base + B]
                    A["cmp_batches"] += 1
                    A["cmp_staged"] += w.shape[0]
                    A["cmp_iters"] += int(w.sum(axis=0).max())
                A["useful"] += int(live[:, P.reshape(-1)].sum())
    scale = T / pick.size
    print(f"tiles sampled {pick.size} of {T}, longest list {lens.max()} (sampled)")
    print(f"{'layout':6s} {'waves':>6s} {'iters':>10s} {'staged':>10s} {'batches':>9s} {'evals':>11s} "
          f"{'useful':>11s} {'use/eval':>8s} {'tail iters':>10s}")
    print(f"batch {B}")
    for name, A in acc.items():
        print(f"{name}: wave steps with a barrier per batch {A['iters'] * scale:.0f}, "
              f"without (lanes at their own pace) {A.get('free', 0) * scale:.0f}, " +
              ", ".join(f"window {K}: {A.get(f'win{K}', 0) * scale:.0f}" for K in a.window) +
              "; compacted, " + ", ".join(f"window {K}: {A.get(f'cwin{K}', 0) * scale:.0f}" for K in a.window))
        print(f"{name}: compacted staging (the wave's own records only): wave steps {A.get('cmp_iters', 0) * scale:.0f}, "
              f"batches {A.get('cmp_batches', 0) * scale:.0f}, staged {A.get('cmp_staged', 0) * scale:.0f}")
    for name, A in acc.items():
        nw = len(lay[name]) * T
        print(f"{name:6s} {nw:6d} {A['iters'] * scale:10.0f} {A['staged'] * scale:10.0f} {A['batches'] * scale:9.0f} "
              f"{A['evals'] * scale:11.0f} {A['useful'] * scale:11.0f} {A['useful'] / max(A['evals'], 1):8.3f} "
              f"{A['tail']:10d}")


if __name__ == "__main__":
    main()
