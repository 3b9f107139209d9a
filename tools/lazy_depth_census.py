"""How deep into a big list (> 2048 keys) the blend goes (CPU census, oracle
data, config 5 = 8M clustered Gaussians at 4K, orbit view k).

For a sample of big tiles: the list in blend order, and per pixel the record at
which it saturates (the reference's `break`), or the list's end.  Prints per
tile the deepest record any pixel needs (D) and how many keys past the lazy
prefix (1536) the continuation must provide, unfiltered and filtered by the
live pixels' box -- the numbers a second lazy prefix would be sized on.

  python tools/lazy_depth_census.py [--view 0] [--tiles 80]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussian_splat_ipu_amd import camera, scene  # noqa: E402
from oracle import oracle  # noqa: E402
from blend_census import boxes  # noqa: E402

PREFIX = 1536


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--view", type=int, default=0)
    ap.add_argument("--tiles", type=int, default=80)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    W, H, TW = 3840, 2160, 16
    src = scene.load_ply(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "point_cloud_12.ply"))
    cl = np.stack([src["x"], src["y"], src["z"]], 1)
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=8_000_000, seed=8, sh_degree=0,
                                                                cluster_xyz=cl, cluster_sigma=0.02)))
    _, proj = camera.headless(bb, W, H)
    view = camera.orbit_view(a.view)
    fr = oracle.make_frame(view, proj, W, H, TW, TW, camera.FOV_DEFAULT, 1.0)
    p = oracle.project(g, fr, 8)
    ts, lst = oracle.bin_lists(p, fr, 8)
    tx_n = -(-W // TW)
    op = oracle._g(g)[:, 7]
    _, bx0, bx1, by0, by1 = boxes(p["mean2d"], p["conic"], op)
    lens = np.diff(ts)
    big = np.nonzero(lens > 2048)[0]
    rng = np.random.default_rng(a.seed)
    pick = rng.choice(big, min(a.tiles, big.size), replace=False)
    print(f"big lists {big.size}, sampled {pick.size}")
    rows = []
    for t in pick:
        ids = lst[ts[t]:ts[t + 1]]  # blend order (depth, input index)
        tx, ty = t % tx_n, t // tx_n
        X0, Y0 = tx * TW, ty * TW
        keep = ~((bx0[ids] > X0 + TW - 1) | (bx1[ids] < X0) | (by0[ids] > Y0 + TW - 1) | (by1[ids] < Y0))
        idk = ids[keep]  # the binned list (pair cull), still in order
        L = idk.size
        ys, xs = np.mgrid[Y0:Y0 + TW, X0:X0 + TW]
        px = xs.reshape(-1).astype(np.float32)
        py = ys.reshape(-1).astype(np.float32)
        Tt = np.ones(px.size, np.float32)
        sat = np.full(px.size, L, np.int64)
        m = p["mean2d"][idk].astype(np.float32)
        c = p["conic"][idk].astype(np.float32)
        o = op[idk].astype(np.float32)
        for r0 in range(0, L, 4096):
            r1 = min(L, r0 + 4096)
            dx = m[r0:r1, 0:1] - px[None]
            dy = m[r0:r1, 1:2] - py[None]
            power = np.float32(-0.5) * (c[r0:r1, 0:1] * dx * dx + c[r0:r1, 2:3] * dy * dy) - c[r0:r1, 1:2] * dx * dy
            alpha = np.minimum(np.float32(0.99), o[r0:r1, None] * np.exp(power))
            hit = (power <= 0) & (alpha >= np.float32(1 / 255.0)) & (o[r0:r1, None] != 0)
            for r in range(r1 - r0):
                h = hit[r] & (sat == L)
                if not h.any():
                    continue
                tT = Tt * (np.float32(1) - alpha[r])
                brk = h & (tT < np.float32(1e-4))
                Tt = np.where(h & ~brk, tT, Tt)
                sat = np.where(brk, r0 + r, sat)
            if (sat < L).all():
                break
        D = int(sat.max())  # deepest record needed (L: some pixel never saturates)
        live = sat >= PREFIX
        if live.any():
            lx0, lx1 = px[live].min(), px[live].max()
            ly0, ly1 = py[live].min(), py[live].max()
            rest = idk[PREFIX:min(L, D + 1)]
            fl = ~((bx0[rest] > lx1) | (bx1[rest] < lx0) | (by0[rest] > ly1) | (by1[rest] < ly0))
            nf = int(fl.sum())
            allrest = idk[PREFIX:]
            fa = ~((bx0[allrest] > lx1) | (bx1[allrest] < lx0) | (by0[allrest] > ly1) | (by1[allrest] < ly0))
            nfa = int(fa.sum())
        else:
            nf = nfa = 0
        never = int((sat == L).sum())
        rows.append((t, L, D, never, nf, nfa, int(live.sum())))
        print(f"tile {t}: L {L} deepest {D} never-saturate px {never} live after prefix {int(live.sum())} "
              f"keys needed past prefix: {max(0, D + 1 - PREFIX)} (box-filtered {nf} of {nfa})", flush=True)
    r = np.array(rows)
    cont = r[r[:, 2] >= PREFIX]
    print(f"continued lists {len(cont)} of {len(r)}")
    if len(cont):
        need = cont[:, 2] + 1 - PREFIX
        for q in (2048, 4096, 8192, 16384):
            print(f"  needing <= {q} keys past the prefix: {(need <= q).sum()} ; box-filtered <= {q}: "
                  f"{(cont[:, 4] <= q).sum()}")
        print(f"  with a never-saturating pixel: {(cont[:, 3] > 0).sum()}")


if __name__ == "__main__":
    main()
