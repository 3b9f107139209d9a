"""Blend work census on the bench scene (CPU, oracle data): how many
(wave, record) evaluations the blend performs for a given pixel-group shape,
and how many of the lane evaluations are useful hits.

  python tools/blend_stats.py [--n 1000000] [--tiles 600] [--group 8x8]

A sample of tiles is simulated exactly (fp32 numpy, expf via the exact
formula is unnecessary for counting: hits use power/pcut/alpha)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussian_splat_ipu_amd import camera, scene  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--tiles", type=int, default=600)
    ap.add_argument("--groups", default="8x8x8x8,8x8x4x4,8x8x2x2,8x8x1x1,8x8x2x1,16x4x2x2")
    a = ap.parse_args()
    W, H, TW = 1920, 1080, 16
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=a.n, seed=1, sh_degree=3)))
    view, proj = camera.headless(bb, W, H)
    fr = oracle.make_frame(view, proj, W, H, TW, TW, camera.FOV_DEFAULT, 1.0)
    p = oracle.project(g, fr, 8)
    ts, lst = oracle.bin_lists(p, fr, 8)
    T = ts.size - 1
    tx_n = -(-W // TW)
    gg = oracle._g(g)
    op = gg[:, 7]
    rng = np.random.default_rng(0)
    lens = np.diff(ts)
    # sample tiles weighted toward the work: half uniform, half by list length
    pick = np.unique(np.concatenate([rng.choice(T, a.tiles // 2, replace=False),
                                     rng.choice(T, a.tiles // 2, p=lens / lens.sum())]))
    w_uniform = T / pick.size  # crude scale for totals
    # wave group WxH split into independent record queues of sub-groups wxh
    groups = [tuple(int(v) for v in s.split("x")) for s in a.groups.split(",")]
    tot = {gs: [0, 0, 0] for gs in groups}  # wave-record evals, lane evals, hits
    hits_all = 0
    tot_c, tot_cm = {}, {}
    for t in pick:
        ids = lst[ts[t]:ts[t + 1]]
        if ids.size == 0:
            continue
        tx, ty = t % tx_n, t // tx_n
        ys, xs = np.mgrid[ty * TW:(ty + 1) * TW, tx * TW:(tx + 1) * TW]
        px = xs.reshape(-1).astype(np.float32)
        py = ys.reshape(-1).astype(np.float32)
        m = p["mean2d"][ids]
        c = p["conic"][ids]
        o = op[ids]
        dx = m[:, 0:1] - px[None]
        dy = m[:, 1:2] - py[None]
        power = np.float32(-0.5) * (c[:, 0:1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy
        alpha = np.minimum(np.float32(0.99), o[:, None] * np.exp(power))
        ok = (power <= 0) & (alpha >= 1 / 255.0) & (o[:, None] != 0)
        okc = (power <= 0) & (power >= np.log(1.0 / (255.0 * np.maximum(o, 1e-30)))[:, None] - 0.05)
        # front-to-back with saturation
        Tt = np.ones(px.size, np.float32)
        done = np.zeros(px.size, bool)
        hit = np.zeros_like(ok)
        done_at = np.full(px.size, ids.size, np.int64)
        for r in range(ids.size):
            h = ok[r] & ~done
            tT = Tt * (1 - alpha[r])
            brk = h & (tT < 1e-4)
            upd = h & ~brk
            Tt = np.where(upd, tT, Tt)
            done_at[brk] = r
            done |= brk
            hit[r] = h
        hits_all += int(hit.sum())
        # footprint boxes (ellipse {power >= pcut} bbox, +1 px), as the kernel's
        a_, b_, c_ = c[:, 0].astype(np.float64), c[:, 1].astype(np.float64), c[:, 2].astype(np.float64)
        pc = np.log(1.0 / (255.0 * np.maximum(o, 1e-30))).astype(np.float64)
        det = a_ * c_ - b_ * b_
        hx = np.sqrt(np.maximum(-2 * (pc - 0.05) * c_ / det, 0)) * 1.001
        hy = np.sqrt(np.maximum(-2 * (pc - 0.05) * a_ / det, 0)) * 1.001
        bx0 = np.ceil(m[:, 0] - hx); bx1 = np.floor(m[:, 0] + hx)
        by0 = np.ceil(m[:, 1] - hy); by1 = np.floor(m[:, 1] + hy)
        lx = xs.reshape(-1) - tx * TW
        ly = ys.reshape(-1) - ty * TW
        for gs in groups:
            gw, gh, sw, sh = gs
            for oy in range(0, TW, gh):
                for ox in range(0, TW, gw):
                    mx_it = 0
                    mx_c = 0
                    for sy in range(oy, oy + gh, sh):
                        for sx in range(ox, ox + gw, sw):
                            sel = (lx >= sx) & (lx < sx + sw) & (ly >= sy) & (ly < sy + sh)
                            X0, X1 = tx * TW + sx, tx * TW + sx + sw - 1
                            Y0, Y1 = ty * TW + sy, ty * TW + sy + sh - 1
                            inbox = ~((bx0 > X1) | (bx1 < X0) | (by0 > Y1) | (by1 < Y0))
                            stop = done_at[sel].max()
                            lim = min(stop + 1, ids.size)
                            ev = int(inbox[:lim].sum())
                            cand = int(okc[:lim][:, sel].any(axis=1).sum())
                            tot_c[gs] = tot_c.get(gs, 0) + cand
                            mx_c = max(mx_c, cand)
                            mx_it = max(mx_it, ev)
                            tot[gs][2] += int(hit[:, sel].sum())
                            tot[gs][1] += ev * int(sel.sum())
                    tot[gs][0] += mx_it
                    tot_cm[gs] = tot_cm.get(gs, 0) + mx_c
    print(f"tiles sampled {pick.size} of {T}; P={lst.size}")
    for gs in groups:
        ev, le, h = tot[gs]
        print(f"wave {gs[0]}x{gs[1]} sub {gs[2]}x{gs[3]}: wave iterations {ev} (exact-ellipse {tot_cm[gs]}), sub-lane evals {le}, hits {h}, useful {h / max(le, 1):.3f}")


if __name__ == "__main__":
    main()
