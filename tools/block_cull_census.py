"""Band group-cull census (CPU, oracle data): how many groups of Gaussians
(device = 3D Morton order; 64 = a projection wave's, gs_kernels.hip
group_culled) the per-group bound keeps for each row band, and a soundness
check of that bound against the oracle's rectangles (no Gaussian of a culled
group may have a tile row in the band).  The bound is restated in float64 as
group_culled has it.

  python tools/block_cull_census.py [--n 1000000] [--group 64] [--bands ...]
"""
import argparse
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussian_splat_ipu_amd import camera, scene  # noqa: E402
from oracle import oracle  # noqa: E402


def morton_perm(mean):
    lo = np.nanmin(np.where(np.isfinite(mean), mean, np.nan), axis=0)
    hi = np.nanmax(np.where(np.isfinite(mean), mean, np.nan), axis=0)
    t = np.where(np.isfinite(mean), (mean.astype(np.float64) - lo) / np.maximum(hi - lo, 1e-300), 0.0)
    q = np.clip(t * 2097151.0, 0, 2097151).astype(np.uint64)
    key = np.zeros(mean.shape[0], np.uint64)
    for bit in range(21):
        for a in range(3):
            key |= ((q[:, a] >> np.uint64(bit)) & np.uint64(1)) << np.uint64(3 * bit + a)
    return np.lexsort((np.arange(mean.shape[0]), key))


def spectral_norm2_bound(m):
    """gs_renderer.hip spectral_norm2_bound: >= ||W||_2^2, W the mvp's upper 3x3."""
    W = np.array([[m[i * 4 + k] for k in range(3)] for i in range(3)], np.float64)
    A = W @ W.T
    tr = np.trace(A)
    L = math.log(tr)
    A = A / tr
    for _ in range(6):
        B = A @ A
        t = np.trace(B)
        L = 2 * L + math.log(t)
        A = B / t
    return float(np.nextafter(np.float32(math.exp(L / 64) * (1 + 1e-9)), np.float32(np.inf)))


def block_culled(m, lo, hi, fp):
    """gs_kernels.hip group_culled, restated in float64 (the kernel's float
tail with its margins).  m: the mvp as 16 floats, glm
    column-major (m[c * 4 + r])."""
    if not (hi[3] < math.inf) or not (fp["scale_div"] > 0):
        return False
    vmin, vmax, tzmin, rx, ry = 1e300, -1e300, 1e300, 0.0, 0.0
    pos = neg = True
    for c in range(8):
        x = hi[0] if c & 1 else lo[0]
        y = hi[1] if c & 2 else lo[1]
        z = hi[2] if c & 4 else lo[2]
        tx = (m[0] * x + m[4] * y) + (m[8] * z + m[12])
        cy = (m[1] * x + m[5] * y) + (m[9] * z + m[13])
        cw = (m[3] * x + m[7] * y) + (m[11] * z + m[15])
        tz = (m[2] * x + m[6] * y) + (m[10] * z + m[14])
        wmag = abs(m[3] * x) + abs(m[7] * y) + abs(m[11] * z) + abs(m[15])
        if not (cw > 1e-9 * wmag) or not (cw > 0):
            return False
        v = (cy / cw * 0.5 + 0.5) * fp["H"]
        vmin, vmax = min(vmin, v), max(vmax, v)
        pos = pos and tz > 0
        neg = neg and tz < 0
        tzmin = min(tzmin, abs(tz))
        if tz != 0:
            rx, ry = max(rx, abs(tx) / abs(tz)), max(ry, abs(cy) / abs(tz))
    if not (pos or neg) or not tzmin > 0:
        return False
    lim = 1.3 * fp["tanfov"]
    fx, fy = fp["focal_x"], fp["focal_y"]
    cx, cyy = min(lim, rx * 1.001), min(lim, ry * 1.001)
    j2 = (fx * fx * (1 + cx * cx) + fy * fy * (1 + cyy * cyy)) / (tzmin * tzmin)
    lc = math.exp(2.0 * (hi[3] / fp["scale_div"])) * 1.02
    r = 3.0 * math.sqrt(1.05 * (lc * fp["wnorm2"] * j2) + 1.0) + 2.0
    av = max(abs(vmin), abs(vmax))
    r = r * fp.get("rscale", 1.0)
    r = r * 1.02 + 2.0 + 1e-4 * av + 1.0
    if not (r < 1e6 and av < 1e6):
        return False
    th = fp["th"]
    fy0 = math.floor(math.floor(vmin - r) / th)
    fy1 = math.floor(math.ceil(vmax + r) / th)
    gy1 = fp["tiles_y"] - 1
    if fy1 < 0 or fy0 > gy1:
        return True
    fy0, fy1 = max(fy0, 0), min(fy1, gy1)
    return not (fy0 <= fy1 and fy0 <= fp["band_ty1"] - 1 and fy1 >= fp["band_ty0"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--group", type=int, default=64, help="Gaussians per bound (256: a projection block, 64: a wave)")
    ap.add_argument("--rscale", type=float, default=1.0, help="(estimates only, unsound below 1) radius bound scale")
    ap.add_argument("--bands", default="0,18,23,29,34,39,44,50,68",
                    help="band boundaries in tile rows (default: round 5's balanced 8-band split)")
    a = ap.parse_args()
    W, H, TW = 1920, 1080, 16
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=a.n, seed=1, sh_degree=0)))
    view, proj = camera.headless(bb, W, H)
    fr = oracle.make_frame(view, proj, W, H, TW, TW, camera.FOV_DEFAULT, 1.0)
    p = oracle.project(g, fr, 8)
    G = oracle._g(g)
    perm = morton_perm(G[:, 0:3])
    # the renderer's FrameParams (gs_renderer.hip make_params), in float64
    vw = np.asarray(view, np.float32).reshape(4, 4).T.astype(np.float32)  # glm column-major as [c][r]
    pj = np.asarray(proj, np.float32).reshape(4, 4).T.astype(np.float32)
    # mvp[c][r] = sum_k proj[k][r] * view[c][k] (glm: proj * view), float32 like the host
    mvp = np.zeros((4, 4), np.float32)
    for c in range(4):
        for r_ in range(4):
            s = np.float32(0)
            for k in range(4):
                s = np.float32(s + np.float32(pj[k][r_] * vw[c][k]))
            mvp[c][r_] = s
    m = [float(x) for x in mvp.reshape(16)]
    w2 = spectral_norm2_bound(m)
    tf = math.tan(camera.FOV_DEFAULT / 2)
    fp = dict(H=float(H), th=float(TW), tiles_y=-(-H // TW), scale_div=1.0, tanfov=math.tan(0.5 * camera.FOV_DEFAULT),
              focal_x=W / (2 * tf), focal_y=H / (2 * tf), wnorm2=w2, rscale=a.rscale)
    cr_w = np.where(G[:, 15] <= 0, np.nan, np.where(G[:, 3] != 1.0, np.inf, G[:, 12:15].max(axis=1)))
    G_ = a.group
    nb = (a.n + G_ - 1) // G_
    lo = np.zeros((nb, 3))
    hi = np.zeros((nb, 4))
    for k in range(nb):
        idx = perm[k * G_:(k + 1) * G_]
        mm = G[idx, 0:3]
        sw = cr_w[idx]
        lo[k] = mm.min(axis=0)
        hi[k, :3] = mm.max(axis=0)
        hi[k, 3] = sw.max() if np.all(np.isfinite(sw)) and np.all(np.isfinite(mm)) else math.inf
    b = [int(x) for x in a.bands.split(",")]
    rows0, rows1 = p["rect"][:, 1], p["rect"][:, 3]
    live = (p["rendered"] != 0) & (p["rect"][:, 0] <= p["rect"][:, 2])
    out = []
    for i in range(len(b) - 1):
        fp["band_ty0"], fp["band_ty1"] = b[i], b[i + 1]
        kept = 0
        bad = 0
        for k in range(nb):
            if block_culled(m, lo[k], hi[k], fp):
                idx = perm[k * G_:(k + 1) * G_]
                hit = live[idx] & (rows0[idx] <= b[i + 1] - 1) & (rows1[idx] >= b[i])
                bad += int(hit.sum())
            else:
                kept += 1
        out.append(dict(band=[b[i], b[i + 1]], group=G_, blocks_kept=kept, frac_kept=round(kept / nb, 3), unsound=bad))
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
