"""A second, independent restatement of the reference frame path in pure
Python with explicit float32 rounding after every operation (numpy float32
scalars), used to pin the C oracle on small cases.  Written from the reference
sources (citations in oracle/gs_oracle.cpp), not from the oracle's code.

fmaf has no Python-3.10 builtin; `fmaf` below is exact: the product and sum
are formed in rationals and rounded once to float32 (ties to even).
"""
from __future__ import annotations

import ctypes
import math
from fractions import Fraction

import numpy as np

f32 = np.float32
_LIBM = ctypes.CDLL("libm.so.6")
_LIBM.tanf.restype = ctypes.c_float
_LIBM.tanf.argtypes = [ctypes.c_float]


def _round_f32(q: Fraction) -> np.float32:
    if q == 0:
        return f32(0.0)
    sign = -1 if q < 0 else 1
    a = -q if q < 0 else q
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    e = max(e, -126)  # subnormals share the 2^-149 quantum
    scale = Fraction(2) ** (e - 23)
    m = a / scale
    r = round(m)  # Fraction.__round__: ties to even
    v = float(r * scale)
    if v > 3.4028234663852886e38:
        return f32(sign * np.inf)
    return f32(sign * v)


def fmaf(a, b, c) -> np.float32:
    a, b, c = f32(a), f32(b), f32(c)
    if not (np.isfinite(a) and np.isfinite(b) and np.isfinite(c)):
        return f32(a * b + c)
    return _round_f32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def expf(x) -> np.float32:
    """The shared expf specification (Cody-Waite + degree-6 polynomial)."""
    x = f32(x)
    if x != x:
        return x
    xc = f32(min(max(float(x), -104.0), 89.0))
    k = f32(np.rint(f32(xc * f32(1.44269502162933349609))))
    r = fmaf(k, f32(-0.693145751953125), xc)
    r = fmaf(k, f32(-1.428606765330187045e-06), r)
    p = f32(1.9875691500e-4)
    for c in (1.3981999507e-3, 8.3334519073e-3, 4.1665795894e-2, 1.6666665459e-1, 5.0000001201e-1):
        p = fmaf(p, r, f32(c))
    r2 = f32(r * r)
    p = fmaf(p, r2, r)
    p = f32(p + f32(1.0))
    ki = int(k)
    if ki < -125:
        p = f32(p * f32(5.42101086242752217004e-20))
        ki += 64
    if ki > 127:
        p = f32(p * f32(2.0))
        ki -= 1
    scale = np.array([(ki + 127) << 23], np.uint32).view(np.float32)[0]
    res = f32(p * scale)
    if x < f32(-103.972084045410):
        res = f32(0.0)
    if x > f32(88.72283935546875):
        res = f32(np.inf)
    return res


# ---------------------------------------------------------------- glm, column-major m[c][r]
def m4_from_rowmajor(rm):
    rm = np.asarray(rm, np.float32).reshape(4, 4)
    return [[f32(rm[r][c]) for r in range(4)] for c in range(4)]


def m4_mul(A, B):
    R = [[f32(0)] * 4 for _ in range(4)]
    for c in range(4):
        for r in range(4):
            s = f32(A[0][r] * B[c][0])
            s = f32(s + f32(A[1][r] * B[c][1]))
            s = f32(s + f32(A[2][r] * B[c][2]))
            s = f32(s + f32(A[3][r] * B[c][3]))
            R[c][r] = s
    return R


def m4_vec(M, v):
    out = []
    for r in range(4):
        a = f32(f32(M[0][r] * v[0]) + f32(M[1][r] * v[1]))
        b = f32(f32(M[2][r] * v[2]) + f32(M[3][r] * v[3]))
        out.append(f32(a + b))
    return out


def m3_mul(A, B):
    R = [[f32(0)] * 3 for _ in range(3)]
    for c in range(3):
        for r in range(3):
            s = f32(A[0][r] * B[c][0])
            s = f32(s + f32(A[1][r] * B[c][1]))
            s = f32(s + f32(A[2][r] * B[c][2]))
            R[c][r] = s
    return R


def m3_t(A):
    return [[A[r][c] for r in range(3)] for c in range(3)]


def smax(a, b):
    return a if a > b else b


def smin(a, b):
    return a if a < b else b


def cov3d(rot, scale):
    qw, qx, qy, qz = (f32(v) for v in rot)
    dot = f32(f32(f32(qw * qw) + f32(qx * qx)) + f32(f32(qy * qy) + f32(qz * qz)))
    ln = f32(np.sqrt(dot))
    if ln <= 0:
        w, x, y, z = f32(1), f32(0), f32(0), f32(0)
    else:
        inv = f32(f32(1) / ln)
        w, x, y, z = f32(qw * inv), f32(qx * inv), f32(qy * inv), f32(qz * inv)
    one, two = f32(1), f32(2)
    qxx, qyy, qzz = f32(x * x), f32(y * y), f32(z * z)
    qxz, qxy, qyz = f32(x * z), f32(x * y), f32(y * z)
    qwx, qwy, qwz = f32(w * x), f32(w * y), f32(w * z)
    R = [[None] * 3 for _ in range(3)]
    R[0][0] = f32(one - f32(two * f32(qyy + qzz)))
    R[0][1] = f32(two * f32(qxy + qwz))
    R[0][2] = f32(two * f32(qxz - qwy))
    R[1][0] = f32(two * f32(qxy - qwz))
    R[1][1] = f32(one - f32(two * f32(qxx + qzz)))
    R[1][2] = f32(two * f32(qyz + qwx))
    R[2][0] = f32(two * f32(qxz + qwy))
    R[2][1] = f32(two * f32(qyz - qwx))
    R[2][2] = f32(one - f32(two * f32(qxx + qyy)))
    S = [[f32(0)] * 3 for _ in range(3)]
    for i in range(3):
        S[i][i] = expf(scale[i])
    return m3_mul(m3_mul(m3_mul(R, S), m3_t(S)), m3_t(R))


def project(g16, view_rm, proj_rm, W, H, tw, th, fov, scale_div, guard_band=15.0):
    """Per-Gaussian (mean2d, conic, clip z, radius, rendered, rect) of
    renderInternal (codelets.cpp:437-499) + converged binning rectangle."""
    mvp = m4_mul(m4_from_rowmajor(proj_rm), m4_from_rowmajor(view_rm))
    tanfov = f32(math.tan(0.5 * float(f32(fov))))
    tf = f32(_LIBM.tanf(float(f32(f32(fov) / f32(2)))))  # glm::tan(float) -> libm tanf
    fx = f32(f32(W) / f32(f32(2) * tf))
    fy = f32(f32(H) / f32(f32(2) * tf))
    thr = f32(f32(np.sqrt(f32(f32(f32(tw) * f32(tw)) + f32(f32(th) * f32(th))))) * f32(guard_band))
    tiles_x, tiles_y = -(-W // tw), -(-H // th)
    out = []
    for g in np.asarray(g16, np.float32).reshape(-1, 16):
        mean, col, rot, sc, gid = g[0:4], g[4:8], g[8:12], g[12:15], g[15]
        rec = {"rendered": 0, "rect": None}
        if gid <= 0:
            out.append(rec)
            continue
        clip = m4_vec(mvp, [f32(v) for v in mean])
        s = f32(f32(0.5) / clip[3])
        vx = f32(f32(f32(f32(clip[0] * s) + f32(0.5)) * f32(W)) + f32(0))
        vy = f32(f32(f32(f32(clip[1] * s) + f32(0.5)) * f32(H)) + f32(0))
        t = m4_vec(mvp, [mean[0], mean[1], mean[2], f32(1)])
        tx, ty, tz = t[0], t[1], t[2]
        lim = f32(f32(1.3) * tanfov)
        tx = f32(smin(lim, smax(f32(-lim), f32(tx / tz))) * tz)
        ty = f32(smin(lim, smax(f32(-lim), f32(ty / tz))) * tz)
        tz2 = f32(tz * tz)
        J = [[f32(fx / tz), f32(0), f32(f32(-f32(fx * tx)) / tz2)],
             [f32(0), f32(fy / tz), f32(f32(-f32(fy * ty)) / tz2)],
             [f32(0), f32(0), f32(0)]]
        Wm = [[mvp[c][r] for r in range(3)] for c in range(3)]
        T = m3_mul(Wm, J)
        C3 = cov3d(rot, [f32(v / f32(scale_div)) for v in sc])
        cov = m3_mul(m3_mul(m3_t(T), m3_t(C3)), T)
        a, b, c = f32(cov[0][0] + f32(0.3)), cov[0][1], f32(cov[1][1] + f32(0.3))
        det = f32(f32(a * c) - f32(b * b))
        mid = f32(f32(0.5) * f32(a + c))
        q = f32(np.sqrt(smax(f32(0.1), f32(f32(mid * mid) - det))))
        l1, l2 = f32(mid + q), f32(mid - q)
        radius = f32(np.ceil(f32(f32(3) * f32(np.sqrt(smax(l1, l2))))))
        mnx, mny, mxx, mxy = f32(vx - radius), f32(vy - radius), f32(vx + radius), f32(vy + radius)
        dx, dy = f32(mxx - mnx), f32(mxy - mny)
        within = f32(np.sqrt(f32(f32(dx * dx) + f32(dy * dy)))) < thr
        if det == 0:
            conic = (f32(0), f32(0), f32(0), f32(0))
        else:
            inv = f32(f32(1) / det)
            conic = (f32(c * inv), f32(f32(-b) * inv), f32(a * inv), f32(col[3]))
        rec.update(mean2d=(vx, vy), conic=conic, clip_z=clip[2], radius=radius)
        if within and clip[2] < 0:
            rec["rendered"] = 1
            x0 = np.floor(f32(np.floor(mnx) / f32(tw)))
            x1 = np.floor(f32(np.ceil(mxx) / f32(tw)))
            y0 = np.floor(f32(np.floor(mny) / f32(th)))
            y1 = np.floor(f32(np.ceil(mxy) / f32(th)))
            x0, y0 = max(x0, 0.0), max(y0, 0.0)
            x1, y1 = min(x1, tiles_x - 1.0), min(y1, tiles_y - 1.0)
            if x0 <= x1 and y0 <= y1:
                rec["rect"] = (int(x0), int(y0), int(x1), int(y1))
        out.append(rec)
    return out


def render(g16, proj, W, H, tw, th):
    """Converged binning + renderTile (codelets.cpp:358-421): RGBA f32, H x W."""
    g16 = np.asarray(g16, np.float32).reshape(-1, 16)
    tiles_x, tiles_y = -(-W // tw), -(-H // th)
    lists = [[] for _ in range(tiles_x * tiles_y)]
    for i, p in enumerate(proj):
        if p["rendered"] and p["rect"]:
            x0, y0, x1, y1 = p["rect"]
            for ty in range(y0, y1 + 1):
                for tx in range(x0, x1 + 1):
                    lists[ty * tiles_x + tx].append(i)
    img = np.zeros((H, W, 4), np.float32)
    for t, lst in enumerate(lists):
        lst.sort(key=lambda i: (float(proj[i]["clip_z"]), i))
        tx, ty = t % tiles_x, t // tiles_x
        for y in range(ty * th, min((ty + 1) * th, H)):
            for x in range(tx * tw, min((tx + 1) * tw, W)):
                T = f32(1)
                C = [f32(0)] * 4
                for i in lst:
                    k0, k1, k2, k3 = proj[i]["conic"]
                    if k3 == 0:
                        continue
                    dx = f32(proj[i]["mean2d"][0] - f32(x))
                    dy = f32(proj[i]["mean2d"][1] - f32(y))
                    inner = f32(f32(f32(k0 * dx) * dx) + f32(f32(k2 * dy) * dy))
                    power = f32(f32(f32(-0.5) * inner) - f32(f32(k1 * dx) * dy))
                    if power > 0:
                        continue
                    v = f32(k3 * expf(power))
                    alpha = v if v < f32(0.99) else f32(0.99)
                    if alpha < f32(f32(1) / f32(255)):
                        continue
                    test_T = f32(T * f32(f32(1) - alpha))
                    if test_T < f32(0.0001):
                        break
                    col = g16[i, 4:8]
                    C = [f32(C[j] + f32(f32(col[j] * alpha) * T)) for j in range(4)]
                    T = test_T
                img[y, x] = [f32(f32(0) + cj) for cj in C]
    return img, lists
