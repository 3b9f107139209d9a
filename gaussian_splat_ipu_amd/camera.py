"""Camera and matrix helpers (glm conventions, column-major 4x4).

numpy arrays of shape (4, 4) here are indexed ``m[c, r]`` (column, row) like
glm; ``to_wire`` gives the row-major float[16] that IpuSplatter streams to the
device (ipu_rasteriser.cpp:86-102).  All arithmetic runs in the C++ host code
(csrc/host/gs_camera.cpp) so it is identical to what the render server uses.
"""
from __future__ import annotations

import math

import numpy as np

from ._lib import check, fptr, lib


def _m(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32).reshape(4, 4)


def _v(a, n) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32).reshape(n)


def identity() -> np.ndarray:
    return np.eye(4, dtype=np.float32)


def mat4_mul(a, b) -> np.ndarray:
    a, b = _m(a), _m(b)
    out = np.empty((4, 4), np.float32)
    check(lib().gs_mat4_mul(fptr(a), fptr(b), fptr(out)))
    return out


def mat4_mul_vec4(m, v) -> np.ndarray:
    m, v = _m(m), _v(v, 4)
    out = np.empty(4, np.float32)
    check(lib().gs_mat4_mul_vec4(fptr(m), fptr(v), fptr(out)))
    return out


def make_mat4(values) -> np.ndarray:
    """glm::make_mat4: 16 floats read column-major."""
    return _v(values, 16).reshape(4, 4).copy()


def transpose(m) -> np.ndarray:
    return np.ascontiguousarray(_m(m).T)


def to_wire(m) -> np.ndarray:
    """glm::transpose(m) flattened: the row-major floats of updateModelView."""
    return np.ascontiguousarray(_m(m).T).reshape(16)


def look_at(eye, center, up) -> np.ndarray:
    out = np.empty((4, 4), np.float32)
    check(lib().gs_cam_look_at(fptr(_v(eye, 3)), fptr(_v(center, 3)), fptr(_v(up, 3)), fptr(out)))
    return out


def frustum(l, r, b, t, n, f) -> np.ndarray:
    out = np.empty((4, 4), np.float32)
    check(lib().gs_cam_frustum(l, r, b, t, n, f, fptr(out)))
    return out


def fit_frustum(bb_min, bb_max, fov, aspect) -> np.ndarray:
    """splat::fitFrustumToBoundingBox (src/splat/geometry.cpp:9-24)."""
    out = np.empty((4, 4), np.float32)
    check(lib().gs_cam_fit_frustum(fptr(_v(bb_min, 3)), fptr(_v(bb_max, 3)), fov, aspect, fptr(out)))
    return out


def look_at_bbox(bb_min, bb_max, up, scale) -> np.ndarray:
    """splat::lookAtBoundingBox (src/splat/camera.cpp:10-15)."""
    out = np.empty((4, 4), np.float32)
    check(lib().gs_cam_look_at_bbox(fptr(_v(bb_min, 3)), fptr(_v(bb_max, 3)), fptr(_v(up, 3)), scale, fptr(out)))
    return out


def rotate(m, angle_rad, axis) -> np.ndarray:
    out = np.empty((4, 4), np.float32)
    check(lib().gs_cam_rotate(fptr(_m(m)), angle_rad, fptr(_v(axis, 3)), fptr(out)))
    return out


def translate(m, v) -> np.ndarray:
    out = np.empty((4, 4), np.float32)
    check(lib().gs_cam_translate(fptr(_m(m)), fptr(_v(v, 3)), fptr(out)))
    return out


def mvp_start() -> np.ndarray:
    """The hard-coded first-frame view of the render server (splat.cpp:235-241)."""
    out = np.empty((4, 4), np.float32)
    check(lib().gs_cam_mvp_start(fptr(out)))
    return out


def radians(deg: float) -> float:
    """glm::radians in float32: degrees * 0.01745329251994329576923690768489f."""
    return float(np.float32(deg) * np.float32(0.01745329251994329576923690768489))


def headless(bb6, width: int, height: int, fov: float | None = None):
    """(view_rowmajor[16], proj_rowmajor[16]) of the headless render server:
    view = mvpStart, projection = fitFrustumToBoundingBox(bb in eye space,
    fov, width / height) (splat.cpp:186-199,235-244)."""
    fov = FOV_DEFAULT if fov is None else fov
    v = np.empty(16, np.float32)
    p = np.empty(16, np.float32)
    check(lib().gs_cam_headless(fptr(_v(bb6, 6)), width, height, fov, fptr(v), fptr(p)))
    return v, p


def orbit_view(k: int, n_frames: int = 120) -> np.ndarray:
    """Orbit camera of config 5: V_k = mvpStart * Ry(360 deg * k / n) (row-major wire)."""
    m = rotate(mvp_start(), radians(360.0 * k / n_frames), (0.0, 1.0, 0.0))
    return to_wire(m)


FOV_DEFAULT = radians(40.0)  # glm::radians(40.f), splat.cpp:170
