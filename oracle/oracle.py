"""ctypes binding of the CPU ORACLE (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")


class Frame(C.Structure):
    _fields_ = [
        ("view_rm", C.c_float * 16),
        ("proj_rm", C.c_float * 16),
        ("fov", C.c_float),
        ("scale_div", C.c_float),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("tile_w", C.c_int32),
        ("tile_h", C.c_int32),
        ("guard_tile_w", C.c_int32),
        ("guard_tile_h", C.c_int32),
        ("guard_band", C.c_float),
        ("band_ty0", C.c_int32),
        ("band_ty1", C.c_int32),
    ]


class Proj(C.Structure):
    _fields_ = [
        ("mean2d", C.c_float * 2),
        ("cov2d", C.c_float * 3),
        ("conic", C.c_float * 4),
        ("clip_z", C.c_float),
        ("radius", C.c_float),
        ("rendered", C.c_int32),
        ("rect", C.c_int32 * 4),
    ]


PROJ_DTYPE = np.dtype(
    [
        ("mean2d", "<f4", (2,)),
        ("cov2d", "<f4", (3,)),
        ("conic", "<f4", (4,)),
        ("clip_z", "<f4"),
        ("radius", "<f4"),
        ("rendered", "<i4"),
        ("rect", "<i4", (4,)),
    ]
)
assert PROJ_DTYPE.itemsize == C.sizeof(Proj)


class Stats(C.Structure):
    _fields_ = [
        ("n_rendered", C.c_int64),
        ("n_pairs", C.c_int64),
        ("max_list", C.c_int64),
        ("n_tiles", C.c_int32),
        ("tiles_x", C.c_int32),
        ("tiles_y", C.c_int32),
    ]


_lib = None
_FP = C.POINTER(C.c_float)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_expf.restype = C.c_float
        L.or_expf.argtypes = [C.c_float]
        L.or_mat4_mul.argtypes = [_FP, _FP, _FP]
        L.or_mat4_mul_vec4.argtypes = [_FP, _FP, _FP]
        L.or_frame_scalars.argtypes = [C.POINTER(Frame), _FP, _FP, _FP, _FP]
        L.or_project.restype = C.c_int
        L.or_project.argtypes = [_FP, C.c_int64, C.POINTER(Frame), C.c_void_p, C.c_int]
        L.or_bin.restype = C.c_int64
        L.or_bin.argtypes = [C.c_void_p, C.c_int64, C.POINTER(Frame), C.POINTER(C.c_int64), C.POINTER(C.c_uint32), C.c_int64, C.c_int]
        L.or_blend.restype = C.c_int
        L.or_blend.argtypes = [_FP, C.c_void_p, C.POINTER(Frame), C.POINTER(C.c_int64), C.POINTER(C.c_uint32), _FP, C.c_int]
        L.or_pack_bgr8.argtypes = [_FP, C.c_int64, C.POINTER(C.c_uint8)]
        L.or_render.restype = C.c_int
        L.or_render.argtypes = [_FP, C.c_int64, C.POINTER(Frame), _FP, C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(Stats), C.c_int]
        L.or_point_splat.restype = C.c_uint32
        L.or_point_splat.argtypes = [_FP, C.c_int64, _FP, _FP, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.c_int]
        L.or_lattice_create.restype = C.c_void_p
        L.or_lattice_create.argtypes = [_FP, C.c_int64, C.POINTER(Frame)]
        L.or_lattice_step.restype = C.c_int
        L.or_lattice_step.argtypes = [C.c_void_p, C.POINTER(Frame), C.c_int]
        L.or_lattice_total_slots.restype = C.c_int64
        L.or_lattice_total_slots.argtypes = [C.c_void_p]
        L.or_lattice_read.argtypes = [C.c_void_p, _FP, C.POINTER(C.c_uint32), _FP, C.POINTER(C.c_uint64)]
        L.or_lattice_destroy.argtypes = [C.c_void_p]
        L.or_sh_colours.argtypes = [_FP, C.c_int64, _FP, _FP, C.c_int, _FP, _FP]
        L.or_camera_position.argtypes = [_FP, _FP]
        L.or_omp_team_cpus.restype = C.c_int
        L.or_omp_team_cpus.argtypes = [C.c_int, C.POINTER(C.c_int), C.c_int, C.c_double]
        _lib = L
    return _lib


def make_frame(view_rm, proj_rm, width, height, tile_w, tile_h, fov, scale_div,
               guard_band=15.0, guard_tile=None, band=None) -> Frame:
    f = Frame()
    v = np.ascontiguousarray(view_rm, np.float32).reshape(16)
    p = np.ascontiguousarray(proj_rm, np.float32).reshape(16)
    for i in range(16):
        f.view_rm[i] = v[i]
        f.proj_rm[i] = p[i]
    f.fov, f.scale_div = fov, scale_div
    f.width, f.height, f.tile_w, f.tile_h = width, height, tile_w, tile_h
    gw, gh = guard_tile if guard_tile else (0, 0)
    f.guard_tile_w, f.guard_tile_h = gw, gh
    f.guard_band = guard_band
    f.band_ty0, f.band_ty1 = band if band else (0, 0)
    return f


def expf(x: float) -> float:
    return lib().or_expf(x)


def _g(g64):
    a = np.ascontiguousarray(g64).view(np.float32).reshape(-1, 16)
    return a


def project(g64, frame: Frame, nthreads: int = 0) -> np.ndarray:
    a = _g(g64)
    out = np.zeros(a.shape[0], PROJ_DTYPE)
    lib().or_project(a.ctypes.data_as(_FP), a.shape[0], C.byref(frame), out.ctypes.data, nthreads)
    return out


def bin_lists(proj: np.ndarray, frame: Frame, nthreads: int = 0):
    """(tile_start[T+1] int64, list[P] uint32)."""
    tiles_x = -(-frame.width // frame.tile_w)
    tiles_y = -(-frame.height // frame.tile_h)
    ty1 = frame.band_ty1 if frame.band_ty1 > frame.band_ty0 else tiles_y
    T = tiles_x * (min(ty1, tiles_y) - frame.band_ty0)
    ts = np.zeros(T + 1, np.int64)
    rect = proj["rect"]
    ok = (proj["rendered"] != 0) & (rect[:, 0] <= rect[:, 2])
    P = int(((rect[ok, 2] - rect[ok, 0] + 1).astype(np.int64) * (rect[ok, 3] - rect[ok, 1] + 1)).sum())
    lst = np.zeros(max(P, 1), np.uint32)
    got = lib().or_bin(proj.ctypes.data, proj.shape[0], C.byref(frame), ts.ctypes.data_as(C.POINTER(C.c_int64)),
                       lst.ctypes.data_as(C.POINTER(C.c_uint32)), lst.size, nthreads)
    assert got == P, (got, P)
    return ts, lst[:P]


def render(g64, frame: Frame, nthreads: int = 0, want_rgba: bool = True):
    """Full oracle frame -> dict(rgba, bgr, hist, stats)."""
    a = _g(g64)
    tiles_x = -(-frame.width // frame.tile_w)
    tiles_y = -(-frame.height // frame.tile_h)
    ty0 = frame.band_ty0
    ty1 = frame.band_ty1 if frame.band_ty1 > frame.band_ty0 else tiles_y
    ty1 = min(ty1, tiles_y)
    rows = max(0, min(frame.height, ty1 * frame.tile_h) - ty0 * frame.tile_h)
    T = tiles_x * (ty1 - ty0)
    rgba = np.zeros((rows, frame.width, 4), np.float32) if want_rgba else None
    bgr = np.zeros((rows, frame.width, 3), np.uint8)
    hist = np.zeros(max(T, 1), np.uint32)
    st = Stats()
    rc = lib().or_render(
        a.ctypes.data_as(_FP), a.shape[0], C.byref(frame),
        rgba.ctypes.data_as(_FP) if want_rgba else None,
        bgr.ctypes.data_as(C.POINTER(C.c_uint8)),
        hist.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(st), nthreads,
    )
    assert rc == 0
    return {
        "rgba": rgba,
        "bgr": bgr,
        "hist": hist[:T],
        "stats": {k: getattr(st, k) for k, _ in Stats._fields_},
    }


def point_splat(xyz, view_rm, proj_rm, width, height, tile_w, tile_h, nthreads: int = 0):
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    img = np.zeros((height, width, 3), np.uint8)
    hist = np.zeros((width // tile_w) * (height // tile_h), np.uint32)
    v = np.ascontiguousarray(view_rm, np.float32)
    p = np.ascontiguousarray(proj_rm, np.float32)
    cnt = lib().or_point_splat(
        xyz.ctypes.data_as(_FP), xyz.shape[0], v.ctypes.data_as(_FP), p.ctypes.data_as(_FP),
        width, height, tile_w, tile_h, img.ctypes.data_as(C.POINTER(C.c_uint8)),
        hist.ctypes.data_as(C.POINTER(C.c_uint32)), nthreads,
    )
    return img, hist, int(cnt)


class Lattice:
    """The reference's multi-frame lattice migration, one
    step() per frame: or_lattice_* in gs_oracle.cpp."""

    def __init__(self, g64, frame: Frame):
        a = _g(g64)
        self._keep = a
        self.width, self.height = frame.width, frame.height
        self.T = (frame.width // frame.tile_w) * (frame.height // frame.tile_h)
        self.h = lib().or_lattice_create(a.ctypes.data_as(_FP), a.shape[0], C.byref(frame))
        if not self.h:
            raise ValueError("or_lattice_create: invalid lattice configuration")
        self.total_slots = int(lib().or_lattice_total_slots(self.h))

    def step(self, frame: Frame, nthreads: int = 0):
        assert lib().or_lattice_step(self.h, C.byref(frame), nthreads) == 0

    def read(self):
        """dict(rgba (H, W, 4), hist (T,), slots (gid per vertsIn slot),
        frames, dropped, send_failed, overrun, gpt, rem)."""
        rgba = np.zeros((self.height, self.width, 4), np.float32)
        hist = np.zeros(self.T, np.uint32)
        slots = np.zeros(self.total_slots, np.float32)
        cnt = np.zeros(6, np.uint64)
        lib().or_lattice_read(self.h, rgba.ctypes.data_as(_FP), hist.ctypes.data_as(C.POINTER(C.c_uint32)),
                              slots.ctypes.data_as(_FP), cnt.ctypes.data_as(C.POINTER(C.c_uint64)))
        out = {"rgba": rgba, "hist": hist, "slots": slots}
        out.update({k: int(v) for k, v in zip(("frames", "dropped", "send_failed", "overrun", "gpt", "rem"), cnt)})
        return out

    def close(self):
        if self.h:
            lib().or_lattice_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def omp_team_cpus(nthreads: int = 0, spin_ms: float = 50.0):
    """The CPU ids the OpenMP team's threads ran on (one per thread)."""
    cpus = (C.c_int * 1024)()
    n = lib().or_omp_team_cpus(int(nthreads), cpus, 1024, float(spin_ms))
    return [int(cpus[i]) for i in range(min(n, 1024))]


def camera_position(view_rm):
    v = np.ascontiguousarray(view_rm, np.float32).reshape(16)
    out = np.zeros(3, np.float32)
    lib().or_camera_position(v.ctypes.data_as(_FP), out.ctypes.data_as(_FP))
    return out


def sh_colours(g64, f_dc, f_rest, degree: int, view_rm):
    """The scene with every colour replaced by its SH colour for the camera of
    view_rm (the product's gs_set_sh, restated)."""
    g = _g(g64)
    n = g.shape[0]
    dc = np.ascontiguousarray(f_dc, np.float32).reshape(n, 3)
    rest = None if f_rest is None else np.ascontiguousarray(f_rest, np.float32).reshape(n, 45)
    out = np.empty_like(g)
    cp = camera_position(view_rm)
    lib().or_sh_colours(g.ctypes.data_as(_FP), n, dc.ctypes.data_as(_FP),
                        None if rest is None else rest.ctypes.data_as(_FP), int(degree), cp.ctypes.data_as(_FP),
                        out.ctypes.data_as(_FP))
    return out.view(np.ascontiguousarray(g64).dtype).reshape(np.shape(g64))
