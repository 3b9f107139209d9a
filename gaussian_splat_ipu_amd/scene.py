"""Host-side data path: PLY/XYZ ingest, synthetic scenes, scene preparation.

Python face of the C++ loader in ``csrc/host/gs_scene.cpp`` (reference:
src/splat/file_io.cpp:11-77 for loading, src/main/splat.cpp:83-163 for the
scene preparation of the render server).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import Gaussian3D, SynthParams, check, fptr, lib

# Gaussian3D as a numpy record view (ipu_geometry.hpp:305-311)
GAUSSIAN_DTYPE = np.dtype(
    [("mean", "<f4", (4,)), ("colour", "<f4", (4,)), ("rot", "<f4", (4,)), ("scale", "<f4", (3,)), ("gid", "<f4")]
)
assert GAUSSIAN_DTYPE.itemsize == 64


class Ply:
    """A loaded vertex element: named float32 columns (splat::Ply,
    include/splat/file_io.hpp:14-25, plus any f_rest_* SH coefficients)."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle)

    def __del__(self):
        try:
            if self._h:
                lib().gs_ply_free(self._h)
                self._h = None
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def __len__(self) -> int:
        return int(lib().gs_ply_count(self._h))

    def has(self, name: str) -> bool:
        return bool(lib().gs_ply_has(self._h, name.encode()))

    def __getitem__(self, name: str) -> np.ndarray:
        out = np.empty(len(self), dtype=np.float32)
        check(lib().gs_ply_get(self._h, name.encode(), fptr(out), out.size), f"property {name}")
        return out

    def save(self, path: str) -> None:
        check(lib().gs_ply_save(self._h, str(path).encode()), "gs_ply_save")


def load_ply(path: str) -> Ply:
    """splat::loadPoints (file_io.cpp:44-55): .ply (all 14 3DGS properties
    required) or .xyz."""
    h = C.c_void_p()
    check(lib().gs_ply_load(str(path).encode(), C.byref(h)), f"load {path}")
    return Ply(h.value)


@dataclass
class SynthSpec:
    n: int = 1_000_000
    seed: int = 1
    sh_degree: int = 3
    bb_min: tuple = (-4.36, -3.12, -2.58)
    bb_max: tuple = (4.36, 3.12, 2.58)
    log_scale_mu: float = -5.6  # median radius 4 px at 1080p with fxy[1] = 1 (tools/calibrate_synth.py)
    log_scale_sigma: float = 0.5
    opacity_lo: float = 0.5
    opacity_hi: float = 8.0
    cluster_xyz: np.ndarray | None = None
    cluster_sigma: float = 0.02


def synthetic(spec: SynthSpec) -> Ply:
    """Seeded synthetic 3DGS scene in the INRIA vertex layout (SURVEY §8 d)."""
    sp = SynthParams()
    check(lib().gs_synth_params_init(C.byref(sp)))
    sp.n = spec.n
    sp.seed = spec.seed
    sp.sh_degree = spec.sh_degree
    for i in range(3):
        sp.bb_min[i] = spec.bb_min[i]
        sp.bb_max[i] = spec.bb_max[i]
    sp.log_scale_mu = spec.log_scale_mu
    sp.log_scale_sigma = spec.log_scale_sigma
    sp.opacity_lo = spec.opacity_lo
    sp.opacity_hi = spec.opacity_hi
    keep = None
    if spec.cluster_xyz is not None:
        keep = np.ascontiguousarray(spec.cluster_xyz, dtype=np.float32).reshape(-1, 3)
        sp.cluster_xyz = keep.ctypes.data_as(C.POINTER(C.c_float))
        sp.n_cluster = keep.shape[0]
        sp.cluster_sigma = spec.cluster_sigma
    h = C.c_void_p()
    check(lib().gs_ply_synthetic(C.byref(sp), C.byref(h)), "gs_ply_synthetic")
    del keep
    return Ply(h.value)


def prepare_scene(ply: Ply):
    """Scene preparation of the render server (splat.cpp:83-163).

    Returns ``(gaussians, bb)``: a (N,) GAUSSIAN_DTYPE array (64-B records)
    and the 6-float bounding box (min xyz, max xyz) of the centred points."""
    n = len(ply)
    g = np.zeros(n, dtype=GAUSSIAN_DTYPE)
    bb = np.zeros(6, dtype=np.float32)
    check(
        lib().gs_scene_prepare(ply.handle, g.ctypes.data_as(C.POINTER(Gaussian3D)), n, fptr(bb)),
        "gs_scene_prepare",
    )
    return g, bb


def as_float16(g: np.ndarray) -> np.ndarray:
    """(N,) GAUSSIAN_DTYPE -> (N, 16) float32 view."""
    return np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)


def from_float16(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32).reshape(-1, 16)
    return a.view(GAUSSIAN_DTYPE).reshape(-1)


def sh_arrays(ply: Ply):
    """(f_dc n x 3, f_rest n x 45 or None) of a 3DGS PLY in input order: the
    view-dependent colour's coefficients (GpuSplatter.set_sh)."""
    dc = np.stack([ply[f"f_dc_{c}"] for c in range(3)], 1).astype(np.float32)
    rest = None
    if ply.has("f_rest_0"):
        rest = np.stack([ply[f"f_rest_{k}"] for k in range(45)], 1).astype(np.float32)
    return dc, rest
