"""The render server's ``--device cpu`` path: the reference's CPU point
splatter (src/splat/cpu_rasteriser.cpp:9-92: projectPoints, splatPoints,
buildTileHistogram), through libgsplat's host code (gs_cpu_point_splat).

This is a separate device of the render server (splat.cpp:250-256), a point
splatter -- not a Gaussian rasteriser and not a fallback of GpuSplatter."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, fptr, lib


def splat_points(xyz, view_rm, proj_rm, width: int, height: int, tile_w: int, tile_h: int, value: int = 25,
                 image: np.ndarray | None = None, nthreads: int = 0):
    """(image H x W x 3 uint8 BGR, tile histogram (W//tw)*(H//th) uint32,
    splatted count).  ``image`` (zeroed if None) is accumulated into, as the
    reference's cv::Mat (splat.cpp:247 zeroes it per frame)."""
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    img = np.zeros((height, width, 3), np.uint8) if image is None else image
    assert img.shape == (height, width, 3) and img.dtype == np.uint8 and img.flags.c_contiguous
    hist = np.zeros((width // tile_w) * (height // tile_h), np.uint32)
    v = np.ascontiguousarray(view_rm, np.float32).reshape(16)
    p = np.ascontiguousarray(proj_rm, np.float32).reshape(16)
    cnt = C.c_uint32(0)
    check(lib().gs_cpu_point_splat(fptr(xyz), xyz.shape[0], fptr(v), fptr(p), width, height, tile_w, tile_h,
                                   value, img.ctypes.data_as(C.POINTER(C.c_uint8)),
                                   hist.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(cnt), nthreads),
          "gs_cpu_point_splat")
    return img, hist, int(cnt.value)
