"""gaussian_splat_ipu_amd: MI355X-native Gaussian-splat tile rasteriser.

The project -> bin -> sort -> blend frame path of Nmjfry/gaussian_splat_ipu
runs as hand-written HIP kernels for gfx950 behind the C ABI of
``lib/libgsplat.so`` (include/gsplat.h).  This package is the Python face of
that ABI (ctypes) and of the host-side data path (PLY ingest, scene
preparation, camera).
"""
from ._lib import GsError, GsplatLibraryError, lib  # noqa: F401
from .tiles import Bounds2f, Direction, TiledFramebuffer  # noqa: F401

__all__ = ["GsError", "GsplatLibraryError", "lib", "TiledFramebuffer", "Bounds2f", "Direction"]
