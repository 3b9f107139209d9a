"""ctypes binding of libgsplat.so (the C ABI declared in include/gsplat.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C gaussian_splat_ipu_amd/csrc``).  There is no fallback: if the library
is missing, importing the renderer raises ``GsplatLibraryError`` -- the frame
path only exists as HIP code.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSPLAT_LIB", os.path.join(_HERE, "lib", "libgsplat.so"))

GS_OK, GS_EINVAL, GS_EDEVICE, GS_EOOM, GS_EOVERFLOW, GS_EIO = range(6)
GS_FLAG_NO_RGBA32F = 1
GS_FLAG_PROFILE = 2
GS_FLAG_BIN_GLOBAL = 4
GS_FLAG_INPUT_ORDER = 8
GS_FLAG_BAND_INTERLEAVED = 16
GS_FLAG_BAND_CULL = 32
GS_FLAG_NO_PAIR_CULL = 64
GS_FLAG_NO_REBALANCE = 128
GS_FLAG_GATHER_COPY = 256
GS_FLAG_LATTICE = 512
GS_FLAG_FAST_EXP = 1024
GS_MAX_GPUS = 16
GS_LAYOUT_ROW_MAJOR = 0
GS_LAYOUT_REF_TILE_MAJOR = 1
GS_K_PROJECT, GS_K_SCAN, GS_K_EMIT, GS_K_SORT, GS_K_BLEND, GS_K_GATHER, GS_K_BLEND_CONT, GS_K_COUNT = range(8)
KERNEL_NAMES = ("project", "scan", "emit", "sort", "blend", "gather", "blend_cont")

_STATUS_NAMES = {
    GS_EINVAL: "GS_EINVAL",
    GS_EDEVICE: "GS_EDEVICE",
    GS_EOOM: "GS_EOOM",
    GS_EOVERFLOW: "GS_EOVERFLOW",
    GS_EIO: "GS_EIO",
}


class GsplatLibraryError(ImportError):
    pass


class GsError(RuntimeError):
    """A non-zero gs_status from the C ABI (the reference throws
    std::runtime_error / logic_error in the same situations)."""

    def __init__(self, status: int, message: str):
        self.status = status
        super().__init__(f"{_STATUS_NAMES.get(status, status)}: {message}")


class Gaussian3D(C.Structure):
    """splat::Gaussian3D (include/splat/ipu_geometry.hpp:305-311), 64 bytes."""

    _fields_ = [
        ("mean", C.c_float * 4),
        ("colour", C.c_float * 4),
        ("rot", C.c_float * 4),
        ("scale", C.c_float * 3),
        ("gid", C.c_float),
    ]


class Config(C.Structure):
    _fields_ = [
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("tile_width", C.c_uint32),
        ("tile_height", C.c_uint32),
        ("guard_tile_width", C.c_uint32),
        ("guard_tile_height", C.c_uint32),
        ("guard_band", C.c_float),
        ("device", C.c_int32),
        ("band_index", C.c_uint32),
        ("band_count", C.c_uint32),
        ("pair_capacity", C.c_uint64),
        ("flags", C.c_uint32),
        ("band_row_begin", C.c_uint32),
        ("band_row_end", C.c_uint32),
        ("band_pad_rows", C.c_uint32),
        # ABI 6: row-band group
        ("num_gpus", C.c_uint32),
        ("device_ids", C.c_int32 * 16),
        ("frames_in_flight", C.c_uint32),
    ]


class CommId(C.Structure):
    """gs_comm_id: the 128 bytes of an ncclUniqueId."""

    _fields_ = [("bytes", C.c_ubyte * 128)]


class FrameStats(C.Structure):
    _fields_ = [
        ("n_gaussians", C.c_uint64),
        ("n_rendered", C.c_uint64),
        ("n_pairs", C.c_uint64),
        ("max_list", C.c_uint64),
        ("pair_capacity", C.c_uint64),
        ("n_tiles", C.c_uint32),
        ("tiles_x", C.c_uint32),
        ("tiles_y", C.c_uint32),
        ("band_y0", C.c_uint32),
        ("band_rows", C.c_uint32),
        ("n_big_tiles", C.c_uint32),
        ("band_stride", C.c_uint32),
        ("n_pairs_binned", C.c_uint64),
        ("bin_global", C.c_uint32),
        ("paths", C.c_uint32),
        ("blend_records", C.c_uint64),
        ("blend_cont_records", C.c_uint64),
        ("cont_keys", C.c_uint64),
        ("cont_lists", C.c_uint32),
        ("cont_max", C.c_uint32),
        ("prefix_overflows", C.c_uint32),
        ("cont_full_sorts", C.c_uint32),
        ("big_pairs", C.c_uint64),
        ("big_prefix_keys", C.c_uint64),
        ("big_window_keys", C.c_uint64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class GroupInfo(C.Structure):
    """gs_group_info (ABI 10)."""

    _fields_ = [
        ("world", C.c_uint32),
        ("local_bands", C.c_uint32),
        ("comm_ranks", C.c_int32),
        ("multi_process", C.c_uint32),
        ("threaded", C.c_uint32),
        ("frames_in_flight", C.c_uint32),
        ("frames", C.c_uint64),
        ("rebalances", C.c_uint64),
        ("timed_frames", C.c_uint64),
        ("bounds", C.c_uint32 * (GS_MAX_GPUS + 1)),
        ("band_rank", C.c_int32 * GS_MAX_GPUS),
        ("device", C.c_int32 * GS_MAX_GPUS),
        ("band_ms", C.c_double * GS_MAX_GPUS),
        ("gather_ms", C.c_double * GS_MAX_GPUS),
    ]

    def as_dict(self):
        k = self.local_bands
        return {
            "world": self.world,
            "local_bands": k,
            "comm_ranks": self.comm_ranks,
            "multi_process": bool(self.multi_process),
            "threaded": bool(self.threaded),
            "frames_in_flight": self.frames_in_flight,
            "frames": self.frames,
            "rebalances": self.rebalances,
            "timed_frames": self.timed_frames,
            "bounds": list(self.bounds[: self.world + 1]),
            "band_rank": list(self.band_rank[:k]),
            "device": list(self.device[:k]),
            "band_ms": list(self.band_ms[:k]),
            "gather_ms": list(self.gather_ms[:k]),
        }


class LatticeStats(C.Structure):
    _fields_ = [
        ("frames", C.c_uint64),
        ("total_slots", C.c_uint64),
        ("dropped", C.c_uint64),
        ("send_failed", C.c_uint64),
        ("zbuf_overrun", C.c_uint64),
        ("records_per_tile", C.c_uint32),
        ("extra_records", C.c_uint32),
        ("slots_per_tile", C.c_uint32),
        ("channel_slots", C.c_uint32),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class SynthParams(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("seed", C.c_uint64),
        ("sh_degree", C.c_int32),
        ("bb_min", C.c_float * 3),
        ("bb_max", C.c_float * 3),
        ("log_scale_mu", C.c_float),
        ("log_scale_sigma", C.c_float),
        ("opacity_lo", C.c_float),
        ("opacity_hi", C.c_float),
        ("cluster_xyz", C.POINTER(C.c_float)),
        ("n_cluster", C.c_uint64),
        ("cluster_sigma", C.c_float),
    ]


_P = C.c_void_p
_FP = C.POINTER(C.c_float)
_SIGS = {
    "gs_abi_version": (C.c_int, []),
    "gs_last_error": (C.c_char_p, []),
    "gs_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "gs_config_init": (C.c_int, [C.POINTER(Config)]),
    "gs_create": (C.c_int, [C.POINTER(Gaussian3D), C.c_size_t, C.POINTER(Config), C.POINTER(_P)]),
    "gs_destroy": (None, [_P]),
    "gs_comm_id_create": (C.c_int, [C.POINTER(CommId)]),
    "gs_create_rank": (C.c_int, [C.POINTER(Gaussian3D), C.c_size_t, C.POINTER(Config), C.POINTER(CommId),
                                 C.c_int, C.c_int, C.POINTER(_P)]),
    "gs_group_bands": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_size_t]),
    "gs_group_get_info": (C.c_int, [_P, C.POINTER(GroupInfo)]),
    "gs_balanced_bands": (C.c_int, [C.POINTER(C.c_double), C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    "gs_group_decide": (C.c_int, [C.POINTER(C.c_uint32), C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_int, C.POINTER(C.c_uint32),
                                  C.POINTER(C.c_uint64)]),
    "gs_get_lattice_stats": (C.c_int, [_P, C.POINTER(LatticeStats)]),
    "gs_read_lattice_slots": (C.c_int, [_P, _FP, C.c_size_t]),
    "gs_set_view": (C.c_int, [_P, _FP]),
    "gs_set_projection": (C.c_int, [_P, _FP]),
    "gs_set_focal": (C.c_int, [_P, C.c_float, C.c_float]),
    "gs_set_sh": (C.c_int, [_P, _FP, _FP, C.c_size_t, C.c_int]),
    "gs_set_band_rows": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32]),
    "gs_set_stream": (C.c_int, [_P, _P]),
    "gs_get_stream": (C.c_int, [_P, C.POINTER(_P)]),
    "gs_render": (C.c_int, [_P]),
    "gs_render_async": (C.c_int, [_P]),
    "gs_sync": (C.c_int, [_P]),
    "gs_read_bgr8": (C.c_int, [_P, C.POINTER(C.c_uint8), C.c_size_t]),
    "gs_read_rgba32f": (C.c_int, [_P, _FP, C.c_size_t, C.c_int]),
    "gs_read_tile_histogram": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_size_t]),
    "gs_get_stats": (C.c_int, [_P, C.POINTER(FrameStats)]),
    "gs_read_bins": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_uint32), C.c_size_t]),
    "gs_read_projected": (C.c_int, [_P, _FP, C.c_size_t]),
    "gs_bgr8_device": (C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_size_t)]),
    "gs_copy_bgr8_device": (C.c_int, [_P, _P, C.c_size_t]),
    "gs_set_bgr8_target": (C.c_int, [_P, _P, C.c_size_t]),
    "gs_kernel_times": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_int]),
    "gs_reset_kernel_times": (C.c_int, [_P]),
    "gs_set_profile_interval": (C.c_int, [_P, C.c_uint32]),
    "gs_ply_load": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "gs_ply_save": (C.c_int, [_P, C.c_char_p]),
    "gs_ply_free": (None, [_P]),
    "gs_ply_count": (C.c_int64, [_P]),
    "gs_ply_has": (C.c_int, [_P, C.c_char_p]),
    "gs_ply_get": (C.c_int, [_P, C.c_char_p, _FP, C.c_size_t]),
    "gs_synth_params_init": (C.c_int, [C.POINTER(SynthParams)]),
    "gs_ply_synthetic": (C.c_int, [C.POINTER(SynthParams), C.POINTER(_P)]),
    "gs_scene_prepare": (C.c_int, [_P, C.POINTER(Gaussian3D), C.c_size_t, _FP]),
    "gs_cpu_point_splat": (C.c_int, [_FP, C.c_size_t, _FP, _FP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_uint8, C.POINTER(C.c_uint8), C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint32), C.c_int]),
    "gs_mat4_mul": (C.c_int, [_FP, _FP, _FP]),
    "gs_mat4_mul_vec4": (C.c_int, [_FP, _FP, _FP]),
    "gs_mat4_transpose": (C.c_int, [_FP, _FP]),
    "gs_cam_look_at": (C.c_int, [_FP, _FP, _FP, _FP]),
    "gs_cam_frustum": (C.c_int, [C.c_float] * 6 + [_FP]),
    "gs_cam_fit_frustum": (C.c_int, [_FP, _FP, C.c_float, C.c_float, _FP]),
    "gs_cam_look_at_bbox": (C.c_int, [_FP, _FP, _FP, C.c_float, _FP]),
    "gs_cam_rotate": (C.c_int, [_FP, C.c_float, _FP, _FP]),
    "gs_cam_translate": (C.c_int, [_FP, _FP, _FP]),
    "gs_cam_mvp_start": (C.c_int, [_FP]),
    "gs_cam_headless": (C.c_int, [_FP, C.c_uint32, C.c_uint32, C.c_float, _FP, _FP]),
    "gs_test_set": (C.c_int, [C.c_char_p, C.c_int64]),
}

_lib = None
_lock = threading.Lock()


def lib():
    """Load libgsplat.so once; raise GsplatLibraryError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise GsplatLibraryError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C gaussian_splat_ipu_amd/csrc` (there is no CPU fallback)"
            )
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        # a GSPLAT_LIB override may be an older A/B build: entry points it
        # lacks are left unbound there (the default library must have all)
        lenient = "GSPLAT_LIB" in os.environ
        for name, (res, args) in _SIGS.items():
            if lenient and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    msg = lib().gs_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "") -> None:
    if rc != GS_OK:
        raise GsError(rc, f"{what}: {last_error()}" if what else last_error())


def fptr(a):
    """float32 numpy array -> float*"""
    return a.ctypes.data_as(_FP)
