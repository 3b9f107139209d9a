"""GpuSplatter: the MI355X drop-in for ``splat::IpuSplatter``
(include/splat/ipu_rasteriser.hpp:20-55, src/splat/ipu_rasteriser.cpp).

Same surface, same argument meaning::

    IpuSplatter(const Gaussians&, TiledFramebuffer&, bool noAMP)   -> GpuSplatter(gaussians, fb)
    updateModelView(glm::mat4) / updateProjection(glm::mat4)      -> update_model_view / update_projection
    updateFocalLengths(fov, lambda1 / 10)                          -> update_focal_lengths
    GraphManager::execute(splatter)                                -> execute()
    getFrameBuffer(cv::Mat&)  (8-bit BGR, H x W)                   -> get_frame_buffer()
    getIPUHistogram(std::vector<u32>&)                             -> get_histogram()

Every call goes through the C ABI of libgsplat.so; there is no CPU path.
Errors raise GsError (the reference throws std::runtime_error).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import camera
from ._lib import (
    GS_FLAG_BAND_CULL,
    GS_FLAG_GATHER_COPY,
    GS_FLAG_LATTICE,
    GS_FLAG_FAST_EXP,
    GS_FLAG_NO_PAIR_CULL,
    GS_FLAG_NO_REBALANCE,
    GS_FLAG_BAND_INTERLEAVED,
    GS_FLAG_BIN_GLOBAL,
    GS_FLAG_INPUT_ORDER,
    GS_FLAG_NO_RGBA32F,
    GS_FLAG_PROFILE,
    GS_K_COUNT,
    GS_LAYOUT_REF_TILE_MAJOR,
    GS_LAYOUT_ROW_MAJOR,
    KERNEL_NAMES,
    CommId,
    Config,
    FrameStats,
    Gaussian3D,
    GroupInfo,
    LatticeStats,
    check,
    fptr,
    lib,
)
from .scene import GAUSSIAN_DTYPE, from_float16
from .tiles import TiledFramebuffer


def device_count() -> int:
    c = C.c_int(0)
    rc = lib().gs_device_count(C.byref(c))
    return c.value if rc == 0 else 0


def comm_id_create() -> bytes:
    """Rank 0 of a one-process-per-GPU group: a fresh ncclUniqueId (128 bytes)
    to hand to every rank's GpuSplatter(comm_id=...)."""
    cid = CommId()
    check(lib().gs_comm_id_create(C.byref(cid)), "gs_comm_id_create")
    return bytes(cid.bytes)


class GpuSplatter:
    """One renderer (a band of one device), or -- with ``num_gpus`` or
    ``comm_id`` -- a row-band group: the tile rows split over several GPUs and
    gathered by one all-gather per frame inside execute() (gs_group.hip)."""

    def __init__(
        self,
        gaussians,
        fb: TiledFramebuffer,
        *,
        guard_band: float = 15.0,
        guard_tile=None,
        device: int = -1,
        band_index: int = 0,
        band_count: int = 1,
        pair_capacity: int = 0,
        write_rgba: bool = True,
        profile: bool = False,
        bin_global: bool = False,
        input_order: bool = False,
        band_interleaved: bool = False,
        band_cull: bool = False,
        pair_cull: bool = True,
        band_rows=None,
        band_pad_rows: int = 0,
        num_gpus: int = 0,
        device_ids=None,
        frames_in_flight: int = 0,
        rebalance: bool = True,
        gather_copy: bool = False,
        comm_id: bytes | None = None,
        rank: int = 0,
        world: int = 1,
        lattice: bool = False,
        fast_exp: bool = False,
    ):
        g = gaussians
        if isinstance(g, np.ndarray) and g.dtype != GAUSSIAN_DTYPE:
            g = from_float16(g)
        g = np.ascontiguousarray(g)
        self.n = int(g.shape[0])
        self.fb = fb
        cfg = Config()
        check(lib().gs_config_init(C.byref(cfg)))
        cfg.width, cfg.height = fb.width, fb.height
        cfg.tile_width, cfg.tile_height = fb.tile_width, fb.tile_height
        if guard_tile is not None:
            cfg.guard_tile_width, cfg.guard_tile_height = guard_tile
        cfg.guard_band = guard_band
        cfg.device = device
        cfg.band_index, cfg.band_count = band_index, band_count
        cfg.pair_capacity = pair_capacity
        if band_rows is not None:  # explicit contiguous band: tile rows [begin, end)
            cfg.band_row_begin, cfg.band_row_end = int(band_rows[0]), int(band_rows[1])
        cfg.band_pad_rows = int(band_pad_rows)
        cfg.flags = (
            (0 if write_rgba else GS_FLAG_NO_RGBA32F)
            | (GS_FLAG_PROFILE if profile else 0)
            | (GS_FLAG_BIN_GLOBAL if bin_global else 0)
            | (GS_FLAG_INPUT_ORDER if input_order else 0)
            | (GS_FLAG_BAND_INTERLEAVED if band_interleaved else 0)
            | (GS_FLAG_BAND_CULL if band_cull else 0)
            | (0 if pair_cull else GS_FLAG_NO_PAIR_CULL)
            | (0 if rebalance else GS_FLAG_NO_REBALANCE)
            | (GS_FLAG_GATHER_COPY if gather_copy else 0)
            | (GS_FLAG_LATTICE if lattice else 0)
            | (GS_FLAG_FAST_EXP if fast_exp else 0)
        )
        cfg.num_gpus = int(num_gpus)
        if device_ids is not None:
            for k, d in enumerate(device_ids):
                cfg.device_ids[k] = int(d)
        cfg.frames_in_flight = int(frames_in_flight)
        self.cfg = cfg
        self.group = num_gpus > 0 or comm_id is not None
        self.world = world if comm_id is not None else max(1, int(num_gpus))
        h = C.c_void_p()
        gp = g.ctypes.data_as(C.POINTER(Gaussian3D)) if self.n else None
        if comm_id is not None:
            cid = CommId()
            C.memmove(cid.bytes, bytes(comm_id), 128)
            check(lib().gs_create_rank(gp, self.n, C.byref(cfg), C.byref(cid), int(rank), int(world), C.byref(h)),
                  "gs_create_rank")
        else:
            check(lib().gs_create(gp, self.n, C.byref(cfg), C.byref(h)), "gs_create")
        self._h = h
        st = self.stats()
        self.n_tiles = st["n_tiles"]
        self.band_y0 = st["band_y0"]
        self.band_rows = st["band_rows"]
        # reference defaults: fov = radians(40), fxy[1] = lambda1 / 10 = 0.1
        self.update_focal_lengths(camera.FOV_DEFAULT, 0.1)

    # ------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().gs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------ inputs
    def update_model_view(self, mv) -> None:
        """IpuSplatter::updateModelView (ipu_rasteriser.cpp:86-93): takes a
        glm-layout (column-major) 4x4 and streams its transpose."""
        self.set_view_wire(camera.to_wire(mv))

    def update_projection(self, mp) -> None:
        self.set_projection_wire(camera.to_wire(mp))

    def set_view_wire(self, rowmajor) -> None:
        a = np.ascontiguousarray(rowmajor, dtype=np.float32).reshape(16)
        check(lib().gs_set_view(self._h, fptr(a)))

    def set_projection_wire(self, rowmajor) -> None:
        a = np.ascontiguousarray(rowmajor, dtype=np.float32).reshape(16)
        check(lib().gs_set_projection(self._h, fptr(a)))

    def update_focal_lengths(self, fov: float, scale_divisor: float) -> None:
        """IpuSplatter::updateFocalLengths (ipu_rasteriser.cpp:108-110)."""
        check(lib().gs_set_focal(self._h, fov, scale_divisor))
        self.fov, self.scale_divisor = fov, scale_divisor

    def set_sh(self, f_dc, f_rest=None, degree: int = 3) -> None:
        """Opt-in view-dependent colour (gs_set_sh): f_dc (n x 3) and f_rest
        (n x 45, the PLY's f_rest_0..44) in input order; degree < 0 = off."""
        if degree < 0:
            check(lib().gs_set_sh(self._h, None, None, 0, -1), "gs_set_sh")
            return
        dc = np.ascontiguousarray(f_dc, np.float32).reshape(self.n, 3)
        rest = None if f_rest is None else np.ascontiguousarray(f_rest, np.float32).reshape(self.n, 45)
        check(lib().gs_set_sh(self._h, fptr(dc), None if rest is None else fptr(rest), self.n, int(degree)),
              "gs_set_sh")

    def set_band_rows(self, row_begin: int, row_end: int, pad_rows: int = 0) -> None:
        """Move this renderer's contiguous band to tile rows [row_begin, row_end)
        (gs_set_band_rows; the renderer must have been created with room for
        them, e.g. band_rows=(0, tiles_y))."""
        check(lib().gs_set_band_rows(self._h, int(row_begin), int(row_end), int(pad_rows)), "gs_set_band_rows")
        # (the stats keep the last frame's band until the next frame)
        th = self.fb.tile_height
        self.n_tiles = (int(row_end) - int(row_begin)) * self.fb.tiles_across
        self.band_y0 = int(row_begin) * th
        self.band_rows = min(self.fb.height, int(row_end) * th) - self.band_y0

    def set_stream(self, stream_ptr: int | None) -> None:
        check(lib().gs_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    # ------------------------------------------------------------ execute
    def get_stream(self) -> int:
        """hipStream_t (as int) the frames are enqueued on; wrap it with
        torch.cuda.ExternalStream to order work after a frame."""
        s = C.c_void_p()
        check(lib().gs_get_stream(self._h, C.byref(s)))
        return int(s.value or 0)

    def execute(self) -> None:
        """GraphManager::execute -> IpuSplatter::execute (blocking)."""
        check(lib().gs_render(self._h), "gs_render")

    def execute_async(self) -> None:
        check(lib().gs_render_async(self._h), "gs_render_async")

    def sync(self) -> None:
        check(lib().gs_sync(self._h), "gs_sync")

    # ------------------------------------------------------------ outputs
    def get_frame_buffer(self, out: np.ndarray | None = None) -> np.ndarray:
        """IpuSplatter::getFrameBuffer: rows x W x 3 uint8 BGR, row-major
        (into ``out`` when given: a C-contiguous uint8 array of at least that
        many bytes, e.g. pinned host memory)."""
        if out is None:
            out = np.empty((self.band_rows, self.fb.width, 3), np.uint8)
        elif not (out.dtype == np.uint8 and out.flags.c_contiguous and out.nbytes >= self.band_rows * self.fb.width * 3):
            raise ValueError("get_frame_buffer: out must be a C-contiguous uint8 array of rows x W x 3 bytes")
        check(lib().gs_read_bgr8(self._h, out.ctypes.data_as(C.POINTER(C.c_uint8)), out.nbytes), "gs_read_bgr8")
        return out

    def get_rgba(self, layout: str = "row_major") -> np.ndarray:
        if layout == "row_major":
            out = np.empty((self.band_rows, self.fb.width, 4), np.float32)
            lay = GS_LAYOUT_ROW_MAJOR
        else:
            out = np.empty(self.n_tiles * self.fb.tile_width * self.fb.tile_height * 4, np.float32)
            lay = GS_LAYOUT_REF_TILE_MAJOR
        check(lib().gs_read_rgba32f(self._h, fptr(out), out.size, lay), "gs_read_rgba32f")
        return out

    def get_histogram(self) -> np.ndarray:
        """IpuSplatter::getIPUHistogram: per-tile render-list length."""
        out = np.empty(self.n_tiles, np.uint32)
        check(lib().gs_read_tile_histogram(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size))
        return out

    def stats(self) -> dict:
        st = FrameStats()
        check(lib().gs_get_stats(self._h, C.byref(st)))
        return st.as_dict()

    def lattice_stats(self) -> dict:
        """lattice=True: the emulated lattice after the last frame
        (gs_get_lattice_stats)."""
        st = LatticeStats()
        check(lib().gs_get_lattice_stats(self._h, C.byref(st)))
        return st.as_dict()

    def lattice_slots(self) -> np.ndarray:
        """lattice=True: the gid of every vertsIn slot, tile-major (0 = empty)."""
        n = self.lattice_stats()["total_slots"]
        out = np.empty(n, np.float32)
        check(lib().gs_read_lattice_slots(self._h, fptr(out), out.size))
        return out

    def get_bins(self):
        """(tile_start[T+1] uint64, list[P] uint32): depth-sorted per-tile lists."""
        st = self.stats()
        ts = np.empty(st["n_tiles"] + 1, np.uint64)
        lst = np.empty(max(st["n_pairs"], 1), np.uint32)
        check(
            lib().gs_read_bins(
                self._h,
                ts.ctypes.data_as(C.POINTER(C.c_uint64)),
                ts.size,
                lst.ctypes.data_as(C.POINTER(C.c_uint32)),
                lst.size,
            )
        )
        return ts, lst[: st["n_pairs"]]

    def get_projected(self) -> np.ndarray:
        """(N, 12) float32: mean2d[2], conic[4], clip z, radius, rect tx0 ty0 tx1 ty1."""
        out = np.empty((self.n, 12), np.float32)
        check(lib().gs_read_projected(self._h, fptr(out), out.size))
        return out

    def bgr8_device(self):
        p = C.c_void_p()
        nbytes = C.c_size_t()
        check(lib().gs_bgr8_device(self._h, C.byref(p), C.byref(nbytes)))
        return p.value, nbytes.value

    def set_bgr8_target(self, dst_ptr, nbytes: int = 0) -> None:
        """Later frames write their padded BGR8 band at device address dst_ptr
        (None: the renderer's own buffer)."""
        check(lib().gs_set_bgr8_target(self._h, C.c_void_p(dst_ptr or 0), nbytes))

    def copy_bgr8_device(self, dst_ptr: int, nbytes: int) -> None:
        check(lib().gs_copy_bgr8_device(self._h, C.c_void_p(dst_ptr), nbytes))

    def bands(self):
        """Group: the split of the last frame, [(ty0, ty1), ...] tile rows per band."""
        b = (C.c_uint32 * (self.world + 1))()
        check(lib().gs_group_bands(self._h, b, self.world + 1))
        return [(b[i], b[i + 1]) for i in range(self.world)]

    def group_info(self) -> dict:
        """Group: world, local bands, RCCL rank count (ncclCommCount), whether
        one host thread per band enqueues, and each local band's average band
        and all-gather times of the profiled frames (gs_group_get_info)."""
        gi = GroupInfo()
        check(lib().gs_group_get_info(self._h, C.byref(gi)), "gs_group_get_info")
        return gi.as_dict()

    def kernel_times(self) -> dict:
        avg = (C.c_double * GS_K_COUNT)()
        cnt = (C.c_uint64 * GS_K_COUNT)()
        check(lib().gs_kernel_times(self._h, avg, cnt, GS_K_COUNT))
        return {KERNEL_NAMES[k]: (avg[k], cnt[k]) for k in range(GS_K_COUNT)}

    def reset_kernel_times(self) -> None:
        check(lib().gs_reset_kernel_times(self._h))

    def set_profile_interval(self, every: int) -> None:
        """Stage events on every `every`-th frame only (each event costs device time)."""
        check(lib().gs_set_profile_interval(self._h, every))

    # reference-spelled aliases (ipu_rasteriser.hpp:20-55)
    updateModelView = update_model_view
    updateProjection = update_projection
    updateFocalLengths = update_focal_lengths
    getFrameBuffer = get_frame_buffer
    getIPUHistogram = get_histogram
