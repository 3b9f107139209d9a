"""Row-band decomposition of the framebuffer across GPUs (one process per GPU).

Tile rows are split into ``world`` bands: contiguous (TiledFramebuffer.band_rows)
or interleaved (rank r owns tile rows r, r + world, ...: every rank gets an
equal share of a scene's dense rows; GS_FLAG_BAND_INTERLEAVED).  Rank r renders
its band into a buffer padded to ``rows_per_band_padded`` rows so every rank
contributes the same number of bytes, and one all-gather (RCCL over xGMI on
MI355X, gloo in the CPU tests) collects the padded bands band-major.
``assemble`` drops the padding and returns the H x W x C frame.
"""
from __future__ import annotations

import numpy as np

from .tiles import TiledFramebuffer


def band_bytes(fb: TiledFramebuffer, world: int, channels: int = 3, itemsize: int = 1) -> int:
    return fb.rows_per_band_padded(world) * fb.width * channels * itemsize


def pad_band(band: np.ndarray, fb: TiledFramebuffer, world: int) -> np.ndarray:
    """(rows, W, C) -> (rows_per_band_padded, W, C), zero rows appended."""
    rows = fb.rows_per_band_padded(world)
    out = np.zeros((rows,) + band.shape[1:], band.dtype)
    out[: band.shape[0]] = band
    return out


def assemble(gathered: np.ndarray, fb: TiledFramebuffer, world: int, channels: int = 3,
             interleaved: bool = False) -> np.ndarray:
    """Band-major padded all-gather output -> (H, W, C) frame."""
    rows = fb.rows_per_band_padded(world)
    g = np.asarray(gathered).reshape(world, rows, fb.width, channels)
    if not interleaved:
        parts = [g[r, : b[3]] for r, b in enumerate(fb.band_rows(world))]
        return np.concatenate(parts, 0)
    th = fb.tile_height
    out = np.zeros((fb.height, fb.width, channels), g.dtype)
    for r in range(world):
        for k, ty in enumerate(fb.interleaved_tile_rows(world, r)):
            y0 = ty * th
            n = min(th, fb.height - y0)
            out[y0:y0 + n] = g[r, k * th:k * th + n]
    return out


def extract_band(frame: np.ndarray, fb: TiledFramebuffer, world: int, rank: int,
                 interleaved: bool = False) -> np.ndarray:
    """The rows of ``frame`` that band ``rank`` renders, in its output layout
    (interleaved bands: whole tiles, rows past the image zero)."""
    if not interleaved:
        _, _, py0, n = fb.band_rows(world)[rank]
        return frame[py0:py0 + n]
    th = fb.tile_height
    rows = fb.interleaved_tile_rows(world, rank)
    out = np.zeros((len(rows) * th,) + frame.shape[1:], frame.dtype)
    for k, ty in enumerate(rows):
        y0 = ty * th
        n = min(th, fb.height - y0)
        out[k * th:k * th + n] = frame[y0:y0 + n]
    return out


def row_work(hist: np.ndarray, fb: TiledFramebuffer, tile_cost: float = 128.0) -> np.ndarray:
    """Work per tile row from a frame's tile histogram (list lengths): the
    pairs of the row (sort + blend work) plus a fixed cost per tile (its blend
    workgroup; gs_group.hip kTileCost).  128 pairs per tile since round 6: 8
    balanced bands of config 4, three frames in flight, slowest band 34.9 µs
    at 64, 31.8 at 128, 32.1 at 192, 32.2 at 256 (profiles/r06_direct/)."""
    h = np.asarray(hist, np.float64).reshape(fb.tiles_down, fb.tiles_across)
    return h.sum(1) + tile_cost * fb.tiles_across


def balanced_bands(work, world: int):
    """Contiguous tile-row bands [(ty0, ty1), ...] of nearly equal work: band
    k ends at the row where the cumulative work is closest to k / world of the
    total, every band keeping at least one row (needs len(work) >= world).
    Deterministic, so every rank computes the same split from the same
    histogram."""
    w = np.asarray(work, np.float64)
    T = w.size
    if T < world:
        raise ValueError(f"{T} tile rows cannot make {world} non-empty bands")
    c = np.concatenate([[0.0], np.cumsum(w)])
    bounds = [0]
    for k in range(1, world):
        target = c[-1] * k / world
        b = int(np.searchsorted(c, target))
        if b > 0 and abs(c[b - 1] - target) <= abs(c[min(b, T)] - target):
            b -= 1
        b = max(bounds[-1] + 1, min(b, T - (world - k)))
        bounds.append(b)
    bounds.append(T)
    return [(bounds[i], bounds[i + 1]) for i in range(world)]


def assemble_bands(gathered: np.ndarray, fb: TiledFramebuffer, bands, channels: int = 3) -> np.ndarray:
    """All-gather output of explicit contiguous bands (each padded to the
    tallest band, GpuSplatter(band_rows=..., band_pad_rows=...)) -> (H, W, C)."""
    world = len(bands)
    pad = max(t1 - t0 for t0, t1 in bands) * fb.tile_height
    g = np.asarray(gathered).reshape(world, pad, fb.width, channels)
    parts = []
    for r, (t0, t1) in enumerate(bands):
        y0 = t0 * fb.tile_height
        y1 = min(fb.height, t1 * fb.tile_height)
        parts.append(g[r, : max(0, y1 - y0)])
    return np.concatenate(parts, 0)


def share_comm_id(rank: int, make_id) -> bytes:
    """The row-band group's RCCL id on every rank of an initialised
    torch.distributed group (any backend; bench.py uses gloo): rank 0 calls
    make_id() (splatter.comm_id_create), the others receive its 128 bytes."""
    import torch.distributed as tdist

    box = [make_id() if rank == 0 else None]
    tdist.broadcast_object_list(box, src=0)
    cid = box[0]
    if not isinstance(cid, (bytes, bytearray)) or len(cid) != 128:
        raise RuntimeError("share_comm_id: rank 0 sent no 128-byte RCCL id")
    return bytes(cid)
