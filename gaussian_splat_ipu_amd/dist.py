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
