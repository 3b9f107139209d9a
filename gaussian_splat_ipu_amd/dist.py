"""Row-band decomposition of the framebuffer across GPUs (one process per GPU).

Tile rows are split into ``world`` contiguous bands (TiledFramebuffer.band_rows);
rank r renders band r into a buffer padded to ``rows_per_band_padded`` rows so
every rank contributes the same number of bytes, and one all-gather (RCCL over
xGMI on MI355X, gloo in the CPU tests) collects the padded bands band-major.
``assemble`` drops the padding rows and returns the H x W x C frame.
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


def assemble(gathered: np.ndarray, fb: TiledFramebuffer, world: int, channels: int = 3) -> np.ndarray:
    """Band-major padded all-gather output -> (H, W, C) frame."""
    rows = fb.rows_per_band_padded(world)
    g = np.asarray(gathered).reshape(world, rows, fb.width, channels)
    parts = [g[r, : b[3]] for r, b in enumerate(fb.band_rows(world))]
    return np.concatenate(parts, 0)
