"""Tile geometry of the framebuffer: splat::TiledFramebuffer
(include/tileMapping/tile_config.hpp:19-139), float32 arithmetic as in the
reference, with one documented change: the tile grid is ``ceil(W / tw)`` x
``ceil(H / th)`` (partial tiles are rendered and masked) where the reference
uses uint16 integer division and drops the partial row/column
(tile_config.hpp:38-39).  ``ref_tiles_across/down`` keep the
reference's counts.
"""
from __future__ import annotations

import enum
import math

import numpy as np

f32 = np.float32


class Direction(enum.IntEnum):
    """splat::direction (ipu_geometry.hpp:94-100)"""

    left = 0
    right = 1
    up = 2
    down = 3
    none = 4


class Bounds2f:
    """splat::Bounds2f (ipu_geometry.hpp:102-177), float32."""

    def __init__(self, mn, mx):
        self.min = (f32(mn[0]), f32(mn[1]))
        self.max = (f32(mx[0]), f32(mx[1]))

    def centroid(self):
        return (f32((self.max[0] + self.min[0]) * f32(0.5)), f32((self.max[1] + self.min[1]) * f32(0.5)))

    def diagonal(self):
        return (f32(self.max[0] - self.min[0]), f32(self.max[1] - self.min[1]))

    def contains(self, v) -> bool:
        x, y = f32(v[0]), f32(v[1])
        return bool(
            np.ceil(x) >= self.min[0] and np.floor(x) < self.max[0] and np.ceil(y) >= self.min[1] and np.floor(y) < self.max[1]
        )

    def clip(self, fixed: "Bounds2f"):
        """Bounds2f::clip (ipu_geometry.hpp:133-155): (clipped, dirs dict)."""
        tl = list(self.min)
        br = list(self.max)
        dirs = {
            "left": bool(np.floor(tl[0]) < fixed.min[0]),
            "up": bool(np.floor(tl[1]) < fixed.min[1]),
            "right": bool(np.ceil(br[0]) >= fixed.max[0]),
            "down": bool(np.ceil(br[1]) >= fixed.max[1]),
        }
        if dirs["left"]:
            tl[0] = fixed.min[0]
        if dirs["up"]:
            tl[1] = fixed.min[1]
        if dirs["right"]:
            br[0] = fixed.max[0]
        if dirs["down"]:
            br[1] = fixed.max[1]
        return Bounds2f(tl, br), dirs


class TiledFramebuffer:
    def __init__(self, width: int, height: int, tile_width: int, tile_height: int):
        self.width = int(width)
        self.height = int(height)
        self.tile_width = int(tile_width)
        self.tile_height = int(tile_height)
        self.ref_tiles_across = f32(self.width // self.tile_width)  # uint16 division, stored as float
        self.ref_tiles_down = f32(self.height // self.tile_height)
        self.tiles_across = -(-self.width // self.tile_width)
        self.tiles_down = -(-self.height // self.tile_height)
        self.num_tiles = self.tiles_across * self.tiles_down

    # ---- reference helpers (tile_config.hpp:43-126), reference grid width
    def pix_coord_to_tile(self, row: float, col: float) -> float:
        r = f32(np.rint(f32(row)))
        c = f32(np.rint(f32(col)))
        tc = f32(np.floor(f32(c / f32(self.tile_width))))
        tr = f32(np.floor(f32(r / f32(self.tile_height))))
        return f32(tr * self.ref_tiles_across + tc)

    def get_tile_bounds(self, tid: int) -> Bounds2f:
        div = f32(np.floor(f32(f32(tid) / self.ref_tiles_across)))
        mod = f32(f32(tid) - f32(div * self.ref_tiles_across))
        tl = (f32(np.floor(f32(mod * f32(self.tile_width)))), f32(np.floor(f32(div * f32(self.tile_height)))))
        br = (f32(tl[0] + f32(self.tile_width)), f32(tl[1] + f32(self.tile_height)))
        return Bounds2f(tl, br)

    def get_nearby_tile(self, tid: int, received_from: Direction) -> int:
        nta = int(self.ref_tiles_across)
        return {
            Direction.left: tid - 1,
            Direction.right: tid + 1,
            Direction.up: tid - nta,
            Direction.down: tid + nta,
        }.get(received_from, tid)

    @staticmethod
    def manhattan_distance(a, b) -> float:
        return f32(abs(f32(a[0]) - f32(b[0])) + abs(f32(a[1]) - f32(b[1])))

    def get_best_direction(self, src, dst) -> Direction:
        """y-first priority (tile_config.hpp:92-110)."""
        if self.manhattan_distance(src, dst) == 0:
            return Direction.none
        if src[1] < dst[1]:
            return Direction.down
        if src[1] > dst[1]:
            return Direction.up
        if src[0] < dst[0]:
            return Direction.right
        if src[0] > dst[0]:
            return Direction.left
        return Direction.none

    # ---- the build's grid
    def tile_rect_of_bbox(self, bb_min, bb_max):
        """Converged lattice binning: the inclusive tile
        rectangle [floor(floor(min)/t), floor(ceil(max)/t)] clipped to the grid,
        or None."""
        tw, th = f32(self.tile_width), f32(self.tile_height)
        x0 = np.floor(f32(np.floor(f32(bb_min[0])) / tw))
        x1 = np.floor(f32(np.ceil(f32(bb_max[0])) / tw))
        y0 = np.floor(f32(np.floor(f32(bb_min[1])) / th))
        y1 = np.floor(f32(np.ceil(f32(bb_max[1])) / th))
        x0, y0 = max(x0, 0.0), max(y0, 0.0)
        x1, y1 = min(x1, self.tiles_across - 1.0), min(y1, self.tiles_down - 1.0)
        if not (x0 <= x1 and y0 <= y1):
            return None
        return int(x0), int(y0), int(x1), int(y1)

    def band_rows(self, band_count: int):
        """Row bands of tile rows used by the multi-GPU path: list of
        (tile_row0, tile_row1, pixel_row0, pixel_rows)."""
        rpb = math.ceil(self.tiles_down / band_count)
        out = []
        for b in range(band_count):
            ty0 = min(self.tiles_down, b * rpb)
            ty1 = min(self.tiles_down, ty0 + rpb)
            py0 = ty0 * self.tile_height
            rows = max(0, min(self.height, ty1 * self.tile_height) - py0)
            out.append((ty0, ty1, py0, rows))
        return out

    def interleaved_tile_rows(self, band_count: int, band_index: int):
        """Tile rows of an interleaved band (GS_FLAG_BAND_INTERLEAVED): rows
        band_index, band_index + band_count, ...; the band's output holds them
        back to back, tile_height pixel rows each."""
        return list(range(band_index, self.tiles_down, band_count))

    def rows_per_band_padded(self, band_count: int) -> int:
        return math.ceil(self.tiles_down / band_count) * self.tile_height
