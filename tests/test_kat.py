"""Known-answer tests carried over from the reference's own tests
(tests/test.cpp, codelets/tests/codelets.cpp), run against both the product's
host math (csrc/host/gs_camera.cpp via the C ABI, tiles.py) and the oracle's
independent glm restatement."""
import ctypes as C
import math

import numpy as np
import pytest

from gaussian_splat_ipu_amd import Direction, TiledFramebuffer


def _oracle_mat4_mul_vec4(m, v):
    from oracle import oracle as O

    m = np.ascontiguousarray(m, np.float32).reshape(16)
    v = np.ascontiguousarray(v, np.float32)
    out = np.zeros(4, np.float32)
    fp = C.POINTER(C.c_float)
    O.lib().or_mat4_mul_vec4(m.ctypes.data_as(fp), v.ctypes.data_as(fp), out.ctypes.data_as(fp))
    return out


def test_glm_mat4_times_vec4(built):
    """tests/test.cpp:21-34 and codelets/tests/codelets.cpp:34-51:
    transpose(make_mat4(1..16)) * (2,4,6,8) = (60,140,220,300)."""
    from gaussian_splat_ipu_amd import camera

    m = camera.transpose(camera.make_mat4(np.arange(1, 17, dtype=np.float32)))
    v = np.array([2, 4, 6, 8], np.float32)
    np.testing.assert_array_equal(camera.mat4_mul_vec4(m, v), [60, 140, 220, 300])
    np.testing.assert_array_equal(_oracle_mat4_mul_vec4(m, v), [60, 140, 220, 300])


def test_glm_look_at_transform(built):
    """codelets/tests/codelets.cpp:53-69: lookAt((10,10,10), 0, (0,1,0)) * origin
    = (0, 0, -sqrt(300), 1) with |z err| <= 1e-5."""
    from gaussian_splat_ipu_amd import camera

    view = camera.look_at((10, 10, 10), (0, 0, 0), (0, 1, 0))
    t = camera.mat4_mul_vec4(view, (0, 0, 0, 1))
    assert t[0] == 0.0 and t[1] == 0.0 and t[3] == 1.0
    assert abs(-math.sqrt(300.0) - t[2]) <= 1e-5
    t2 = _oracle_mat4_mul_vec4(view, np.array([0, 0, 0, 1], np.float32))
    np.testing.assert_array_equal(t, t2)


def test_tile_bounds_and_distances():
    """codelets/tests/codelets.cpp:71-97 at the reference's 32x20 tiles."""
    tfb = TiledFramebuffer(1280, 720, 32, 20)
    tb = tfb.get_tile_bounds(3)
    tb1 = tfb.get_tile_bounds(1)
    assert tfb.manhattan_distance(tb.min, tb1.min) == 2 * 32
    mid120 = tfb.get_tile_bounds(120).centroid()
    nxt = tfb.get_nearby_tile(120, Direction.right)
    down = tfb.get_nearby_tile(120, Direction.down)
    assert tfb.manhattan_distance(mid120, tfb.get_tile_bounds(nxt).centroid()) == 32
    assert tfb.manhattan_distance(mid120, tfb.get_tile_bounds(down).centroid()) == 20


def test_best_direction_y_first():
    """codelets/tests/codelets.cpp:99-140.  The consistent expectations (dir,
    dir3, dir4, dir5) hold; the two stale ones (:122, :128 expect `right`) are
    recorded with the value the code actually computes -- getBestDirection
    checks y before x (tile_config.hpp:92-110)."""
    tfb = TiledFramebuffer(1280, 720, 32, 20)
    tb, tb2, tb3 = (tfb.get_tile_bounds(t).centroid() for t in (0, 40, 39))
    assert tfb.get_best_direction(tb, tb2) == Direction.down
    assert tfb.get_best_direction(tb2, tb) == Direction.up
    assert tfb.get_best_direction(tb2, tb2) == Direction.none
    assert tfb.get_best_direction(tb3, tb) == Direction.left
    # stale in the reference (expects right): y-first gives up
    assert tfb.get_best_direction(tb2, tb3) == Direction.up
    # stale (expects right): tile 0 -> the tile holding (640, 360) is below
    dst = tfb.pix_coord_to_tile(640.0, 360.0)
    assert tfb.get_best_direction(tb, tfb.get_tile_bounds(int(dst)).centroid()) == Direction.down


def test_pix_coord_to_tile_log_line():
    """splat.cpp:123-126 logs the tile of pixel (719, 1279): 35 * 40 + 39."""
    tfb = TiledFramebuffer(1280, 720, 32, 20)
    assert tfb.pix_coord_to_tile(719.0, 1279.0) == 1439.0
    assert tfb.num_tiles == 1440 and int(tfb.ref_tiles_across) == 40


def test_bounds_clip_directions():
    """Bounds2f::clip (ipu_geometry.hpp:133-155): the halo directions whose
    converged union is the binning rectangle."""
    from gaussian_splat_ipu_amd.tiles import Bounds2f

    tile = Bounds2f((32, 20), (64, 40))
    _, d = Bounds2f((30.5, 25.0), (40.0, 39.0)).clip(tile)
    assert d == {"left": True, "up": False, "right": False, "down": False}
    _, d = Bounds2f((33.0, 21.0), (63.5, 39.2)).clip(tile)
    assert d == {"left": False, "up": False, "right": True, "down": True}


@pytest.mark.parametrize("w,h,tw,th", [(1280, 720, 32, 20), (1920, 1080, 16, 16), (1920, 1080, 48, 30)])
def test_band_layout_covers_the_frame(w, h, tw, th):
    tfb = TiledFramebuffer(w, h, tw, th)
    for n in (1, 2, 3, 4, 8):
        bands = tfb.band_rows(n)
        assert bands[0][2] == 0
        assert sum(b[3] for b in bands) == h
        for (ty0, ty1, py0, rows), nxt in zip(bands, bands[1:]):
            assert ty1 == nxt[0] and py0 + rows == nxt[2]
        assert max(b[3] for b in bands) <= tfb.rows_per_band_padded(n)
