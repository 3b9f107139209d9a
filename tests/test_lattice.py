"""The lattice-migration emulator's oracle (oracle/gs_oracle.cpp
or_lattice_*), on the CPU.

Parity status: the reference cannot run here (Poplar), so the lattice is
pinned by two properties the reference's own code implies, not by its output:
  * the initial distribution of the records is calculateMapping /
    applyTileMapping (ipu_rasteriser.cpp:164-214), restated independently
    below, and the first frame renders exactly each tile's initial records
    that pass the guard band and z < 0 (renderInternal, codelets.cpp:437-505);
  * without channel overflow the lattice converges to the single-frame
    binning the build uses everywhere else (SURVEY §8 a9's derivation of the
    converged rectangle): after enough frames its RGBA frame is bit-identical
    to or_render's, and its splatted counters equal the converged list
    lengths on every tile that renders something (the reference never resets
    the counter of a tile that renders nothing, codelets.cpp:501-504).
"""
import math

import numpy as np
import pytest

from conftest import PC12


@pytest.fixture(scope="module")
def pc12(built):
    from gaussian_splat_ipu_amd import scene

    return scene.prepare_scene(scene.load_ply(PC12))


def _frame(view, proj, scale_div, W=1280, H=720, TW=32, TH=20):
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    return O.make_frame(view, proj, W, H, TW, TH, camera.FOV_DEFAULT, scale_div)


def _subsample(g, step):
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[::step].copy()
    a[:, 15] = np.arange(1, a.shape[0] + 1, dtype=np.float32)  # gid = index + 1 (splat.cpp:161)
    return a


def _mapping(n, T):
    """calculateMapping of n 64-float records over T tiles
    (ipu_rasteriser.cpp:164-193): (grains per tile, tiles' slot counts)."""
    gpt = math.ceil(float(np.float32(n * 64) / np.float32(T * 64.0)))
    full = n // gpt
    rem = n - full * gpt
    return gpt, rem


@pytest.mark.parametrize("n", [7, 1440, 1440 * 3, 5000, 14005])
def test_initial_distribution(built, pc12, n):
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = pc12
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)
    a = np.resize(a, (n, 16)).copy()
    a[:, 15] = np.arange(1, n + 1, dtype=np.float32)
    view, proj = camera.headless(bb, 1280, 720)
    L = O.Lattice(a, _frame(view, proj, 0.1))
    r = L.read()
    T = 40 * 36
    gpt, rem = _mapping(n, T)
    assert (r["gpt"], r["rem"]) == (gpt, rem)
    per = gpt + 600
    assert L.total_slots == T * per + rem
    want = np.zeros(L.total_slots, np.float32)
    j = np.arange(n)
    t = j // gpt  # applyTileMapping: elementsPerTile floats per tile, in order
    want[t * per + (j - t * gpt)] = j + 1
    np.testing.assert_array_equal(r["slots"], want)
    assert r["frames"] == 0


def test_first_frame_renders_each_tiles_initial_records(built, pc12):
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = pc12
    view, proj = camera.headless(bb, 1280, 720)
    f = _frame(view, proj, 0.1)
    L = O.Lattice(g, f)
    L.step(f)
    r = L.read()
    n = np.ascontiguousarray(g).shape[0]
    gpt, _ = _mapping(n, 1440)
    rendered = O.project(g, f)["rendered"] != 0
    want = np.bincount(np.arange(n)[rendered] // gpt, minlength=1440).astype(np.uint32)
    np.testing.assert_array_equal(r["hist"], want)
    assert r["frames"] == 1 and r["dropped"] == 0


@pytest.mark.parametrize("scale_div,step", [(0.1, 16), (1.0, 32)])
def test_lattice_converges_to_the_single_frame_render(built, pc12, scale_div, step):
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = pc12
    a = _subsample(g, step)  # sparse enough that no channel overflows
    view, proj = camera.headless(bb, 1280, 720)
    f = _frame(view, proj, scale_div)
    L = O.Lattice(a, f)
    ref = O.render(a, f)
    for _ in range(60):
        L.step(f)
    r = L.read()
    assert r["dropped"] == 0 and r["send_failed"] == 0 and r["overrun"] == 0
    same = r["rgba"].view(np.uint32) == ref["rgba"].view(np.uint32)
    assert same.all(), f"{(~same).sum()} values differ from the converged frame"
    live = ref["hist"] > 0
    np.testing.assert_array_equal(r["hist"][live], ref["hist"][live])
    # every record rests on the tiles that "contain" its projected mean:
    # Bounds2f::contains tests ceil(x) >= min.x (ipu_geometry.hpp:163-165), so
    # a mean less than a pixel left of / above a tile counts for it too, and a
    # record can anchor in up to 2 x 2 tiles
    gids = r["slots"][r["slots"] > 0].astype(np.int64)
    cnt = np.bincount(gids)
    assert cnt.max() <= 4 and (cnt > 1).sum() < 0.2 * len(gids)


def test_lattice_transients_overflow_on_the_reference_scene(built, pc12):
    """The full point_cloud_12 scene overflows the 75-record channels and the
    tiles' vertsIn on the way to convergence (counted, as the reference drops
    silently); the frames are deterministic."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = pc12
    view, proj = camera.headless(bb, 1280, 720)
    f = _frame(view, proj, 1.0)
    runs = []
    for _ in range(2):
        L = O.Lattice(g, f)
        failed = 0
        for _ in range(8):
            L.step(f)
            failed += L.read()["send_failed"]
        runs.append((L.read(), failed))
    (a, fa), (b, fb) = runs
    assert fa == fb and fa > 0
    np.testing.assert_array_equal(a["rgba"].view(np.uint32), b["rgba"].view(np.uint32))
    np.testing.assert_array_equal(a["slots"], b["slots"])
