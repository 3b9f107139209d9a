"""Frames from recycled device memory (gs_test_set("debug_poison", 1): every
device buffer the renderer allocates starts as 0xA5 bytes instead of the zeros a fresh
process's first allocation happens to hold).  A stage that reads memory no
earlier stage of the frame wrote gives a different frame -- or faults -- here,
while passing every test in a fresh process.  Each case is checked bit for
bit against the CPU oracle's whole frame.

The global-atomic binning's scan used to count the slots past the last tile of
its 8192-tile round as small lists; the sort then read tile ids past the end
of the small-list queue and re-sorted whatever tiles those stale words named
(wrong frames in row bands, a faulting sort under this poison).
"""
import numpy as np
import pytest

from test_gpu_fullsize import _check_frame, _splatter
from test_gpu_group import _check, _group, _oracle

pytestmark = pytest.mark.gpu


@pytest.fixture
def poison(test_hook):
    test_hook("debug_poison", 1)


@pytest.fixture(scope="module")
def clustered(built):
    from conftest import PC12
    from gaussian_splat_ipu_amd import scene

    src = scene.load_ply(PC12)
    centres = np.stack([src["x"], src["y"], src["z"]], 1)
    return scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=120_000, seed=8, sh_degree=0, cluster_xyz=centres,
                                                               cluster_sigma=0.02)))


@pytest.mark.parametrize("bin_global", [False, True])
@pytest.mark.parametrize("T", [16, 32])
def test_poisoned_full_frame(clustered, poison, bin_global, T):
    """Both binning paths, three frames (the second and third take the
    big-list hint: lazy prefixes with the chunked binning, the sample sort with
    the global one)."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = clustered
    W, H = 1920, 1080
    view, proj = camera.headless(bb, W, H)
    s = _splatter(g, view, proj, W, H, T, bin_global=bin_global)
    f = O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0)
    ref = O.render(g, f)
    for k in range(3):
        s.execute()
        _check_frame(s, g, f, ref, lists=(k == 2))
    assert s.stats()["bin_global"] == int(bin_global)
    s.close()


@pytest.mark.parametrize("bin_global", [False, True])
def test_poisoned_row_bands(clustered, poison, bin_global):
    """8 emulated row bands (copy transport), 2 frames in flight, an orbit:
    the band renderers, their re-balanced splits and the assembled frames."""
    from gaussian_splat_ipu_amd import camera

    g, bb = clustered
    W, H, T = 1280, 720, 16
    _, proj = camera.headless(bb, W, H)
    with _group(g, W, H, T, num_gpus=8, device_ids=[0] * 8, frames_in_flight=2, bin_global=bin_global) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        for k in (0, 30, 30, 60):
            view = camera.orbit_view(k)
            s.set_view_wire(view)
            s.execute()
            f, ref = _oracle(g, view, proj, W, H, T)
            _check(s, g, f, ref, lists=(k == 60))
