"""GPU parity of the lattice-migration emulator (GS_FLAG_LATTICE, SURVEY §8
f4; gs_lattice.hip) against the CPU oracle's (or_lattice_*), frame by frame:
RGBA f32 bit-identical, BGR8, the splatted histogram, the gid of every vertsIn
slot and the overflow counters all equal.  The frames are the reference's
transient ones (codelets.cpp:143-641 + the exchange of edge_builder.cpp:15-84),
stepped from its initial distribution of the records by index."""
import numpy as np
import pytest

from conftest import PC12
from test_gpu_parity import assert_same_bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pc12(built):
    from gaussian_splat_ipu_amd import scene

    return scene.prepare_scene(scene.load_ply(PC12))


def _pair(g, W, H, TW, TH):
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    return GpuSplatter(g, TiledFramebuffer(W, H, TW, TH), device=0, lattice=True)


def _step_both(s, L, g, view, proj, scale_div, W, H, TW, TH):
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, scale_div)
    s.execute()
    f = O.make_frame(view, proj, W, H, TW, TH, camera.FOV_DEFAULT, scale_div)
    L.step(f)


def _check(s, L, what):
    from oracle import oracle as O

    r = L.read()
    assert_same_bits(s.get_rgba(), r["rgba"], f"{what}: RGBA f32")
    bgr = np.zeros((r["rgba"].shape[0] * r["rgba"].shape[1], 3), np.uint8)
    O.lib().or_pack_bgr8(r["rgba"].ctypes.data_as(O._FP), bgr.shape[0],
                         bgr.ctypes.data_as(O.C.POINTER(O.C.c_uint8)))
    np.testing.assert_array_equal(s.get_frame_buffer().reshape(-1, 3), bgr, err_msg=f"{what}: BGR8")
    np.testing.assert_array_equal(s.get_histogram(), r["hist"], err_msg=f"{what}: splatted")
    np.testing.assert_array_equal(s.lattice_slots(), r["slots"], err_msg=f"{what}: vertsIn slots")
    st = s.lattice_stats()
    assert st["frames"] == r["frames"]
    assert (st["dropped"], st["send_failed"], st["zbuf_overrun"]) == (r["dropped"], r["send_failed"],
                                                                       r["overrun"]), what
    assert (st["records_per_tile"], st["extra_records"]) == (r["gpt"], r["rem"])
    return r


@pytest.mark.parametrize("scale_div,frames,every", [(0.1, 6, 1), (1.0, 24, 6)])
def test_lattice_frames_equal_the_oracle(pc12, scale_div, frames, every):
    """point_cloud_12 at the reference's own geometry (1280x720, 32x20 tiles,
    headless camera).  At fxy[1] = 1 the channels overflow within a few frames
    and the tiles' vertsIn within ~20: the failure paths are compared too."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = pc12
    view, proj = camera.headless(bb, 1280, 720)
    s = _pair(g, 1280, 720, 32, 20)
    L = O.Lattice(g, O.make_frame(view, proj, 1280, 720, 32, 20, camera.FOV_DEFAULT, scale_div))
    failed = 0
    for k in range(frames):
        _step_both(s, L, g, view, proj, scale_div, 1280, 720, 32, 20)
        if (k + 1) % every == 0 or k == 0:
            r = _check(s, L, f"frame {k}")
            failed += r["send_failed"]
    if scale_div == 1.0:
        assert failed > 0


def test_lattice_orbit_small_scene_and_16x16_tiles(pc12):
    """Fewer records than tiles (one per tile, the last tile's remainder), a
    moving camera (records change anchors every frame), 16 x 16 tiles."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = pc12
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[::37][:3000].copy()
    a[:, 15] = np.arange(1, a.shape[0] + 1, dtype=np.float32)
    _, proj = camera.headless(bb, 1280, 720)
    s = _pair(a, 1280, 720, 16, 16)
    L = O.Lattice(a, O.make_frame(camera.orbit_view(0), proj, 1280, 720, 16, 16, camera.FOV_DEFAULT, 1.0))
    for k in range(10):
        _step_both(s, L, a, camera.orbit_view(3 * k), proj, 1.0, 1280, 720, 16, 16)
        _check(s, L, f"orbit frame {k}")


def test_lattice_converges_to_the_gpu_frame_path(pc12):
    """Without overflow the lattice converges to the converged binning: after
    60 steps the emulator's frame is bit-identical to the frame path's (two
    independent GPU paths), its histogram equal on every rendering tile."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    g, bb = pc12
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[::16].copy()
    a[:, 15] = np.arange(1, a.shape[0] + 1, dtype=np.float32)
    view, proj = camera.headless(bb, 1280, 720)
    s = _pair(a, 1280, 720, 32, 20)
    ref = GpuSplatter(a, TiledFramebuffer(1280, 720, 32, 20), device=0)
    for x in (s, ref):
        x.set_view_wire(view)
        x.set_projection_wire(proj)
        x.update_focal_lengths(camera.FOV_DEFAULT, 0.1)
    ref.execute()
    for _ in range(60):
        s.execute_async()
    s.sync()
    st = s.lattice_stats()
    assert st["frames"] == 60 and st["dropped"] == 0 and st["send_failed"] == 0
    assert_same_bits(s.get_rgba(), ref.get_rgba(), "converged lattice vs frame path")
    h, rh = s.get_histogram(), ref.get_histogram()
    np.testing.assert_array_equal(h[rh > 0], rh[rh > 0])


def test_render_server_lattice_mode(built, tmp_path):
    """bin/splat --lattice: the render server's frames are the emulated IPU's
    (every frame one lattice step); after 5 frames its test.png equals the
    oracle lattice's fifth frame."""
    import os
    import struct
    import subprocess
    import zlib

    from conftest import ROOT
    from gaussian_splat_ipu_amd import camera, scene
    from oracle import oracle as O

    exe = os.path.join(ROOT, "gaussian_splat_ipu_amd", "bin", "splat")
    out = tmp_path / "test.png"
    r = subprocess.run([exe, "--input", PC12, "--device", "gpu", "--lattice", "--out", str(out), "--frames", "5"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    data = out.read_bytes()
    w, h = struct.unpack(">II", data[16:24])
    idat = data[data.index(b"IDAT") + 4:data.index(b"IEND") - 8]
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * 3)[:, 1:].reshape(h, w, 3)
    g, bb = scene.prepare_scene(scene.load_ply(PC12))
    view, proj = camera.headless(bb, 1280, 720)
    f = O.make_frame(view, proj, 1280, 720, 32, 20, camera.FOV_DEFAULT, 0.1)
    L = O.Lattice(g, f)
    for _ in range(5):
        L.step(f)
    rgba = L.read()["rgba"]
    bgr = np.zeros((h * w, 3), np.uint8)
    O.lib().or_pack_bgr8(rgba.ctypes.data_as(O._FP), h * w, bgr.ctypes.data_as(O.C.POINTER(O.C.c_uint8)))
    np.testing.assert_array_equal(raw[:, :, ::-1].reshape(-1, 3), bgr)
