"""GPU parity at the BASELINE.json configs' full sizes, plus the readback /
overflow / fallback contracts of the C ABI.

Every headline number of bench.py is measured on one of these workloads, so
each is rendered here through the C ABI and compared bit for bit with the CPU
oracle (oracle/, test infrastructure):

- config 3 (configs[2]): synthetic 1M Gaussians, SH degree 3, 1920x1080,
  16x16 tiles, seed 1, headless camera, fxy[1] = 1 -- bench.py's exact scene;
- config 4 (configs[3]): the same scene under the 8-band work-balanced row
  split with the band cull, bands assembled back into the full frame;
- config 5 (configs[4]): 8M Gaussians clustered around point_cloud_12's
  positions (N(0, 0.02) jitter, seed 8), 3840x2160, orbit frames k = 0, 30,
  60, 90 of the 120-frame orbit.

The tile lists are compared through their offsets and a SHA-256 of the list
array (36 M entries at config 5), the frames bit for bit.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import PC12

pytestmark = pytest.mark.gpu


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _same_bits(a, b, what):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), f"{what}: {(~same).sum()} of {a.size} values differ"


@pytest.fixture(scope="module")
def config3(built):
    from gaussian_splat_ipu_amd import camera, scene

    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=1_000_000, seed=1, sh_degree=3)))
    view, proj = camera.headless(bb, 1920, 1080)
    return g, view, proj


def _splatter(g, view, proj, W, H, T, **kw):
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    s = GpuSplatter(g, TiledFramebuffer(W, H, T, T), device=0, **kw)
    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
    return s


def _check_frame(s, g, f, ref, lists=True):
    from oracle import oracle as O

    st = s.stats()
    assert st["n_rendered"] == ref["stats"]["n_rendered"]
    assert st["n_pairs"] == ref["stats"]["n_pairs"]
    assert st["max_list"] == ref["stats"]["max_list"]
    np.testing.assert_array_equal(s.get_histogram(), ref["hist"])
    _same_bits(s.get_rgba(), ref["rgba"], "RGBA f32")
    np.testing.assert_array_equal(s.get_frame_buffer(), ref["bgr"])
    if lists:
        ts, lst = s.get_bins()
        rts, rlst = O.bin_lists(O.project(g, f), f)
        np.testing.assert_array_equal(ts.astype(np.int64), rts)
        assert _sha(lst) == _sha(rlst), "tile lists differ"


def test_config3_1m_1080p_full_size(config3):
    """configs[2] at its stated size: the bench's exact scene and camera."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, view, proj = config3
    s = _splatter(g, view, proj, 1920, 1080, 16, profile=False)
    s.execute()
    f = O.make_frame(view, proj, 1920, 1080, 16, 16, camera.FOV_DEFAULT, 1.0)
    ref = O.render(g, f)
    assert ref["stats"]["n_pairs"] > 2_000_000
    _check_frame(s, g, f, ref)
    s.close()


def test_config4_1m_8_band_split_assembles_to_oracle(config3):
    """configs[3]: the 1M scene under the 8-band work-balanced split with the
    band cull (what bench.py --gpus 8 renders per rank).  Every band equals
    the oracle's band, and the padded all-gather layout reassembles the
    oracle's full frame."""
    from gaussian_splat_ipu_amd import camera, dist as gdist
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    g, view, proj = config3
    W, H, T = 1920, 1080, 16
    fb = TiledFramebuffer(W, H, T, T)
    full = O.render(g, O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0))
    bands = gdist.balanced_bands(gdist.row_work(full["hist"], fb), 8)
    pad = max(t1 - t0 for t0, t1 in bands)
    gathered, rgba = [], []
    for t0, t1 in bands:
        s = _splatter(g, view, proj, W, H, T, band_rows=(t0, t1), band_pad_rows=pad, band_cull=True)
        s.execute()
        band = s.get_frame_buffer()
        y0, y1 = t0 * T, min(H, t1 * T)
        np.testing.assert_array_equal(band, full["bgr"][y0:y1])
        np.testing.assert_array_equal(s.get_histogram(), full["hist"].reshape(-1, fb.tiles_across)[t0:t1].reshape(-1))
        rgba.append(s.get_rgba())
        slot = np.zeros((pad * T, W, 3), np.uint8)
        slot[: y1 - y0] = band
        gathered.append(slot)
        s.close()
    np.testing.assert_array_equal(gdist.assemble_bands(np.stack(gathered), fb, bands), full["bgr"])
    _same_bits(np.concatenate(rgba, 0), full["rgba"], "stacked band RGBA")


@pytest.mark.parametrize("k", [0, 30, 60, 90])
def test_config5_8m_4k_orbit_full_size(built, config5_scene, k):
    """configs[4] at its stated size: 8M clustered Gaussians at 3840x2160,
    orbit frame k (big lists > 2048 keys: the sample sort on the second frame
    of the renderer)."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, proj, s = config5_scene
    view = camera.orbit_view(k)
    s.set_view_wire(view)
    s.execute()
    s.execute()  # the second frame takes the big-list launch (hint from the first)
    f = O.make_frame(view, proj, 3840, 2160, 16, 16, camera.FOV_DEFAULT, 1.0)
    ref = O.render(g, f)
    assert s.stats()["n_big_tiles"] > 0
    _check_frame(s, g, f, ref)



def test_config5_8m_4k_8_band_group(built, config5_scene):
    """configs[4] as the 8-GPU job renders it: the row-band group over 8 bands
    (emulated on this GPU: repeated device ids, device-copy gather -- every
    other part is the 8-GPU code), two orbit frames (the split re-balances
    between them), every frame bit for bit the oracle's whole frame."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    g, proj, _ = config5_scene
    W, H, T = 3840, 2160, 16
    with GpuSplatter(g, TiledFramebuffer(W, H, T, T), num_gpus=8, device_ids=[0] * 8, frames_in_flight=2) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        for k in (0, 30):
            view = camera.orbit_view(k)
            s.set_view_wire(view)
            s.execute()
            s.execute()  # (the second frame: the big-list launch and a re-balanced split)
            ref = O.render(g, O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0))
            st = s.stats()
            assert st["n_pairs"] == ref["stats"]["n_pairs"]
            assert st["max_list"] == ref["stats"]["max_list"]
            np.testing.assert_array_equal(s.get_histogram(), ref["hist"])
            np.testing.assert_array_equal(s.get_frame_buffer(), ref["bgr"])
            _same_bits(s.get_rgba(), ref["rgba"], f"RGBA f32, orbit frame {k}")
            b = s.bands()
            assert len(b) == 8 and b[0][0] == 0 and b[-1][1] == (H + T - 1) // T

@pytest.fixture(scope="module")
def config5_scene(built):
    from gaussian_splat_ipu_amd import camera, scene

    src = scene.load_ply(PC12)
    centres = np.stack([src["x"], src["y"], src["z"]], 1)
    ply = scene.synthetic(scene.SynthSpec(n=8_000_000, seed=8, sh_degree=0, cluster_xyz=centres,
                                          cluster_sigma=0.02))
    g, bb = scene.prepare_scene(ply)
    del ply
    _, proj = camera.headless(bb, 3840, 2160)
    s = _splatter(g, camera.orbit_view(0), proj, 3840, 2160, 16)
    yield g, proj, s
    s.close()


# ------------------------------------------------------------- readbacks
def test_readbacks_return_the_rendered_frame(built):
    """gs_read_projected / gs_read_bins reproduce the LAST RENDERED frame (its
    camera), not the current one; they never touch the framebuffer, the
    caller's BGR8 target, the stats or the histogram."""
    import torch

    from gaussian_splat_ipu_amd import camera, scene
    from oracle import oracle as O

    g, bb = scene.prepare_scene(scene.load_ply(PC12))
    W, H = 1280, 720
    view, proj = camera.headless(bb, W, H)
    s = _splatter(g, view, proj, W, H, 16)
    tgt = torch.zeros(s.bgr8_device()[1], dtype=torch.uint8, device="cuda")
    s.set_bgr8_target(tgt.data_ptr(), tgt.numel())
    s.execute()
    torch.cuda.synchronize()
    before_tgt = tgt.cpu().numpy().copy()
    bgr0, rgba0, hist0, st0 = s.get_frame_buffer(), s.get_rgba(), s.get_histogram(), s.stats()
    # move the camera; no frame rendered with it
    s.set_view_wire(camera.orbit_view(40))
    s.update_focal_lengths(camera.FOV_DEFAULT, 0.5)
    f = O.make_frame(view, proj, W, H, 16, 16, camera.FOV_DEFAULT, 1.0)
    p = O.project(g, f)
    gp = s.get_projected()
    live = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[:, 15] > 0
    _same_bits(gp[live, 0:2], p["mean2d"][live], "mean2d of the rendered frame")
    _same_bits(gp[live, 7], p["radius"][live], "radius of the rendered frame")
    ts, lst = s.get_bins()
    rts, rlst = O.bin_lists(p, f)
    np.testing.assert_array_equal(ts.astype(np.int64), rts)
    np.testing.assert_array_equal(lst, rlst)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tgt.cpu().numpy(), before_tgt)
    np.testing.assert_array_equal(s.get_frame_buffer(), bgr0)
    _same_bits(s.get_rgba(), rgba0, "RGBA after the readbacks")
    np.testing.assert_array_equal(s.get_histogram(), hist0)
    assert s.stats() == st0
    s.set_bgr8_target(None)
    s.close()


def test_overflow_is_sticky_across_async_frames(built):
    """A frame that overflows the pair capacity, followed by frames that do
    not, all enqueued with gs_render_async: gs_sync must still report
    GS_EOVERFLOW (the scan ORs every frame's overflow into a sticky word),
    and the next sync is clean."""
    from gaussian_splat_ipu_amd import _lib, camera, scene

    g, bb = scene.prepare_scene(scene.load_ply(PC12))
    W, H = 1280, 720
    view, proj = camera.headless(bb, W, H)
    s = _splatter(g, view, proj, W, H, 16, pair_capacity=2000)
    away = np.array(view, np.float32).reshape(16).copy()
    away[3] += 1000.0  # every mean far off-screen to the side: no pairs
    s.execute_async()          # overflows
    s.set_view_wire(away)
    s.execute_async()          # no pairs
    s.execute_async()
    with pytest.raises(_lib.GsError) as e:
        s.sync()
    assert e.value.status == _lib.GS_EOVERFLOW
    s.execute_async()
    s.sync()                   # clean: the sticky word was cleared
    assert s.stats()["n_pairs"] == 0
    s.close()


@pytest.mark.parametrize("chunk,pair_cull", [(256, True), (128, True), (256, False)])
def test_binning_more_than_256_chunks(built, test_hook, chunk, pair_cull):
    """Scenes beyond 256 binning chunks (~16.7 M Gaussians at 65535 per chunk)
    stay on the chunked binning: gs_colscan_kernel reads a wave's rows past
    its 16th twice.  The bin_chunk_size test hook shrinks the chunks so 120 k
    Gaussians make 469 / 938 of them; the frame and the lists stay bit-exact."""
    from gaussian_splat_ipu_amd import camera, scene
    from oracle import oracle as O

    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=120_000, seed=2, sh_degree=0)))
    view, proj = camera.headless(bb, 1920, 1080)
    test_hook("bin_chunk_size", chunk)
    s = _splatter(g, view, proj, 1920, 1080, 16, pair_cull=pair_cull)
    test_hook("bin_chunk_size", 0)
    assert s.stats()["bin_global"] == 0
    f = O.make_frame(view, proj, 1920, 1080, 16, 16, camera.FOV_DEFAULT, 1.0)
    ref = O.render(g, f)
    for _ in range(2):
        s.execute()
        _check_frame(s, g, f, ref)
    s.close()


@pytest.mark.parametrize("tw,th", [(32, 20), (16, 16)])
def test_ref_tile_major_readback(built, tw, th):
    """gs_read_rgba32f(GS_LAYOUT_REF_TILE_MAJOR): the IPU framebuffer layout
    (one tile's tw*th*4 floats after another, pixel (x, y) of a tile at
    (x + y*tw)*4, codelets.cpp:174-176) -- the oracle's row-major RGBA
    re-tiled must match bit for bit."""
    from gaussian_splat_ipu_amd import camera, scene
    from oracle import oracle as O

    g, bb = scene.prepare_scene(scene.load_ply(PC12))
    W, H = 1280, 720
    view, proj = camera.headless(bb, W, H)
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    s = GpuSplatter(g, TiledFramebuffer(W, H, tw, th), device=0)
    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, 0.1)
    s.execute()
    ref = O.render(g, O.make_frame(view, proj, W, H, tw, th, camera.FOV_DEFAULT, 0.1))["rgba"]
    tx, ty = -(-W // tw), -(-H // th)
    pad = np.zeros((ty * th, tx * tw, 4), np.float32)
    pad[:H, :W] = ref
    want = pad.reshape(ty, th, tx, tw, 4).transpose(0, 2, 1, 3, 4).reshape(-1)
    _same_bits(s.get_rgba(layout="ref_tile_major"), want, "tile-major RGBA")
    s.close()


# ------------------------------------------------------------- lazy big lists
@pytest.mark.parametrize("op_lo,op_hi", [(0.004, 0.02), (0.02, 0.3)])
def test_lazy_big_lists_continuation(built, op_lo, op_hi):
    """Big lists (> 2048 keys) of faint Gaussians: pixels outlive the sorted
    prefix of ~1.5 k keys, so their blend waves save their state and continue
    over the sorted window of the next keys (pass 1); waves that outlive the
    window too continue over the rest of the list, sorted in full (pass 2;
    gs_kernels.hip, lazy big lists).  The second frame of the renderer takes
    that path; the frame must equal the oracle's bit for bit.  op 0.004-0.02:
    nearly every big tile continues, and some pixels never saturate (pass 2);
    0.02-0.3: some do."""
    from gaussian_splat_ipu_amd import camera, scene
    from oracle import oracle as O

    src = scene.load_ply(PC12)
    centres = np.stack([src["x"], src["y"], src["z"]], 1)[::4]
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(
        n=600_000, seed=21, sh_degree=0, cluster_xyz=centres, cluster_sigma=0.02, opacity_lo=op_lo,
        opacity_hi=op_hi)))
    W, H = 1920, 1080
    view, proj = camera.headless(bb, W, H)
    s = _splatter(g, view, proj, W, H, 16, profile=True)
    f = O.make_frame(view, proj, W, H, 16, 16, camera.FOV_DEFAULT, 1.0)
    ref = O.render(g, f)
    s.execute()
    s.execute()  # with the big-list hint: lazy prefixes + continuation
    st = s.stats()
    assert st["n_big_tiles"] > 10
    assert st["cont_lists"] > 0
    if op_hi <= 0.02:
        assert st["cont_full_sorts"] > 0  # pixels that never saturate: pass 2 ran
    _check_frame(s, g, f, ref, lists=False)
    s.execute()  # the lists that continued are now sorted in full up front
    _check_frame(s, g, f, ref, lists=False)
    s.close()
