"""GPU parity of the row-band group (gs_group.hip, SURVEY §8 b/e): ONE C ABI
handle over several bands, each rendered by its own band renderer, the frame
assembled by one all-gather per frame inside gs_render.

On the one-GPU test box:
- num_gpus = 1 runs the real RCCL path (ncclCommInitAll over one device);
- gs_create_rank with world = 1 runs the one-process-per-GPU path
  (ncclCommInitRank from gs_comm_id_create);
- device_ids that repeat device 0 emulate 2..8 bands on one GPU: everything
  but the transport (device copies instead of RCCL) is the 8-GPU code --
  the split, its re-balancing from the gathered footers, the padded slots,
  the footers and the assembly.
Every frame is compared with the CPU oracle's full frame bit for bit (BGR8,
RGBA f32, histogram, per-tile lists)."""
import numpy as np
import pytest

from test_gpu_parity import assert_same_bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def synth(built):
    from gaussian_splat_ipu_amd import scene

    return scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=60_000, seed=11, sh_degree=0)))


@pytest.fixture(scope="module")
def clustered(built):
    """config 5's kind of scene (clustered around point_cloud_12's positions),
    small: dense rows move with the orbit camera."""
    from conftest import PC12
    from gaussian_splat_ipu_amd import scene

    src = scene.load_ply(PC12)
    centres = np.stack([src["x"], src["y"], src["z"]], 1)
    return scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=80_000, seed=8, sh_degree=0, cluster_xyz=centres,
                                                               cluster_sigma=0.02)))


def _oracle(g, view, proj, W, H, T, sd=1.0):
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    f = O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, sd)
    return f, O.render(g, f)


def _check(s, g, f, ref, lists=True):
    from oracle import oracle as O

    np.testing.assert_array_equal(s.get_frame_buffer(), ref["bgr"])
    np.testing.assert_array_equal(s.get_histogram(), ref["hist"])
    st = s.stats()
    assert st["n_pairs"] == ref["stats"]["n_pairs"]
    assert st["max_list"] == ref["stats"]["max_list"]
    if s.cfg.flags & 1 == 0:  # RGBA f32 kept
        assert_same_bits(s.get_rgba(), ref["rgba"], "RGBA f32 framebuffer")
    if lists:
        ts, lst = s.get_bins()
        rts, rlst = O.bin_lists(O.project(g, f), f)
        np.testing.assert_array_equal(ts.astype(np.int64), rts)
        np.testing.assert_array_equal(lst, rlst)


def _group(g, W, H, T, **kw):
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    return GpuSplatter(g, TiledFramebuffer(W, H, T, T), **kw)


def test_group_one_gpu_over_rccl(synth):
    """num_gpus = 1: ncclCommInitAll + one ncclAllGather per frame."""
    from gaussian_splat_ipu_amd import camera

    g, bb = synth
    W, H, T = 960, 540, 16
    view, proj = camera.headless(bb, W, H)
    f, ref = _oracle(g, view, proj, W, H, T)
    with _group(g, W, H, T, num_gpus=1, device_ids=[0]) as s:
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute()
        _check(s, g, f, ref)
        assert s.bands() == [(0, (H + T - 1) // T)]


def test_group_rank_world_one(synth):
    """gs_create_rank: the one-process-per-GPU path (bench.py under torchrun)."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import comm_id_create

    g, bb = synth
    W, H, T = 640, 360, 16
    view, proj = camera.headless(bb, W, H)
    f, ref = _oracle(g, view, proj, W, H, T)
    cid = comm_id_create()
    assert len(cid) == 128
    with _group(g, W, H, T, comm_id=cid, rank=0, world=1, device=0, frames_in_flight=2) as s:
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        for _ in range(3):
            s.execute()
        np.testing.assert_array_equal(s.get_frame_buffer(), ref["bgr"])
        np.testing.assert_array_equal(s.get_histogram(), ref["hist"])
        assert s.stats()["n_pairs"] == ref["stats"]["n_pairs"]


@pytest.mark.parametrize("G,F", [(2, 1), (3, 2), (8, 3)])
def test_emulated_bands_orbit_rebalance(clustered, G, F):
    """G bands on one GPU (copy transport), F frames in flight, orbit camera:
    every frame equals the oracle's whole frame, and the split moves with the
    camera (re-balanced from the gathered histograms)."""
    from gaussian_splat_ipu_amd import camera

    g, bb = clustered
    W, H, T = 960, 540, 16
    _, proj = camera.headless(bb, W, H)
    with _group(g, W, H, T, num_gpus=G, device_ids=[0] * G, frames_in_flight=F) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        splits = set()
        for k in (0, 20, 40, 40, 40, 40, 75):
            view = camera.orbit_view(k)
            s.set_view_wire(view)
            s.execute()
            splits.add(tuple(s.bands()))
            f, ref = _oracle(g, view, proj, W, H, T)
            _check(s, g, f, ref, lists=(k == 75))
        b = s.bands()
        assert b[0][0] == 0 and b[-1][1] == (H + T - 1) // T
        assert all(b0 < b1 for b0, b1 in b)
        assert len(splits) > 1  # the split followed the camera


def test_emulated_bands_direct_binning(clustered):
    """A group's band renderers bin a repeated view directly (round 6: the
    pairs go into the layout of the view's last scan; no scan or emit launch;
    the blend's last workgroup writes the footer's counters): the gathered
    frames, histograms and counts stay the oracle's."""
    from gaussian_splat_ipu_amd import camera

    g, bb = clustered
    W, H, T = 960, 540, 16
    view, proj = camera.headless(bb, W, H)
    f, ref = _oracle(g, view, proj, W, H, T)
    with _group(g, W, H, T, num_gpus=4, device_ids=[0] * 4, frames_in_flight=2, rebalance=False) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.set_view_wire(view)
        paths = []
        for _ in range(6):
            s.execute()
            paths.append(s.stats()["paths"])
            _check(s, g, f, ref, lists=False)
        assert not paths[0] & 128 and paths[-1] & 128, paths  # (GS_PATH_BIN_DIRECT)


def test_emulated_bands_async_pipeline(synth):
    """gs_render_async of several views, one sync: the last frame is the last
    view's frame (the pipeline keeps F frames in flight)."""
    from gaussian_splat_ipu_amd import camera

    g, bb = synth
    W, H, T = 640, 360, 16
    _, proj = camera.headless(bb, W, H)
    with _group(g, W, H, T, num_gpus=4, device_ids=[0, 0, 0, 0], frames_in_flight=3, write_rgba=False) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        for k in range(12):  # a blocking frame sizes the pair buffers for every view
            s.set_view_wire(camera.orbit_view(k * 10))
            s.execute()
        for k in range(12):
            s.set_view_wire(camera.orbit_view(k * 10))
            s.execute_async()
        s.sync()
        f, ref = _oracle(g, camera.orbit_view(110), proj, W, H, T)
        _check(s, g, f, ref, lists=False)


def test_emulated_bands_overflow_regrows(synth):
    """A pair capacity far too small: gs_render grows every band renderer's
    buffers and re-renders (all bands together), and the frame is exact."""
    from gaussian_splat_ipu_amd import camera

    g, bb = synth
    W, H, T = 640, 360, 16
    view, proj = camera.headless(bb, W, H)
    f, ref = _oracle(g, view, proj, W, H, T)
    with _group(g, W, H, T, num_gpus=3, device_ids=[0, 0, 0], frames_in_flight=2, pair_capacity=1024) as s:
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute()
        _check(s, g, f, ref)


def test_group_projected_and_tile_major(synth):
    """The debug readbacks of a group: projection records (input order) and the
    reference tile-major RGBA layout of the assembled frame."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = synth
    W, H, T = 640, 360, 16
    view, proj = camera.headless(bb, W, H)
    f, ref = _oracle(g, view, proj, W, H, T)
    with _group(g, W, H, T, num_gpus=2, device_ids=[0, 0]) as s:
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute()
        p = O.project(g, f)
        gp = s.get_projected()
        assert_same_bits(gp[:, 0:2], p["mean2d"], "mean2d")
        assert_same_bits(gp[:, 7], p["radius"], "radius")
        tm = s.get_rgba(layout="tile_major")
        fb_tiles = ((W + T - 1) // T) * ((H + T - 1) // T)
        want = np.zeros(fb_tiles * T * T * 4, np.float32)
        tx = (W + T - 1) // T
        for t in range(fb_tiles):
            y0, x0 = (t // tx) * T, (t % tx) * T
            blk = np.zeros((T, T, 4), np.float32)
            src = ref["rgba"][y0:y0 + T, x0:x0 + T]
            blk[: src.shape[0], : src.shape[1]] = src
            want[t * T * T * 4:(t + 1) * T * T * 4] = blk.reshape(-1)
        assert_same_bits(tm, want, "tile-major RGBA")


def _band_pairs(g, views, proj, W, H, T, bounds):
    """Reference pairs of every band (tile rows bounds[r]..bounds[r + 1]) for
    each view, from the oracle's lists (pair cull off: binned = reference)."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    tx = (W + T - 1) // T
    out = []
    for v in views:
        f = O.make_frame(v, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0)
        ts, _ = O.bin_lists(O.project(g, f), f)
        lens = np.diff(ts.astype(np.int64))
        out.append([int(lens[b0 * tx:b1 * tx].sum()) for b0, b1 in zip(bounds[:-1], bounds[1:])])
    return np.array(out)  # [view][band]


def _overflow_views(P, band):
    """(light view, heavy view, cap): at the heavy view only `band` exceeds
    cap; at the light view every band fits."""
    others = np.delete(P, band, axis=1).max(axis=1) if P.shape[1] > 1 else np.zeros(P.shape[0], np.int64)
    heavy = int(np.argmax(P[:, band] - others))
    light = int(np.argmin(P.max(axis=1)))
    cap = max(int(P[light].max()), int(others[heavy])) + 1
    assert cap < P[heavy, band], "no view sequence overflows just one band"
    return light, heavy, cap


def test_async_overflow_in_one_band_is_every_members(clustered):
    """only band 1 of 3 overflows, in frame 1 of 3 in-flight
    frames (the last frame fits everywhere).  The status comes from the
    gathered footers (band 1's sticky word rides in the last frame's footer),
    so gs_sync reports GS_EOVERFLOW for the group; a repeated gs_sync without a
    new frame reports the same; then one blocking gs_render of the heavy view
    regrows every band renderer and matches the oracle."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd._lib import GS_EOVERFLOW, GsError

    g, bb = clustered
    W, H, T, G = 960, 540, 16, 3
    _, proj = camera.headless(bb, W, H)
    views = [camera.orbit_view(k) for k in range(0, 120, 8)]
    with _group(g, W, H, T, num_gpus=G, device_ids=[0] * G, frames_in_flight=3, rebalance=False,
                pair_cull=False, pair_capacity=1 << 26) as probe:
        bounds = [b0 for b0, _ in probe.bands()] + [probe.bands()[-1][1]]
    P = _band_pairs(g, views, proj, W, H, T, bounds)
    light, heavy, cap = _overflow_views(P, 1)
    with _group(g, W, H, T, num_gpus=G, device_ids=[0] * G, frames_in_flight=3, rebalance=False,
                pair_cull=False, pair_capacity=cap) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        for v in (light, heavy, light):
            s.set_view_wire(views[v])
            s.execute_async()
        with pytest.raises(GsError) as ei:
            s.sync()
        assert ei.value.status == GS_EOVERFLOW
        with pytest.raises(GsError) as ei:  # the same frame's decision again
            s.sync()
        assert ei.value.status == GS_EOVERFLOW
        assert s.stats()["n_pairs"] == int(P[light].sum())  # the last frame is the light view's
        s.set_view_wire(views[heavy])
        s.execute()  # grows and renders again on every band
        assert s.stats()["pair_capacity"] >= P[heavy].max()
        f, ref = _oracle(g, views[heavy], proj, W, H, T)
        _check(s, g, f, ref, lists=False)
        # and the pipeline is clean afterwards
        for v in (light, heavy, light):
            s.set_view_wire(views[v])
            s.execute_async()
        s.sync()


def test_rank_world_one_async_overflow_sticky(clustered):
    """The one-process-per-GPU path (RCCL world 1): the sticky word reaches the
    footer by the copy on the communication stream before the ncclAllGather."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd._lib import GS_EOVERFLOW, GsError
    from gaussian_splat_ipu_amd.splatter import comm_id_create

    g, bb = clustered
    W, H, T = 960, 540, 16
    _, proj = camera.headless(bb, W, H)
    views = [camera.orbit_view(k) for k in range(0, 120, 8)]
    P = _band_pairs(g, views, proj, W, H, T, [0, (H + T - 1) // T])
    light, heavy, cap = _overflow_views(P, 0)
    with _group(g, W, H, T, comm_id=comm_id_create(), rank=0, world=1, device=0, frames_in_flight=3,
                pair_cull=False, pair_capacity=cap) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        for v in (light, heavy, light):
            s.set_view_wire(views[v])
            s.execute_async()
        with pytest.raises(GsError) as ei:
            s.sync()
        assert ei.value.status == GS_EOVERFLOW
        s.set_view_wire(views[light])
        s.execute()  # the sticky word was cleared by the sync: this frame fits
        f, ref = _oracle(g, views[light], proj, W, H, T)
        np.testing.assert_array_equal(s.get_frame_buffer(), ref["bgr"])
        s.set_view_wire(views[heavy])
        s.execute()
        f, ref = _oracle(g, views[heavy], proj, W, H, T)
        np.testing.assert_array_equal(s.get_frame_buffer(), ref["bgr"])
        assert s.stats()["n_pairs"] == ref["stats"]["n_pairs"]


def test_readback_on_one_member_keeps_the_split(synth):
    """A readback (local call) between frames neither re-balances nor clears
    the overflow state: the split only moves inside collective calls."""
    from gaussian_splat_ipu_amd import camera

    g, bb = synth
    W, H, T = 640, 360, 16
    view, proj = camera.headless(bb, W, H)
    with _group(g, W, H, T, num_gpus=4, device_ids=[0] * 4, frames_in_flight=2) as s:
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute_async()
        b0 = s.bands()
        s.get_frame_buffer()  # local: waits, reads, changes nothing
        s.get_histogram()
        s.execute_async()
        assert s.bands() == b0  # (the first re-balancing point is frame 8)
        s.sync()
        s.execute()  # collective: re-balances from its own frame
        f, ref = _oracle(g, view, proj, W, H, T)
        _check(s, g, f, ref, lists=False)
