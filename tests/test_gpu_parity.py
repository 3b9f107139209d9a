"""GPU parity: the HIP frame path (through the C ABI) against the CPU oracle.

Bar: projection records, tile binning (per-tile depth-sorted
Gaussian indices) and the tile histogram are compared bit-exactly; the RGBA f32
framebuffer is asserted bit-identical as well (tolerance 0 -- the kernels and
the oracle implement the same IEEE op sequence, -ffp-contract=off, the same
specified expf), and the BGR8 frame exactly.
"""
import numpy as np
import pytest

from conftest import PC12

pytestmark = pytest.mark.gpu


def assert_same_bits(a, b, what=""):
    """Bit-exact float comparison, except that all NaNs compare equal (the NaN
    sign/payload an operation produces differs between x86 -- default NaN
    0xFFC00000 -- and gfx950 -- 0x7FC00000 -- and is not a value)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    if not same.all():
        bad = np.argwhere(~same)
        raise AssertionError(
            f"{what}: {len(bad)} of {a.size} values differ; first {bad[:4].tolist()}: "
            f"{a[tuple(bad[0])]} vs {b[tuple(bad[0])]}"
        )


def _frame_pair(g, view, proj, W, H, TW, TH, scale_div, fov=None, guard_tile=None, band=None, band_count=1,
                band_index=0, pair_capacity=0, bin_global=False, input_order=False):
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    fov = camera.FOV_DEFAULT if fov is None else fov
    fb = TiledFramebuffer(W, H, TW, TH)
    s = GpuSplatter(g, fb, device=0, guard_tile=guard_tile, band_index=band_index, band_count=band_count,
                    pair_capacity=pair_capacity, bin_global=bin_global, input_order=input_order)
    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(fov, scale_div)
    s.execute()
    if band_count > 1:
        ty0, ty1, _, _ = fb.band_rows(band_count)[band_index]
        band = (ty0, ty1) if ty1 > ty0 else None
    f = O.make_frame(view, proj, W, H, TW, TH, fov, scale_div, guard_tile=guard_tile, band=band)
    return s, f


def _assert_parity(s, f, g, check_proj=True, band_culled=False):
    from oracle import oracle as O

    ref = O.render(g, f)
    st = s.stats()
    if band_culled:  # (gsplat.h: a band-culled renderer's n_rendered counts only the Gaussians it projected)
        assert st["n_rendered"] <= ref["stats"]["n_rendered"]
    else:
        assert st["n_rendered"] == ref["stats"]["n_rendered"]
    assert st["n_pairs"] == ref["stats"]["n_pairs"]
    assert st["max_list"] == ref["stats"]["max_list"]
    if check_proj and g.shape[0]:
        p = O.project(g, f)
        gp = s.get_projected()
        live = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[:, 15] > 0
        assert_same_bits(gp[live, 0:2], p["mean2d"][live], "mean2d")
        assert_same_bits(gp[live, 2:6], p["conic"][live], "conic")
        assert_same_bits(gp[live, 6], p["clip_z"][live], "clip z")
        assert_same_bits(gp[live, 7], p["radius"][live], "radius")
        r = p["rect"]
        ok = (p["rendered"] != 0) & (r[:, 0] <= r[:, 2])
        grect = gp[:, 8:12].astype(np.int64)
        gok = grect[:, 0] <= grect[:, 2]
        np.testing.assert_array_equal(gok, ok)
        np.testing.assert_array_equal(grect[ok], r[ok])
    ts, lst = s.get_bins()
    rts, rlst = O.bin_lists(O.project(g, f), f)
    np.testing.assert_array_equal(ts.astype(np.int64), rts)
    np.testing.assert_array_equal(lst, rlst)
    np.testing.assert_array_equal(s.get_histogram(), ref["hist"])
    assert_same_bits(s.get_rgba(), ref["rgba"], "RGBA f32 framebuffer")
    np.testing.assert_array_equal(s.get_frame_buffer(), ref["bgr"])
    return ref


@pytest.fixture(scope="module")
def pc12(built):
    from gaussian_splat_ipu_amd import scene

    g, bb = scene.prepare_scene(scene.load_ply(PC12))
    return g, bb


@pytest.mark.parametrize("scale_div", [0.1, 1.0])
def test_pc12_reference_geometry_720p(pc12, scale_div):
    """config 2 at the reference's own build geometry: 1280x720, 32x20 tiles."""
    from gaussian_splat_ipu_amd import camera

    g, bb = pc12
    view, proj = camera.headless(bb, 1280, 720)
    s, f = _frame_pair(g, view, proj, 1280, 720, 32, 20, scale_div)
    ref = _assert_parity(s, f, g)
    assert ref["stats"]["n_pairs"] > 50000


@pytest.mark.parametrize("tw,th,bin_global,input_order", [
    (16, 16, False, False), (16, 16, True, False), (16, 16, False, True), (48, 30, False, False),
    (32, 20, False, False)])
def test_pc12_1080p(pc12, tw, th, bin_global, input_order):
    """config 2: point_cloud_12 at 1920x1080 (16x16 production tiles, 48x30 =
    the reference macros at 1080p, 32x20); 1080/16 leaves a partial tile row.
    Both binning paths (chunked LDS histograms, global atomics), and both
    device orders of the Gaussians (Morton, input)."""
    from gaussian_splat_ipu_amd import camera

    g, bb = pc12
    view, proj = camera.headless(bb, 1920, 1080)
    s, f = _frame_pair(g, view, proj, 1920, 1080, tw, th, 1.0, bin_global=bin_global,
                       input_order=input_order)
    _assert_parity(s, f, g)


def test_synthetic_1080p_16x16(built):
    from gaussian_splat_ipu_amd import camera, scene

    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=200_000, seed=1, sh_degree=3)))
    view, proj = camera.headless(bb, 1920, 1080)
    s, f = _frame_pair(g, view, proj, 1920, 1080, 16, 16, 1.0)
    _assert_parity(s, f, g)


@pytest.mark.parametrize("band", [None, 0, 1])
def test_large_tile_lists_take_the_radix_path(built, band):
    """A clustered scene (config 5's construction) puts > 2048 Gaussians on
    some tiles: those go through the block-wide LSD radix sort, first inside
    the tile-sort launch (a whole frame) or inside the blend's workgroups
    (band 0 / 1 of two: the in-blend sort), then (second frame) in the
    separate big-list launches (lazy prefixes, the continuation)."""
    from gaussian_splat_ipu_amd import camera, scene

    src = scene.load_ply(PC12)
    cl = np.stack([src["x"], src["y"], src["z"]], 1)[:200]
    ply = scene.synthetic(scene.SynthSpec(n=150_000, seed=8, sh_degree=0, cluster_xyz=cl, cluster_sigma=0.02))
    g, bb = scene.prepare_scene(ply)
    view, proj = camera.headless(bb, 1280, 720)
    if band is None:
        s, f = _frame_pair(g, view, proj, 1280, 720, 16, 16, 1.0)
    else:
        s, f = _frame_pair(g, view, proj, 1280, 720, 16, 16, 1.0, band_count=2, band_index=band)
        assert s.stats()["paths"] & 2  # (GS_PATH_BLEND_SORT)
    _assert_parity(s, f, g)
    assert s.stats()["n_big_tiles"] > 0
    # the next frame sees big lists in the last completed frame's counters and
    # sorts them in their own launches (lazy prefixes, 16x16 tiles)
    s.execute()
    assert s.stats()["paths"] & 16  # (GS_PATH_BIG_LISTS)
    _assert_parity(s, f, g)


@pytest.mark.parametrize("band_count", [3, 8])
def test_interleaved_bands_equal_full_frame_rows(pc12, band_count):
    """GS_FLAG_BAND_INTERLEAVED (the multi-GPU default in bench.py): band b
    renders tile rows b, b + band_count, ...  Its RGBA, BGR8 and per-tile list
    lengths equal those rows of the single-renderer frame (itself checked
    against the oracle), and the all-gather layout assembles back to it."""
    from gaussian_splat_ipu_amd import camera, dist as gdist
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    g, bb = pc12
    W, H, TW, TH = 1920, 1080, 16, 16
    view, proj = camera.headless(bb, W, H)
    full, f = _frame_pair(g, view, proj, W, H, TW, TH, 1.0)
    _assert_parity(full, f, g, check_proj=False)
    fb = TiledFramebuffer(W, H, TW, TH)
    rgba, bgr = full.get_rgba(), full.get_frame_buffer()
    hist = full.get_histogram().reshape(fb.tiles_down, fb.tiles_across)
    gathered = []
    for b in range(band_count):
        s = GpuSplatter(g, fb, device=0, band_index=b, band_count=band_count, band_interleaved=True)
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute()
        rows = fb.interleaved_tile_rows(band_count, b)
        assert s.stats()["band_stride"] == band_count
        assert_same_bits(s.get_rgba(), gdist.extract_band(rgba, fb, band_count, b, True), f"band {b} rgba")
        band_bgr = s.get_frame_buffer()
        np.testing.assert_array_equal(band_bgr, gdist.extract_band(bgr, fb, band_count, b, True))
        np.testing.assert_array_equal(s.get_histogram(), hist[rows].reshape(-1))
        gathered.append(gdist.pad_band(band_bgr, fb, band_count))
        s.close()
    np.testing.assert_array_equal(gdist.assemble(np.stack(gathered), fb, band_count, interleaved=True), bgr)


@pytest.mark.parametrize("band_count", [2, 8])
def test_balanced_explicit_bands_equal_full_frame(pc12, band_count):
    """Work-balanced contiguous bands (gs_config.band_row_begin/end, ABI 4;
    dist.balanced_bands over the full frame's histogram) with the band cull:
    each band equals its rows of the full frame (itself checked against the
    oracle), and the padded all-gather layout assembles back to it."""
    from gaussian_splat_ipu_amd import camera, dist as gdist
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    g, bb = pc12
    W, H, TW, TH = 1920, 1080, 16, 16
    view, proj = camera.headless(bb, W, H)
    full, f = _frame_pair(g, view, proj, W, H, TW, TH, 1.0)
    _assert_parity(full, f, g, check_proj=False)
    fb = TiledFramebuffer(W, H, TW, TH)
    rgba, bgr = full.get_rgba(), full.get_frame_buffer()
    hist = full.get_histogram().reshape(fb.tiles_down, fb.tiles_across)
    bands = gdist.balanced_bands(gdist.row_work(hist, fb), band_count)
    pad = max(t1 - t0 for t0, t1 in bands)
    gathered = []
    for t0, t1 in bands:
        s = GpuSplatter(g, fb, device=0, band_rows=(t0, t1), band_pad_rows=pad, band_cull=True)
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute()
        y0, y1 = t0 * TH, min(H, t1 * TH)
        assert_same_bits(s.get_rgba(), rgba[y0:y1], f"band {t0}-{t1} rgba")
        band_bgr = s.get_frame_buffer()
        np.testing.assert_array_equal(band_bgr, bgr[y0:y1])
        np.testing.assert_array_equal(s.get_histogram(), hist[t0:t1].reshape(-1))
        dev = np.zeros((pad * TH, W, 3), np.uint8)
        dev[: y1 - y0] = band_bgr
        gathered.append(dev)
        s.close()
    np.testing.assert_array_equal(gdist.assemble_bands(np.stack(gathered), fb, bands), bgr)


@pytest.mark.parametrize("band_count", [2, 3, 8])
def test_row_bands_union_equals_full_frame(pc12, band_count):
    """The multi-GPU decomposition: each band renders its tile rows; every band
    matches the oracle restricted to that band, and stacking the bands gives the
    single-renderer frame."""
    from gaussian_splat_ipu_amd import camera

    g, bb = pc12
    W, H, TW, TH = 1920, 1080, 16, 16
    view, proj = camera.headless(bb, W, H)
    full, _ = _frame_pair(g, view, proj, W, H, TW, TH, 1.0)
    whole = full.get_rgba()
    parts = []
    for b in range(band_count):
        s, f = _frame_pair(g, view, proj, W, H, TW, TH, 1.0, band_count=band_count, band_index=b)
        if s.band_rows == 0:
            continue
        _assert_parity(s, f, g, check_proj=False)
        parts.append(s.get_rgba())
    assert_same_bits(np.concatenate(parts, 0), whole, "stacked bands")


def test_edge_cases(built):
    """Empty scene, empty slots (gid <= 0), Gaussians behind the camera,
    degenerate covariance (det == 0), huge Gaussians beyond the guard band,
    non-finite inputs and off-screen means."""
    from gaussian_splat_ipu_amd import camera, scene

    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=5000, seed=3, sh_degree=0)))
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16).copy()
    a[0:50, 15] = 0.0  # empty slots
    a[50:100, 15] = -3.0
    a[100:150, 0:3] = [0.0, 0.0, 40.0]  # behind the camera (world z +40 maps behind)
    a[150:200, 12:15] = 30.0  # huge (guard band drops them)
    a[200:250, 8:12] = 0.0  # zero quaternion -> normalize() returns identity
    a[250:300, 12:15] = -200.0  # scale -> exp underflow (det == 0 path)
    a[300:310, 0] = np.nan
    a[310:320, 0] = np.inf
    a[320:370, 0] = 30.0  # far off-screen
    a[370:400, 4:7] = -1.0  # negative colour
    view, proj = camera.headless(bb, 800, 600)
    for tw, th in [(16, 16), (32, 20)]:
        s, f = _frame_pair(a, view, proj, 800, 600, tw, th, 1.0)
        _assert_parity(s, f, a)
    # empty scene
    s, f = _frame_pair(a[:0], view, proj, 800, 600, 16, 16, 1.0)
    assert s.stats()["n_pairs"] == 0
    assert not s.get_frame_buffer().any()


def _band_render(g, view, proj, fb, scale_div, band_index, band_count, interleaved, cull):
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter

    s = GpuSplatter(g, fb, device=0, band_index=band_index, band_count=band_count,
                    band_interleaved=interleaved, band_cull=cull)
    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, scale_div)
    s.execute()
    return s


def test_pair_cull_changes_nothing(pc12):
    """By default a Gaussian is binned only into the tiles its alpha >= 1/255
    box meets.  Frame, RGBA, histogram, reference lists (gs_read_bins re-bins
    them) and pair count must equal GS_FLAG_NO_PAIR_CULL's, on point_cloud_12
    (reference geometry and 1080p), the edge-case scene and interleaved bands;
    and the culled frames must bin fewer pairs."""
    from gaussian_splat_ipu_amd import camera, scene
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    ge, bbe = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=5000, seed=3, sh_degree=0)))
    a = np.ascontiguousarray(ge).view(np.float32).reshape(-1, 16).copy()
    a[50:100, 15] = -3.0
    a[100:150, 0:3] = [0.0, 0.0, 40.0]
    a[150:200, 12:15] = 30.0
    a[250:300, 12:15] = -200.0
    a[300:310, 0] = np.nan
    a[310:320, 0] = np.inf
    a[320:370, 7] = 1.0 / 255.0  # opacities at the cut
    a[370:420, 7] = 0.5 / 255.0
    g, bb = pc12
    cases = [(g, bb, 1920, 1080, 16, 16, 1.0, 1, 0), (g, bb, 1280, 720, 32, 20, 0.1, 1, 0),
             (g, bb, 1280, 720, 16, 16, 1.0, 3, 1), (a, bbe, 800, 600, 16, 16, 1.0, 1, 0)]
    for scn, box, W, H, TW, TH, sd, bc, bi in cases:
        view, proj = camera.headless(box, W, H)
        fb = TiledFramebuffer(W, H, TW, TH)
        out = []
        for pc in (True, False):
            s = GpuSplatter(scn, fb, device=0, band_index=bi, band_count=bc, band_interleaved=bc > 1,
                            pair_cull=pc)
            s.set_view_wire(view)
            s.set_projection_wire(proj)
            s.update_focal_lengths(camera.FOV_DEFAULT, sd)
            s.execute()
            st = s.stats()
            out.append((s.get_rgba(), s.get_frame_buffer(), s.get_histogram(), st, s.get_bins()))
            s.close()
        (r1, b1, h1, s1, (t1, l1)), (r2, b2, h2, s2, (t2, l2)) = out
        assert_same_bits(r1, r2, f"{W}x{H} rgba")
        np.testing.assert_array_equal(b1, b2)
        np.testing.assert_array_equal(h1, h2)
        np.testing.assert_array_equal(t1, t2)
        np.testing.assert_array_equal(l1, l2)
        assert s1["n_pairs"] == s2["n_pairs"] == s2["n_pairs_binned"]
        assert s1["max_list"] == s2["max_list"]
        assert s1["n_pairs_binned"] < s1["n_pairs"]


@pytest.mark.parametrize("interleaved", [False, True])
def test_band_cull_changes_nothing(pc12, interleaved):
    """GS_FLAG_BAND_CULL skips the projection of Gaussians whose conservative
    extent misses the band.  Every band's frame, RGBA, lists and histogram must
    equal the unculled band's, on point_cloud_12 and on the edge-case scene
    (non-finite, behind-camera, huge, degenerate Gaussians); the projection
    readback must still cover every Gaussian."""
    from gaussian_splat_ipu_amd import camera, scene
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    ge, bbe = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=5000, seed=3, sh_degree=0)))
    a = np.ascontiguousarray(ge).view(np.float32).reshape(-1, 16).copy()
    a[50:100, 15] = -3.0
    a[100:150, 0:3] = [0.0, 0.0, 40.0]
    a[150:200, 12:15] = 30.0
    a[250:300, 12:15] = -200.0
    a[300:310, 0] = np.nan
    a[310:320, 0] = np.inf
    a[320:370, 0] = 30.0
    g, bb = pc12
    for scn, box, W, H, sd in [(g, bb, 1920, 1080, 1.0), (g, bb, 1280, 720, 0.1), (a, bbe, 800, 600, 1.0)]:
        view, proj = camera.headless(box, W, H)
        fb = TiledFramebuffer(W, H, 16, 16)
        culled_any = False
        for bc in (3, 8):
            for bi in range(bc):
                ref = _band_render(scn, view, proj, fb, sd, bi, bc, interleaved, False)
                cul = _band_render(scn, view, proj, fb, sd, bi, bc, interleaved, True)
                assert_same_bits(cul.get_rgba(), ref.get_rgba(), f"band {bi}/{bc} rgba")
                np.testing.assert_array_equal(cul.get_frame_buffer(), ref.get_frame_buffer())
                np.testing.assert_array_equal(cul.get_histogram(), ref.get_histogram())
                t1, l1 = cul.get_bins()
                t2, l2 = ref.get_bins()
                np.testing.assert_array_equal(t1, t2)
                np.testing.assert_array_equal(l1, l2)
                assert cul.stats()["n_pairs"] == ref.stats()["n_pairs"]
                assert cul.stats()["n_rendered"] <= ref.stats()["n_rendered"]
                culled_any |= cul.stats()["n_rendered"] < ref.stats()["n_rendered"]
                if bi == 0:
                    assert_same_bits(cul.get_projected(), ref.get_projected(), "projection readback")
                cul.close()
                ref.close()
        assert culled_any


@pytest.mark.parametrize("tw,th", [(16, 16), (32, 20)])
def test_blend_culling_is_decision_preserving(built, tw, th):
    """Stress the blend's footprint culling (pcut + wave boxes): strongly
    anisotropic Gaussians and opacities around the 1/255 threshold, negative,
    tiny and huge.  The frame must stay bit-identical to the oracle, which
    evaluates every list entry."""
    from gaussian_splat_ipu_amd import camera, scene

    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=30000, seed=11, sh_degree=0, log_scale_mu=-4.0)))
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16).copy()
    rng = np.random.default_rng(5)
    n = a.shape[0]
    # anisotropy: one axis up to e^4 larger
    a[:, 12] += rng.uniform(0.0, 4.0, n).astype(np.float32)
    ops = np.array([-3.0, 0.0, 1 / 255 - 1e-6, 1 / 255, 1 / 255 + 1e-6, 0.004, 0.01, 0.3, 1.0, 8.0, 50.0, 1e6],
                   np.float32)
    a[:, 7] = ops[rng.integers(0, ops.size, n)]
    view, proj = camera.headless(bb, 1280, 720)
    s, f = _frame_pair(a, view, proj, 1280, 720, tw, th, 1.0)
    _assert_parity(s, f, a)


def test_gpu_against_committed_golden(built):
    """The HIP path against the committed fixtures (tests/golden/oracle_golden.npz,
    tools/make_golden.py): frame digests, histogram, list offsets and digests,
    an RGBA crop and the first 256 projection records, bit for bit."""
    from tools_golden import CASES, GOLDEN_PATH, gpu_case

    gold = np.load(GOLDEN_PATH, allow_pickle=False)
    for name in CASES:
        got = gpu_case(name)
        for key, val in got.items():
            want = gold[f"{name}/{key}"]
            if val.dtype == np.float32:
                assert_same_bits(val, want, f"{name}/{key}")
            else:
                np.testing.assert_array_equal(val, want, err_msg=f"{name}/{key}")


def test_overflow_grows_capacity(pc12):
    from gaussian_splat_ipu_amd import camera

    g, bb = pc12
    view, proj = camera.headless(bb, 1280, 720)
    s, f = _frame_pair(g, view, proj, 1280, 720, 16, 16, 1.0, pair_capacity=1000)
    assert s.stats()["pair_capacity"] >= s.stats()["n_pairs_binned"] > 1000
    _assert_parity(s, f, g, check_proj=False)


def test_repeatable_and_async(pc12):
    """Same inputs twice -> identical frames (no atomics-order dependence);
    execute_async + sync gives the same frame."""
    from gaussian_splat_ipu_amd import camera

    g, bb = pc12
    view, proj = camera.headless(bb, 1920, 1080)
    s, _ = _frame_pair(g, view, proj, 1920, 1080, 16, 16, 1.0)
    a = s.get_rgba().copy()
    ts1, l1 = s.get_bins()
    s.execute_async()
    s.sync()
    assert_same_bits(s.get_rgba(), a, "async frame")
    ts2, l2 = s.get_bins()
    np.testing.assert_array_equal(l1, l2)


def test_orbit_frames(pc12):
    """config 5's orbit camera on a few frames (view changes per frame)."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = pc12
    _, proj = camera.headless(bb, 1280, 720)
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    s = GpuSplatter(g, TiledFramebuffer(1280, 720, 16, 16), device=0)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
    for k in (0, 17, 45, 90):
        view = camera.orbit_view(k)
        s.set_view_wire(view)
        s.execute()
        f = O.make_frame(view, proj, 1280, 720, 16, 16, camera.FOV_DEFAULT, 1.0)
        ref = O.render(g, f)
        assert_same_bits(s.get_rgba(), ref["rgba"], f"orbit frame {k}")


@pytest.mark.parametrize("cov_cache", [-1, 0])
def test_focal_changes_between_frames(pc12, test_hook, cov_cache):
    """One renderer, fxy[1] changed between frames: the projection's cached
    3D covariances (computed once per fxy[1]) follow it, frame for frame
    against the oracle, including a frame in flight when it changes.
    cov_cache = 0: no cache (the path a failed cache allocation takes: the
    covariances from the rotation and the scales every frame), a whole frame
    and a row band."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    if cov_cache == 0:
        test_hook("cov_cache", 0)
        g, bb = pc12
        view, proj = camera.headless(bb, 1920, 1080)
        for band_count, band_index in [(1, 0), (8, 3)]:
            s, f = _frame_pair(g, view, proj, 1920, 1080, 16, 16, 0.1, band_count=band_count,
                               band_index=band_index)
            _assert_parity(s, f, g, check_proj=band_count == 1)
            s.close()
    g, bb = pc12
    view, proj = camera.headless(bb, 1280, 720)
    s = GpuSplatter(g, TiledFramebuffer(1280, 720, 16, 16), device=0)
    s.set_view_wire(view)
    s.set_projection_wire(proj)

    def check(sd):
        ref = O.render(g, O.make_frame(view, proj, 1280, 720, 16, 16, camera.FOV_DEFAULT, sd))
        assert_same_bits(s.get_rgba(), ref["rgba"], f"fxy[1] = {sd}")

    for sd in (1.0, 0.1, 0.1, 0.5):
        s.update_focal_lengths(camera.FOV_DEFAULT, sd)
        s.execute()
        check(sd)
    # a change with the previous frame still in flight on the renderer's stream
    s.update_focal_lengths(camera.FOV_DEFAULT, 0.1)
    s.execute_async()
    s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
    s.execute_async()
    s.sync()
    check(1.0)


def test_render_server_cli(built, tmp_path):
    """The headless render server on the C ABI: same flow and
    log line as splat.cpp; its test.png equals the renderer's BGR8 frame."""
    import os
    import struct
    import subprocess
    import zlib

    from conftest import ROOT

    exe = os.path.join(ROOT, "gaussian_splat_ipu_amd", "bin", "splat")
    out = tmp_path / "test.png"
    r = subprocess.run([exe, "--input", PC12, "--device", "gpu", "--out", str(out), "--frames", "2"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Splat time:" in r.stdout and "points/sec:" in r.stdout
    data = out.read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    w, h = struct.unpack(">II", data[16:24])
    assert (w, h) == (1280, 720)
    idat = data[data.index(b"IDAT") + 4:data.index(b"IEND") - 8]
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * 3)[:, 1:].reshape(h, w, 3)
    from gaussian_splat_ipu_amd import camera, scene
    from oracle import oracle as O

    g, bb = scene.prepare_scene(scene.load_ply(PC12))
    view, proj = camera.headless(bb, 1280, 720)
    ref = O.render(g, O.make_frame(view, proj, 1280, 720, 32, 20, camera.FOV_DEFAULT, 0.1))
    np.testing.assert_array_equal(raw[:, :, ::-1], ref["bgr"])
    # the same frame through a row-band group (--gpus 1: gs_create with
    # num_gpus, one RCCL all-gather per frame inside gs_render)
    out2 = tmp_path / "test2.png"
    r = subprocess.run([exe, "--input", PC12, "--device", "gpu", "--gpus", "1", "--out", str(out2)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert out2.read_bytes() == data


@pytest.mark.parametrize("band", [None, 0, 1])
@pytest.mark.parametrize("half_width,log_scale,planes", [
    (1.5, -3.8, 4), (0.3, -4.0, 4), (1.5, -3.8, 64), (0.3, -4.0, 400), (0.3, -4.0, 1)])
def test_equal_depths_keep_input_order(built, half_width, log_scale, planes, band):
    """Gaussians on planes of constant clip z (a view that only translates
    along z), in shuffled input order: the tile lists hold runs of equal
    depth, whose order must be the input index's (the oracle's stable order),
    not the device (Morton) order the pair keys carry.  half_width 1.5 gives
    small lists; 0.3 small, medium and > 2048-key lists (radix sort on the
    first frame, the big-list sample sort on the second).  4 planes make long
    runs (the list is re-sorted), 64 / 400 planes mostly short ones (put in
    order in place); one plane gives big lists of a single depth (one
    sample-sort bucket > 2048 keys: its radix path).  A whole frame (the
    sort launch, two-pixel blend lanes) and the two bands of a 2-way split
    (the tile sort inside the blend's workgroups)."""
    from gaussian_splat_ipu_amd import camera, scene
    from oracle import oracle as O

    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=20000, seed=5, sh_degree=0)))
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16).copy()
    rng = np.random.default_rng(11)
    n = a.shape[0]
    a[:, 0] = rng.uniform(-half_width, half_width, n)
    a[:, 1] = rng.uniform(-half_width, half_width, n)
    a[:, 2] = rng.choice(np.linspace(0.0, 1.5, planes, dtype=np.float32), n)
    a[:, 3] = 1.0
    a[:, 7] = rng.uniform(0.02, 0.3, n)  # low opacities: many records per pixel contribute
    a[:, 12:15] = log_scale + rng.normal(0.0, 0.2, (n, 3))
    _, proj = camera.headless(bb, 1280, 720)
    view = np.float32([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -4.0, 0, 0, 0, 1])
    if band is None:
        s, f = _frame_pair(a, view, proj, 1280, 720, 16, 16, 1.0)
        f_all = f
    else:
        s, f = _frame_pair(a, view, proj, 1280, 720, 16, 16, 1.0, band_count=2, band_index=band)
        f_all = O.make_frame(view, proj, 1280, 720, 16, 16, camera.FOV_DEFAULT, 1.0)
    ref = _assert_parity(s, f, a)
    # the lists really hold equal depths next to each other
    p = O.project(a, f_all)
    ts, lst = O.bin_lists(p, f_all)
    z = p["clip_z"][lst]
    same = (z[1:] == z[:-1]) & (np.diff(np.searchsorted(ts, np.arange(len(lst)), side="right")) == 0)
    assert same.sum() > 500
    if half_width < 1.0 and s.stats()["n_big_tiles"] > 0:
        s.execute()  # big lists through the big-list sample sort
        _assert_parity(s, f, a)
    assert ref["stats"]["n_pairs"] > 0


def test_set_band_rows_moves_one_renderer(pc12):
    """gs_set_band_rows: one renderer created for the whole frame is moved over
    a balanced 3-band split (async frames in flight between the moves, as a
    group member is); each band equals the full frame's rows bit for bit."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd import dist as gdist
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    g, bb = pc12
    W, H, TW, TH = 1920, 1080, 16, 16
    view, proj = camera.headless(bb, W, H)
    full, f = _frame_pair(g, view, proj, W, H, TW, TH, 1.0)
    fb = TiledFramebuffer(W, H, TW, TH)
    rgba, bgr = full.get_rgba(), full.get_frame_buffer()
    hist = full.get_histogram().reshape(fb.tiles_down, fb.tiles_across)
    bands = gdist.balanced_bands(gdist.row_work(hist, fb), 3)
    with GpuSplatter(g, fb, device=0, band_rows=(0, fb.tiles_down), band_cull=True) as s:
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute()
        for t0, t1 in bands + bands[::-1]:
            s.execute_async()  # a frame of the previous rows still in flight
            s.set_band_rows(t0, t1)
            s.execute()
            y0, y1 = t0 * TH, min(H, t1 * TH)
            assert_same_bits(s.get_rgba(), rgba[y0:y1], f"moved band {t0}-{t1} rgba")
            np.testing.assert_array_equal(s.get_frame_buffer(), bgr[y0:y1])
            np.testing.assert_array_equal(s.get_histogram(), hist[t0:t1].reshape(-1))
        with pytest.raises(Exception):
            s.set_band_rows(0, fb.tiles_down + 1)


def test_set_band_rows_keeps_the_in_flight_frame(pc12):
    """gs_set_band_rows does not wait for the frame in flight: that frame keeps
    its rows, its pair overflow still reaches the next gs_sync (sticky), and
    its readbacks are refused after the move (they would read it with the new
    band's geometry) until the next frame renders."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd._lib import GsError
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    g, bb = pc12
    W, H, TW, TH = 1920, 1080, 16, 16
    view, proj = camera.headless(bb, W, H)
    full, f = _frame_pair(g, view, proj, W, H, TW, TH, 1.0)
    fb = TiledFramebuffer(W, H, TW, TH)
    bgr = full.get_frame_buffer()
    with GpuSplatter(g, fb, device=0, band_rows=(0, fb.tiles_down), band_cull=True, pair_capacity=1024) as s:
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute_async()  # overflows the 1024-pair capacity
        s.set_band_rows(10, 30)
        with pytest.raises(GsError) as e:
            s.sync()
        assert "overflow" in str(e.value).lower()
        with pytest.raises(GsError):
            s.get_frame_buffer()  # the frame before the move
        with pytest.raises(GsError):
            s.get_histogram()  # ... and its histogram
        assert s.stats()["band_y0"] == 0 and s.stats()["n_tiles"] == fb.tiles_down * fb.tiles_across
        s.execute()  # regrows, renders the moved band
        np.testing.assert_array_equal(s.get_frame_buffer(), bgr[10 * TH:30 * TH])
        assert s.stats()["pair_capacity"] > 1024
        assert s.stats()["band_y0"] == 10 * TH and s.stats()["n_tiles"] == 20 * fb.tiles_across
        np.testing.assert_array_equal(s.get_histogram(),
                                      full.get_histogram().reshape(fb.tiles_down, -1)[10:30].reshape(-1))


@pytest.mark.parametrize("agg", [True, False])
@pytest.mark.parametrize("tile", [(16, 16), (32, 20)])
def test_binning_paths_bit_exact(pc12, test_hook, agg, tile):
    """Both binning paths of a row band -- the aggregated one (per-tile
    counters summed by the projection's workgroups, one-workgroup scan, emit
    by returning atomics per (workgroup, tile); bands up to 16 384 tiles) and
    the chunked one (count / column scan / emit; wider bands, and every whole
    frame) -- give the oracle's lists, histogram and frame bit for bit."""
    from gaussian_splat_ipu_amd import camera

    if not agg:
        test_hook("bin_agg", 0)
    g, bb = pc12
    W, H = 1920, 1080
    view, proj = camera.headless(bb, W, H)
    for band_count, band_index in [(3, 1), (8, 3)]:
        s, f = _frame_pair(g, view, proj, W, H, tile[0], tile[1], 1.0, band_count=band_count, band_index=band_index)
        assert bool(s.stats()["paths"] & 1) == agg  # (GS_PATH_BIN_AGG)
        _assert_parity(s, f, g, check_proj=False)
        s.close()
    s, f = _frame_pair(g, view, proj, W, H, tile[0], tile[1], 1.0)
    assert not s.stats()["paths"] & 1
    _assert_parity(s, f, g, check_proj=False)
    s.close()


PATH_BIN_DIRECT = 128  # (gs_frame_stats.paths, ABI 14)


@pytest.mark.parametrize("band_count,band_index", [(8, 3), (3, 1), (8, 0)])  # (8, 0): no Gaussian reaches it
def test_direct_binning_bit_exact(pc12, test_hook, band_count, band_index):
    """A row band's direct binning (round 6; band-culled bands, the bench's and
    the group's): a view's frames after its first completed one place their
    pairs straight into the segments that frame's scan laid out (no scan, no
    emit launch; the blend's workgroups write the histogram and the frame
    counters).  The renderer's first frame bins with the scan and emit; the
    next ones take the direct path, and frames, histograms and stats stay the
    oracle's bit for bit.  Forced off (hook 0), the same frames take the scan
    and emit."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    g, bb = pc12
    W, H = 1920, 1080
    view, proj = camera.headless(bb, W, H)
    fb = TiledFramebuffer(W, H, 16, 16)
    ty0, ty1, _, _ = fb.band_rows(band_count)[band_index]
    f = O.make_frame(view, proj, W, H, 16, 16, camera.FOV_DEFAULT, 1.0, band=(ty0, ty1))
    seen = []
    for hook, direct in ((-1, True), (0, False)):
        test_hook("bin_direct", hook)
        s = GpuSplatter(g, fb, device=0, band_index=band_index, band_count=band_count, pair_capacity=1 << 23,
                        band_cull=True)
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.execute()
        assert not s.stats()["paths"] & PATH_BIN_DIRECT  # (the first frame: the scan and emit)
        for _ in range(3):
            s.execute()
            assert bool(s.stats()["paths"] & PATH_BIN_DIRECT) == direct, s.stats()["paths"]
            _assert_parity(s, f, g, check_proj=False, band_culled=True)
            seen.append(s.stats()["n_rendered"])
        s.close()
    assert len(set(seen)) == 1, seen  # (both paths count the same band-culled Gaussians)


def test_direct_binning_overflow_falls_back(pc12, test_hook):
    """A direct frame whose tile segments do not hold its lists (forced on
    before any scan has laid out the pair buffer: every segment empty): the
    dropped pairs flag the frame, the blocking render reports the overflow to
    itself and renders again with the scan and emit: the frame the caller
    gets is the oracle's, and async frames that overflow report GS_EOVERFLOW
    at sync."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd._lib import GsError
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    g, bb = pc12
    W, H = 1920, 1080
    view, proj = camera.headless(bb, W, H)
    fb = TiledFramebuffer(W, H, 16, 16)
    ty0, ty1, _, _ = fb.band_rows(8)[3]
    f = O.make_frame(view, proj, W, H, 16, 16, camera.FOV_DEFAULT, 1.0, band=(ty0, ty1))
    test_hook("bin_direct", 1)
    s = GpuSplatter(g, fb, device=0, band_index=3, band_count=8, pair_capacity=1 << 23, band_cull=True)
    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
    s.execute()  # (forced direct into the empty layout: overflows, then the scan and emit)
    assert not s.stats()["paths"] & PATH_BIN_DIRECT
    _assert_parity(s, f, g, check_proj=False, band_culled=True)
    s.close()
    # async: the first frame of a fresh renderer overflows the empty layout
    s = GpuSplatter(g, fb, device=0, band_index=3, band_count=8, pair_capacity=1 << 23, band_cull=True)
    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
    s.execute_async()
    with pytest.raises(GsError):
        s.sync()
    s.execute()  # a blocking frame after it: the oracle's
    _assert_parity(s, f, g, check_proj=False, band_culled=True)
    s.close()


def test_direct_binning_fast_exp_same_frame(pc12, test_hook):
    """GS_FLAG_FAST_EXP band renderers take the direct binning too (its own
    blend instantiation): the direct frames are bit-identical to the same
    renderer's frames binned by the scan and emit."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    g, bb = pc12
    W, H = 1920, 1080
    view, proj = camera.headless(bb, W, H)
    fb = TiledFramebuffer(W, H, 16, 16)
    out = {}
    for hook in (-1, 0):
        test_hook("bin_direct", hook)
        with GpuSplatter(g, fb, device=0, band_index=3, band_count=8, band_cull=True, fast_exp=True) as s:
            s.set_view_wire(view)
            s.set_projection_wire(proj)
            s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
            s.execute()
            s.execute()
            assert bool(s.stats()["paths"] & PATH_BIN_DIRECT) == (hook != 0)
            out[hook] = (s.get_rgba(), s.get_frame_buffer(), s.get_histogram())
    assert_same_bits(out[-1][0], out[0][0], "fast-exp RGBA, direct against scan")
    np.testing.assert_array_equal(out[-1][1], out[0][1])
    np.testing.assert_array_equal(out[-1][2], out[0][2])


def test_direct_binning_follows_the_view(pc12):
    """Direct frames reuse the layout of their view's last scan: a view
    change (and a band move) sends the next frames to the scan and emit until
    one of the new view's frames has completed, with frames of the old view
    still in flight; every frame is the oracle's."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    g, bb = pc12
    W, H = 1920, 1080
    view, proj = camera.headless(bb, W, H)
    view2 = view.copy()
    view2[3] += np.float32(0.05)
    fb = TiledFramebuffer(W, H, 16, 16)
    ref = {}
    for k, v in (("a", view), ("b", view2)):
        for rows in ((27, 36), (20, 30)):
            f = O.make_frame(v, proj, W, H, 16, 16, camera.FOV_DEFAULT, 1.0, band=rows)
            r = O.render(g, f)
            ref[k, rows] = (r["bgr"], r["hist"])
    with GpuSplatter(g, fb, device=0, band_rows=(0, fb.tiles_down), band_cull=True, pair_capacity=1 << 23) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        rows = (27, 36)
        s.set_band_rows(*rows)
        for k in "aabba" + "M" + "ab":
            if k == "M":  # the band moves
                rows = (20, 30)
                s.set_band_rows(*rows)
                continue
            s.set_view_wire(view if k == "a" else view2)
            s.execute_async()
            s.execute_async()
            s.execute()
            np.testing.assert_array_equal(s.get_frame_buffer(), ref[k, rows][0])
            s.execute()  # (a frame of this view has completed: direct)
            assert s.stats()["paths"] & PATH_BIN_DIRECT, (k, rows)
            np.testing.assert_array_equal(s.get_frame_buffer(), ref[k, rows][0])
            np.testing.assert_array_equal(s.get_histogram(), ref[k, rows][1])


def test_aggregated_binning_4k_clustered(built):
    """The aggregated binning of the two bands of a 4K frame (16 200 tiles
    each: the scan runs two 8192-tile rounds) of a clustered scene
    (workgroups whose pairs fall in a few tiles take the ballot path), three
    orbit views."""
    from conftest import PC12
    from gaussian_splat_ipu_amd import camera, scene

    src = scene.load_ply(PC12)
    centres = np.stack([src["x"], src["y"], src["z"]], 1)
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=150_000, seed=8, sh_degree=0, cluster_xyz=centres,
                                                                cluster_sigma=0.02)))
    W, H = 3840, 2160
    _, proj = camera.headless(bb, W, H)
    for k in (0, 40, 80):
        view = camera.orbit_view(k)
        for band in (0, 1):
            s, f = _frame_pair(g, view, proj, W, H, 16, 16, 1.0, band_count=2, band_index=band)
            assert s.stats()["paths"] & 1  # (GS_PATH_BIN_AGG)
            _assert_parity(s, f, g, check_proj=False)
            s.close()


def test_blend_sort_paths_bit_exact(pc12):
    """The tile sort inside the blend's workgroups (row bands of 16x16 tiles:
    every tile's workgroup sorts its list, then blends it one pixel per lane)
    and the separate sort launch (whole frames: two-pixel lanes) give the
    oracle's lists, histogram and frame bit for bit; the paths each frame took
    are in stats()["paths"]."""
    from gaussian_splat_ipu_amd import camera

    g, bb = pc12
    W, H = 1920, 1080
    view, proj = camera.headless(bb, W, H)
    for band_count, band_index in [(1, 0), (8, 3)]:
        s, f = _frame_pair(g, view, proj, W, H, 16, 16, 1.0, band_count=band_count, band_index=band_index)
        paths = s.stats()["paths"]
        assert bool(paths & 2) == (band_count > 1)  # (GS_PATH_BLEND_SORT)
        assert bool(paths & 4) == (band_count == 1)  # (GS_PATH_BLEND_PX2)
        _assert_parity(s, f, g, check_proj=False)
        s.close()



@pytest.mark.parametrize("bin_global", [False, True])
@pytest.mark.parametrize("W,H", [(1920, 1080), (1000, 700)])
def test_blend_px2_bit_exact(pc12, W, H, bin_global):
    """Two pixels per blend lane (whole frames of 16x16 tiles: a 16x8 half of
    the tile per wave, one mask per pixel pair, two independent chains per
    record, tiles longest list first) gives the oracle's frame bit for bit,
    partial edge tiles included (1000x700).  Each slot's tile and list
    segment come from the sort launch's segment table whenever the frame has
    no big-list launches (pc12 has no list > 2048, so both binning paths take
    it here; test_blend_px2_queues_with_big_lists covers the queue reads).  A
    row band keeps one pixel per lane (the in-blend sort)."""
    from gaussian_splat_ipu_amd import camera

    g, bb = pc12
    view, proj = camera.headless(bb, W, H)
    for band_count, band_index in [(1, 0), (8, 3)]:
        s, f = _frame_pair(g, view, proj, W, H, 16, 16, 1.0, band_count=band_count, band_index=band_index,
                           bin_global=bin_global)
        assert bool(s.stats()["paths"] & 4) == (band_count == 1)
        _assert_parity(s, f, g, check_proj=False)
        s.close()


def test_blend_px2_queues_with_big_lists(built):
    """The two-pixel blend reading its slots' tiles from the sort queues and
    the tile starts (no segment table): a frame with big-list launches and no
    lazy lists -- the global-atomic binning, whose frames keep every list
    sorted before the blend.  A dense scene (lists > 2048 keys), the second
    frame takes the big-list launches (the hint of the first); both frames
    bit for bit."""
    from gaussian_splat_ipu_amd import camera, scene

    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=20000, seed=5, sh_degree=0)))
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16).copy()
    rng = np.random.default_rng(3)
    n = a.shape[0]
    a[:, 0] = rng.uniform(-0.3, 0.3, n)
    a[:, 1] = rng.uniform(-0.3, 0.3, n)
    a[:, 2] = rng.uniform(0.0, 1.5, n)
    a[:, 3] = 1.0
    a[:, 7] = rng.uniform(0.02, 0.3, n)
    a[:, 12:15] = -4.0 + rng.normal(0.0, 0.2, (n, 3))
    _, proj = camera.headless(bb, 1280, 720)
    view = np.float32([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -4.0, 0, 0, 0, 1])
    s, f = _frame_pair(a, view, proj, 1280, 720, 16, 16, 1.0, bin_global=True)
    assert s.stats()["n_big_tiles"] > 0
    _assert_parity(s, f, a, check_proj=False)
    s.execute()
    paths = s.stats()["paths"]
    assert paths & 4 and paths & 16 and not paths & 8, paths  # px2, big-list launches, not lazy
    _assert_parity(s, f, a, check_proj=False)
    s.close()


@pytest.mark.parametrize("tw,th", [(32, 8), (8, 32)])
def test_four_block_tiles_other_than_16x16(pc12, tw, th):
    """Tiles of four 8x8 blend blocks that are not 16x16 (32x8, 8x32) keep
    one pixel per lane: the two-pixel blend maps a wave onto a 16x8 half of a
    16x16 tile.  Whole frames with partial edge tiles, and a row
    band (the in-blend sort, one workgroup per tile), bit for bit."""
    from gaussian_splat_ipu_amd import camera

    g, bb = pc12
    W, H = 1000, 700
    view, proj = camera.headless(bb, W, H)
    for band_count, band_index in [(1, 0), (8, 3)]:
        s, f = _frame_pair(g, view, proj, W, H, tw, th, 1.0, band_count=band_count, band_index=band_index)
        assert not s.stats()["paths"] & 4  # (GS_PATH_BLEND_PX2)
        _assert_parity(s, f, g, check_proj=False)
        s.close()
