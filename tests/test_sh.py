"""Opt-in view-dependent colour (gs_set_sh).  The reference
reads f_dc only (file_io.cpp:66-68, splat.cpp:136-147); its f_rest_* pass
through.  The product evaluates the 3DGS spherical harmonics (degree <= 3)
per frame in the projection; the oracle restates the same fp32 operations
(or_sh_colours).  Not parity-pinned by the reference (it never evaluates
SH); pinned here by (1) degree 0 == the scene preparation's own colours, bit
for bit, and (2) a third restatement in numpy float32."""
import numpy as np
import pytest

C0 = np.float32(0.28209479177387814)
C1 = np.float32(0.4886025119029199)
C2 = [np.float32(v) for v in (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
                              0.5462742152960396)]
C3 = [np.float32(v) for v in (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
                              -0.4570457994644658, 1.445305721320277, -0.5900435899266435)]


def _np_sh(mean, campos, dc, rest, degree):
    """numpy float32, one operation at a time (the order of the 3DGS code)."""
    f = np.float32
    d = (mean[:, :3] - campos[None]).astype(np.float32)
    ln = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
    x, y, z = d[:, 0] / ln, d[:, 1] / ln, -d[:, 2] / ln
    xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
    out = np.zeros((len(mean), 3), np.float32)
    for c in range(3):
        sh = lambda k: rest[:, c * 15 + k - 1]  # noqa: E731
        r = C0 * dc[:, c]
        if degree > 0:
            r = r - C1 * y * sh(1)
            r = r + C1 * z * sh(2)
            r = r - C1 * x * sh(3)
        if degree > 1:
            r = r + C2[0] * xy * sh(4)
            r = r + C2[1] * yz * sh(5)
            r = r + C2[2] * (f(2) * zz - xx - yy) * sh(6)
            r = r + C2[3] * xz * sh(7)
            r = r + C2[4] * (xx - yy) * sh(8)
        if degree > 2:
            r = r + C3[0] * y * (f(3) * xx - yy) * sh(9)
            r = r + C3[1] * xy * z * sh(10)
            r = r + C3[2] * y * (f(4) * zz - xx - yy) * sh(11)
            r = r + C3[3] * z * (f(2) * zz - f(3) * xx - f(3) * yy) * sh(12)
            r = r + C3[4] * x * (f(4) * zz - xx - yy) * sh(13)
            r = r + C3[5] * z * (xx - yy) * sh(14)
            r = r + C3[6] * x * (xx - f(3) * yy) * sh(15)
        r = r + f(0.5)
        out[:, c] = np.where(r < 0, f(0), r)
    return out


def test_sh_oracle_degree0_is_the_prepared_colour_and_matches_numpy(built):
    from gaussian_splat_ipu_amd import camera, scene
    from oracle import oracle as O

    ply = scene.synthetic(scene.SynthSpec(n=5000, seed=3, sh_degree=3))
    g, bb = scene.prepare_scene(ply)
    dc, rest = scene.sh_arrays(ply)
    assert rest.shape == (5000, 45)
    view, _ = camera.headless(bb, 640, 360)
    g0 = O.sh_colours(g, dc, rest, 0, view)
    a, b = O._g(g), O._g(g0)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))  # degree 0 == preparation
    for deg in (1, 2, 3):
        for v in (view, camera.orbit_view(40)):
            gd = O._g(O.sh_colours(g, dc, rest, deg, v))
            want = _np_sh(a[:, 0:4], O.camera_position(v), dc, rest, deg)
            np.testing.assert_array_equal(gd[:, 4:7].view(np.uint32), want.view(np.uint32))
            np.testing.assert_array_equal(gd[:, 7:].view(np.uint32), a[:, 7:].view(np.uint32))
    # the camera position inverts the view: view * (campos, 1) = origin
    for v in (view, camera.orbit_view(77)):
        m = np.asarray(v, np.float64).reshape(4, 4)
        cp = O.camera_position(v).astype(np.float64)
        assert np.abs(m[:3, :3] @ cp + m[:3, 3]).max() < 1e-4 * max(1.0, np.abs(m[:3, 3]).max())


@pytest.mark.gpu
@pytest.mark.parametrize("group", [False, True])
def test_sh_frames_match_the_oracle(built, group):
    """Degree 3 at two views (and degree 0 == the default frame; off again
    after degree -1), single renderer (two-pixel blend lanes) and a 2-band
    group (the in-blend sort, one pixel per lane)."""
    from gaussian_splat_ipu_amd import camera, scene
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    ply = scene.synthetic(scene.SynthSpec(n=60_000, seed=5, sh_degree=3))
    g, bb = scene.prepare_scene(ply)
    dc, rest = scene.sh_arrays(ply)
    W, H, T = 960, 540, 16
    view, proj = camera.headless(bb, W, H)
    kw = dict(num_gpus=2, device_ids=[0, 0]) if group else dict(device=0)
    with GpuSplatter(g, TiledFramebuffer(W, H, T, T), **kw) as s:
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        s.set_sh(dc, rest, 3)
        for v in (view, camera.orbit_view(20)):
            s.set_view_wire(v)
            s.execute()
            ref = O.render(O.sh_colours(g, dc, rest, 3, v), O.make_frame(v, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0))
            np.testing.assert_array_equal(s.get_frame_buffer(), ref["bgr"])
            got, want = s.get_rgba(), ref["rgba"]
            assert ((got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))).all()
        s.set_view_wire(view)
        plain = O.render(g, O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0))
        s.set_sh(dc, None, 0)
        s.execute()
        np.testing.assert_array_equal(s.get_frame_buffer(), plain["bgr"])
        s.set_sh(None, None, -1)
        s.execute()
        np.testing.assert_array_equal(s.get_frame_buffer(), plain["bgr"])
