"""Pinning the CPU oracle (test infrastructure) before it is trusted:

* its expf specification against correctly rounded exp (<= 2 ulp, specials);
* its C restatement against an independent pure-Python float32 restatement
  (tests/pyref.py) -- projection records, binning lists and the blended image
  must agree bit for bit on small scenes;
* its outputs against the committed golden fixtures (tests/golden/, made by
  tools/make_golden.py), so a later change to the oracle cannot drift silently.
The reference's own known-answer tests are in test_kat.py.
"""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, PC12
import pyref


def ulp_err(got: float, want: float) -> float:
    spacing = np.spacing(np.float32(abs(want))) if want != 0 else np.float32(1.4e-45)
    return abs(got - want) / float(spacing)


def test_expf_accuracy(built):
    from oracle import oracle as O

    xs = np.concatenate([
        np.linspace(-103.0, 88.0, 20001, dtype=np.float32),
        np.linspace(-10.0, 0.0, 20001, dtype=np.float32),
        np.float32([-1e-7, 1e-7, 0.5, -0.5, 1.0, -1.0, 80.0, -87.0, -87.5, -100.0]),
    ])
    worst = 0.0
    for x in xs:
        got = O.expf(float(x))
        want = math.exp(float(x))
        if want < 1.17549435e-38:  # subnormal results: absolute error of one quantum
            assert abs(got - want) <= 1.5e-45 * 1.01
            continue
        worst = max(worst, ulp_err(got, want))
    assert worst <= 2.0, worst


def test_expf_specials(built):
    from oracle import oracle as O

    assert math.isnan(O.expf(float("nan")))
    assert O.expf(float("-inf")) == 0.0
    assert O.expf(float("inf")) == float("inf")
    assert O.expf(89.0) == float("inf")
    assert O.expf(-104.0) == 0.0
    assert O.expf(0.0) == 1.0


@pytest.mark.parametrize("x", [-88.0, -20.5, -3.25, -0.75, -1e-3, 0.0, 0.3, 5.0, 50.0, -101.0])
def test_expf_python_restatement_agrees(built, x):
    from oracle import oracle as O

    assert np.float32(O.expf(x)) == pyref.expf(np.float32(x))


def _small_scene(n=40, seed=3):
    from gaussian_splat_ipu_amd import camera, scene

    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=n, seed=seed, sh_degree=0, log_scale_mu=-3.5)))
    a = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16).copy()
    return a, bb


@pytest.mark.parametrize("W,H,tw,th,scale_div", [(96, 64, 16, 16, 1.0), (64, 40, 32, 20, 0.1), (72, 54, 16, 16, 1.0)])
def test_oracle_matches_python_restatement(built, W, H, tw, th, scale_div):
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    a, bb = _small_scene()
    a[3, 15] = 0.0  # an empty slot
    view, proj = camera.headless(bb, W, H)
    f = O.make_frame(view, proj, W, H, tw, th, camera.FOV_DEFAULT, scale_div)
    ref = pyref.project(a, view, proj, W, H, tw, th, camera.FOV_DEFAULT, scale_div)
    got = O.project(a, f)
    for i, r in enumerate(ref):
        assert got["rendered"][i] == r["rendered"], i
        if a[i, 15] <= 0:
            continue
        np.testing.assert_array_equal(got["mean2d"][i], np.float32(r["mean2d"]))
        np.testing.assert_array_equal(got["conic"][i], np.float32(r["conic"]))
        assert got["clip_z"][i] == r["clip_z"] and got["radius"][i] == r["radius"]
        if r["rect"] is not None:
            assert tuple(got["rect"][i]) == r["rect"]
        elif got["rendered"][i]:
            assert got["rect"][i][0] > got["rect"][i][2]
    img, lists = pyref.render(a, ref, W, H, tw, th)
    ts, lst = O.bin_lists(got, f)
    for t, l in enumerate(lists):
        np.testing.assert_array_equal(lst[ts[t]:ts[t + 1]], np.asarray(l, np.uint32))
    out = O.render(a, f)
    np.testing.assert_array_equal(out["rgba"].view(np.uint32), img.view(np.uint32))


def test_pack_bgr8_rounding(built):
    """a14: min(v*255, 255) -> round half to even -> saturate -> RGBA2BGR."""
    from oracle import oracle as O
    import ctypes as C

    rgba = np.array([[0.5 / 255, 1.5 / 255, 2.5 / 255, 0.0], [-1.0, 2.0, np.nan, 1.0],
                     [1.0, 0.999, 0.0019607843, 0.0]], np.float32)
    bgr = np.zeros((3, 3), np.uint8)
    O.lib().or_pack_bgr8(rgba.ctypes.data_as(C.POINTER(C.c_float)), 3, bgr.ctypes.data_as(C.POINTER(C.c_uint8)))
    exp = []
    for px in rgba:
        ch = []
        for v in px[:3]:
            x = np.float32(v) * np.float32(255.0)
            x = np.float32(255.0) if np.float32(255.0) < x else x
            ch.append(0 if np.isnan(x) else int(min(255, max(0, np.rint(x)))))
        exp.append(ch[::-1])
    np.testing.assert_array_equal(bgr, np.array(exp, np.uint8))


GOLDEN_CASES = os.path.join(GOLDEN, "oracle_golden.npz")


def test_oracle_against_committed_golden(built):
    """tests/golden/oracle_golden.npz (tools/make_golden.py): point_cloud_12 at
    the reference geometry and a seeded synthetic 1080p scene."""
    from tools_golden import CASES, run_case

    gold = np.load(GOLDEN_CASES, allow_pickle=False)
    for name in CASES:
        out = run_case(name)
        for key, val in out.items():
            np.testing.assert_array_equal(val, gold[f"{name}/{key}"], err_msg=f"{name}/{key}")
