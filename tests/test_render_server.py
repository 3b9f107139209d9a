"""The render server (bin/splat, SURVEY §8 f1 + f3) driven over its remote-UI
protocol on loopback: the "ready" exchange, the fov packet, one histogram +
preview per frame, state packets that move the camera (splat.cpp:284-314:
consumeState -> refit the projection to the fov -> dynamic view from the
rotations and X/Y/Z), and "stop".  --device cpu is the reference's default
device (the point splatter), so this runs without a GPU; the GPU variant
switches the device to the Gaussian path mid-session."""
import os
import socket
import subprocess

import numpy as np
import pytest

from conftest import PC12, ROOT

EXE = os.path.join(ROOT, "gaussian_splat_ipu_amd", "bin", "splat")
W, H, T = 640, 360, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _camera(bb, env=0.0, env2=0.0, X=640.0, Y=360.0, Z=1.0, fov_deg=None, first=False):
    """The view/projection the server's loop builds from a UI state (row-major wire)."""
    from gaussian_splat_ipu_amd import camera

    if first:  # frame 0: mvpStart and the projection fitted at 40 degrees
        return camera.headless(bb, W, H)
    fov = camera.FOV_DEFAULT if fov_deg is None else float(np.float32(fov_deg * (np.pi / np.float32(180.0))))
    mv = camera.look_at_bbox(bb[:3], bb[3:], (0.0, 1.0, 1.0), 1.0)
    cmin = camera.mat4_mul_vec4(mv, [bb[0], bb[1], bb[2], 1.0])
    cmax = camera.mat4_mul_vec4(mv, [bb[3], bb[4], bb[5], 1.0])
    proj = camera.fit_frustum(cmin[:3], cmax[:3], fov, W / np.float32(H))
    dv = camera.mat4_mul(mv, camera.rotate(camera.identity(), camera.radians(env), (1.0, 0.0, 0.0)))
    dv = camera.rotate(dv, camera.radians(env2), (0.0, 1.0, 0.0))
    dv = camera.translate(dv, (np.float32(X) / np.float32(50.0), np.float32(Y) / np.float32(50.0),
                               -np.float32(Z) / np.float32(20.0) + np.float32(20.0)))
    return camera.to_wire(dv), camera.to_wire(proj), fov


def _start(tmp_path, device):
    port = _free_port()
    out = tmp_path / "test.png"
    p = subprocess.Popen([EXE, "--input", PC12, "--device", device, "--ui-port", str(port), "--width", str(W),
                          "--height", str(H), "--tile-width", str(T), "--tile-height", str(T), "--out", str(out)],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    from gaussian_splat_ipu_amd.remote_ui import UiClient

    return p, UiClient("127.0.0.1", port), out


def _stop(p, c, out):
    c.send("stop", True)
    try:
        rc = p.wait(timeout=60)
    finally:
        if p.poll() is None:
            p.kill()
        c.close()
    assert rc == 0, p.stderr.read()
    assert out.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"


def test_remote_ui_cpu_device(built, pc12_scene, tmp_path):
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, bb = pc12_scene
    xyz = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[:, 0:3]
    p, c, out = _start(tmp_path, "cpu")
    try:
        name, fov = c.recv()  # updateFov (splat.cpp:182)
        assert name == "fov" and fov == np.float32(camera.FOV_DEFAULT)
        hist, img = c.frame()
        view, proj = _camera(bb, first=True)
        rimg, rhist, _ = O.point_splat(xyz, view, proj, W, H, T, T)
        np.testing.assert_array_equal(hist, rhist)
        np.testing.assert_array_equal(img, rimg)
        # a burst of state packets; the loop consumes them between frames
        state = dict(env=30.0, env2=45.0, X=100.0, Y=-50.0, Z=10.0, fov_deg=50.0)
        for k, v in [("env_rotation", 30.0), ("env_rotation_2", 45.0), ("X", 100.0), ("Y", -50.0), ("Z", 10.0),
                     ("fov", 50.0)]:
            c.send(k, v)
        view, proj, _ = _camera(bb, **state)
        rimg, rhist, _ = O.point_splat(xyz, view, proj, W, H, T, T)
        for _ in range(400):
            hist, img = c.frame()
            if np.array_equal(hist, rhist):
                break
        else:
            raise AssertionError("the state change never reached a frame")
        np.testing.assert_array_equal(img, rimg)
        _stop(p, c, out)
    finally:
        if p.poll() is None:
            p.kill()



def test_remote_ui_survives_malformed_device_packets(built, pc12_scene, tmp_path):
    """the "device" packet's u64 length is the client's; lengths the
    payload does not hold (2^64 - 1 wraps 8 + n), or implausibly long names,
    are ignored -- the server keeps serving and the next valid packets apply."""
    import struct

    from oracle import oracle as O

    g, bb = pc12_scene
    xyz = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[:, 0:3]
    p, c, out = _start(tmp_path, "cpu")
    try:
        c.recv()
        c.frame()
        c.send_raw("device", struct.pack("<Q", (1 << 64) - 1))           # wraps 8 + n
        c.send_raw("device", struct.pack("<Q", (1 << 64) - 4) + b"gpu")   # wraps to a small sum
        c.send_raw("device", struct.pack("<Q", 100) + b"x" * 100)        # longer than any device name
        c.send_raw("device", b"\x01\x02")                                 # no length at all
        c.send("X", 100.0)
        view, proj, _ = _camera(bb, X=100.0)
        rimg, rhist, _ = O.point_splat(xyz, view, proj, W, H, T, T)
        for _ in range(400):
            hist, img = c.frame()
            if np.array_equal(hist, rhist):
                break
        else:
            raise AssertionError("the server stopped applying state after malformed packets")
        np.testing.assert_array_equal(img, rimg)  # still the CPU device
        _stop(p, c, out)
    finally:
        if p.poll() is None:
            p.kill()

@pytest.mark.gpu
def test_remote_ui_switches_to_the_gpu_device(built, pc12_scene, tmp_path):
    """The "device" packet moves the loop to the Gaussian frame path (the UI's
    device switch, InterfaceServer.hpp:198-203); frames then equal the oracle's
    Gaussian frame for the current state, histogram included."""
    from oracle import oracle as O

    g, bb = pc12_scene
    p, c, out = _start(tmp_path, "cpu")
    try:
        c.recv()
        c.frame()
        state = dict(env=10.0, env2=-20.0, X=640.0, Y=360.0, Z=1.0, fov_deg=45.0)
        for k, v in [("env_rotation", 10.0), ("env_rotation_2", -20.0), ("fov", 45.0), ("lambda1", 10.0)]:
            c.send(k, v)
        c.send("device", "gpu")
        view, proj, fov = _camera(bb, **state)
        ref = O.render(g, O.make_frame(view, proj, W, H, T, T, fov, 1.0))
        for _ in range(400):
            hist, img = c.frame()
            if hist.size == ref["hist"].size and np.array_equal(hist, ref["hist"]):
                break
        else:
            raise AssertionError("no GPU frame of the new state arrived")
        np.testing.assert_array_equal(img, ref["bgr"])
        _stop(p, c, out)
    finally:
        if p.poll() is None:
            p.kill()
