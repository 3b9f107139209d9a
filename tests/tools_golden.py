"""Golden-fixture cases shared by tools/make_golden.py (writer), the oracle
regression test and the GPU parity test.  Each case is a scene + frame; the
recorded quantities are small: digests of the BGR8 frame and of the sorted
tile lists, the per-tile histogram and list offsets, an RGBA f32 crop and the
projection records of the first 256 Gaussians."""
import hashlib
import os

import numpy as np

from conftest import PC12

CASES = {
    # name: (scene, W, H, tw, th, scale_div)
    "pc12_720p_32x20_sd01": ("pc12", 1280, 720, 32, 20, 0.1),
    "pc12_1080p_16x16_sd1": ("pc12", 1920, 1080, 16, 16, 1.0),
    "synth50k_1080p_16x16_sd1": ("synth50k", 1920, 1080, 16, 16, 1.0),
}
CROP = (slice(300, 364), slice(600, 664))


def scene_of(name):
    from gaussian_splat_ipu_amd import scene

    if name == "pc12":
        return scene.prepare_scene(scene.load_ply(PC12))
    if name == "synth50k":
        return scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=50_000, seed=1, sh_degree=0)))
    raise KeyError(name)


def digest(a) -> np.ndarray:
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def record(bgr, rgba, hist, tile_start, lst, proj_head) -> dict:
    return {
        "bgr_sha256": digest(bgr),
        "rgba_crop": np.ascontiguousarray(rgba[CROP]),
        "hist": np.asarray(hist, np.uint32),
        "tile_start": np.asarray(tile_start, np.int64),
        "list_sha256": digest(np.asarray(lst, np.uint32)),
        "proj_head": np.asarray(proj_head, np.float32),
    }


def frame_args(name):
    from gaussian_splat_ipu_amd import camera

    sc, W, H, tw, th, sd = CASES[name]
    g, bb = scene_of(sc)
    view, proj = camera.headless(bb, W, H)
    return g, view, proj, W, H, tw, th, sd


def run_case(name) -> dict:
    """The oracle's answer for one case."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    g, view, proj, W, H, tw, th, sd = frame_args(name)
    f = O.make_frame(view, proj, W, H, tw, th, camera.FOV_DEFAULT, sd)
    out = O.render(g, f)
    p = O.project(g, f)
    ts, lst = O.bin_lists(p, f)
    head = np.zeros((256, 12), np.float32)
    k = min(256, p.shape[0])
    head[:k, 0:2] = p["mean2d"][:k]
    head[:k, 2:6] = p["conic"][:k]
    head[:k, 6] = p["clip_z"][:k]
    head[:k, 7] = p["radius"][:k]
    r = p["rect"][:k].astype(np.float32)
    empty = (p["rendered"][:k] == 0) | (p["rect"][:k, 0] > p["rect"][:k, 2])
    r[empty] = [1, 1, 0, 0]
    head[:k, 8:12] = r
    return record(out["bgr"], out["rgba"], out["hist"], ts, lst, head)


def gpu_case(name) -> dict:
    """The HIP path's answer for one case (needs a GPU)."""
    from gaussian_splat_ipu_amd import camera
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    g, view, proj, W, H, tw, th, sd = frame_args(name)
    s = GpuSplatter(g, TiledFramebuffer(W, H, tw, th), device=0)
    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, sd)
    s.execute()
    ts, lst = s.get_bins()
    gp = s.get_projected()
    head = np.zeros((256, 12), np.float32)
    k = min(256, gp.shape[0])
    head[:k] = gp[:k]
    empty = head[:k, 8] > head[:k, 10]
    head[:k][empty, 8:12] = [1, 1, 0, 0]
    live = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[:k, 15] <= 0
    head[:k][live] = 0
    rec = record(s.get_frame_buffer(), s.get_rgba(), s.get_histogram(), ts.astype(np.int64), lst, head)
    s.close()
    return rec


GOLDEN_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_golden.npz")
