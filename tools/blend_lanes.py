"""Kernel-counted blend lane utilisation (GPU; a GS_LANES build, never the
default library).  Builds nothing itself: build the counting library here with

  ABDIR=tmp_ab_l bash tools/build_x.sh lanes "-DGS_LANES=1"

then on the GPU box

  GSPLAT_LIB=tmp_ab_l/lanes/libgsplat.so python tools/blend_lanes.py [--frames 20]

It renders config 3 (1M synthetic Gaussians, 1920x1080, 16x16 tiles, the
headless camera: the bench frame) and prints, per frame, what the two-pixel
blend (gs_blend_px2) counted:
  wave_steps   record steps of the waves (per batch, the longest lane walk)
  lane_steps   record steps of the lanes (each lane walks its own records)
  lane_util    lane_steps / (64 wave_steps): lanes busy per wave step
  evals        live-pixel evaluations (each lane step evaluates its two pixels)
  box_evals    ... whose record's integer alpha box holds the pixel
  hits         ... that composited (an update or the saturating break)
  valu_per_wave_step   (with --valu V: the PMC SQ_INSTS_VALU of the default
                        kernel) VALU wave instructions per wave record step
"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402

from gaussian_splat_ipu_amd import camera, scene  # noqa: E402
from gaussian_splat_ipu_amd.splatter import GpuSplatter  # noqa: E402
from gaussian_splat_ipu_amd.tiles import TiledFramebuffer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--valu", type=float, default=0.0, help="SQ_INSTS_VALU per launch of the default gs_blend_px2")
    a = ap.parse_args()
    if "GSPLAT_LIB" not in os.environ:
        sys.exit("set GSPLAT_LIB to a GS_LANES build (see the docstring)")
    fd, path = tempfile.mkstemp(suffix=".lanes")
    os.close(fd)
    os.environ["GSPLAT_LANES_FILE"] = path
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=a.n, seed=1, sh_degree=0)))
    W, H, T = 1920, 1080, 16
    fb = TiledFramebuffer(W, H, T, T)
    view, proj = camera.headless(bb, W, H)
    with GpuSplatter(g, fb, device=0) as s:
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        for _ in range(a.frames):
            s.execute()
        stats = s.stats()
    raw = np.fromfile(path, np.uint64)
    os.unlink(path)
    if raw.size < 8:
        sys.exit("no counters written: is GSPLAT_LIB a GS_LANES build?")
    c = raw.reshape(-1, 8).sum(axis=0).astype(np.float64) / a.frames
    wave_steps, lane_steps, evals, box, hits, batches, waves = c[:7]
    out = {
        "workload": f"config3 {a.n}/{W}x{H} t{T}, gs_blend_px2, per frame (mean of {a.frames})",
        "wave_steps": wave_steps, "lane_steps": lane_steps,
        "lane_util": lane_steps / (64.0 * wave_steps) if wave_steps else None,
        "evals": evals, "box_evals": box, "hits": hits,
        "evals_per_lane_step": evals / lane_steps if lane_steps else None,
        "box_frac": box / evals if evals else None, "hit_frac_of_box": hits / box if box else None,
        "batches": batches, "waves": waves,
    }
    if a.valu > 0 and wave_steps:
        out["valu_per_wave_step"] = a.valu / wave_steps
    out["n_pairs_binned"] = stats.get("n_pairs_binned")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
