"""A scene past 256 binning chunks (default 20 M Gaussians, 306 chunks of
65535) at 1080p: the chunked binning (gs_colscan_kernel's extra rows) against
the global-atomic binning (GS_FLAG_BIN_GLOBAL) -- two independent
GPU paths whose frames, histograms and stats must be identical -- and both
paths' frame times.  Prints one JSON line.

    python tools/big_scene.py [--n 20000000] [--frames 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--frames", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch

    from gaussian_splat_ipu_amd import camera, scene
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    t0 = time.perf_counter()
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=a.n, seed=5, sh_degree=0)))
    print(f"scene ready in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    W, H, T = 1920, 1080, 16
    view, proj = camera.headless(bb, W, H)
    out = {"workload": f"synthetic {a.n} Gaussians, {W}x{H}, {T}x{T} tiles, headless camera"}
    frames = {}
    for name, bin_global in (("chunked", False), ("global", True)):
        s = GpuSplatter(g, TiledFramebuffer(W, H, T, T), device=0, bin_global=bin_global)
        s.set_view_wire(view)
        s.set_projection_wire(proj)
        s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        for _ in range(3):
            s.execute()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.frames):
            s.execute_async()
        s.sync()
        dt = (time.perf_counter() - t0) / a.frames
        st = s.stats()
        frames[name] = (s.get_rgba().copy(), s.get_histogram().copy(), st)
        out[name] = {"ms_per_frame": round(dt * 1e3, 3), "bin_global": st["bin_global"],
                     "n_pairs": st["n_pairs"], "max_list": st["max_list"]}
        s.close()
        print(json.dumps(out[name]), file=sys.stderr, flush=True)
    (ra, ha, sa), (rb, hb, sb) = frames["chunked"], frames["global"]
    out["frames_identical"] = bool(np.array_equal(ra.view(np.uint32), rb.view(np.uint32)))
    out["histograms_identical"] = bool(np.array_equal(ha, hb))
    out["stats_identical"] = all(sa[k] == sb[k] for k in ("n_rendered", "n_pairs", "max_list"))
    print(json.dumps(out), flush=True)
    ok = out["frames_identical"] and out["histograms_identical"] and out["stats_identical"]
    sys.exit(0 if ok and out["chunked"]["bin_global"] == 0 and out["global"]["bin_global"] == 1 else 1)


if __name__ == "__main__":
    main()
