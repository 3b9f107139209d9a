"""Multi-GPU critical path on ONE GPU: render each band of an N-way row split
(band_count = N, the bench's band flags) on this device, one band at a time,
and time its frames.  The slowest band bounds the N-GPU frame rate before the
all-gather (which bench.py overlaps with the next frame).

  python tools/band_emulate.py [--bands 1,2,4,8] [--steps 100] [--inflight 1]
                               [--contiguous] [--no-cull]

Prints one line per N: per-band us/frame, the slowest band, and the speed-up
over N = 1.  Kernel stage times of the slowest band come from the renderer's
sampled HIP events (GS_FLAG_PROFILE).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bands", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--inflight", type=int, default=1)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--contiguous", action="store_true")
    ap.add_argument("--balanced", action="store_true", help="work-balanced contiguous bands (bench.py's N > 1 default)")
    ap.add_argument("--tile-cost", type=float, default=128.0,
                    help="--balanced: the fixed work per tile of a row, in pairs (dist.row_work's default)")
    ap.add_argument("--no-cull", action="store_true")
    ap.add_argument("--bin-global", action="store_true", help="the bands bin with global atomics")
    ap.add_argument("--only-band", type=int, default=-1, help="time just this band (profiling)")
    ap.add_argument("--config5", action="store_true", help="bench.py --config5's scene, 4K, orbit views")
    ap.add_argument("--rebalance", action="store_true",
                    help="orbit views: move each band renderer (gs_set_band_rows) to the split the group "
                         "would use -- re-cut every 8 frames from the histogram of 4 frames earlier")
    a = ap.parse_args()
    import torch

    from gaussian_splat_ipu_amd import camera, scene
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    W, H, TW = 1920, 1080, 16
    views = None
    if a.config5:
        import numpy as np
        W, H = 3840, 2160
        src = scene.load_ply(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "point_cloud_12.ply"))
        cl = np.stack([src["x"], src["y"], src["z"]], 1)
        g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=8_000_000, seed=8, sh_degree=0,
                                                                    cluster_xyz=cl, cluster_sigma=0.02)))
        views = [camera.orbit_view(k) for k in range(120)]
    else:
        g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=a.n, seed=1, sh_degree=3)))
    view, proj = camera.headless(bb, W, H)
    fb = TiledFramebuffer(W, H, TW, TW)
    base = None
    hist = None
    view_hist = None
    if a.balanced:
        from gaussian_splat_ipu_amd import dist as gdist

        cal = GpuSplatter(g, fb, device=0, write_rgba=False)
        cal.set_view_wire(views[0] if views else view)  # (config 5: the orbit's first view)
        cal.set_projection_wire(proj)
        cal.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
        cal.execute()
        hist = cal.get_histogram()
        if a.rebalance and views is not None:
            view_hist = []
            for v in views:
                cal.set_view_wire(v)
                cal.execute()
                view_hist.append(cal.get_histogram())
        cal.close()
    for N in [int(v) for v in a.bands.split(",")]:
        per_band, stages, host = [], [], []
        bands = gdist.balanced_bands(gdist.row_work(hist, fb, a.tile_cost), N) if hist is not None and N > 1 else None
        pad = max(t1 - t0 for t0, t1 in bands) if bands else 0
        # the group's policy: frame k renders with the split cut at frame
        # 8 (k // 8) from the footers of 4 frames before it
        view_bands = None
        if view_hist is not None and N > 1:
            view_bands = [gdist.balanced_bands(gdist.row_work(h, fb, a.tile_cost), N) for h in view_hist]
            pad = fb.tiles_down
        for r in range(N):
            if a.only_band >= 0 and r != a.only_band:
                continue
            R, S = [], []
            for f in range(a.inflight):
                if view_bands is not None:  # room for any band; moved per frame
                    s = GpuSplatter(g, fb, device=0, band_rows=(0, fb.tiles_down), profile=(f == 0),
                                    band_cull=not a.no_cull, write_rgba=False, bin_global=a.bin_global)
                elif bands is not None:
                    s = GpuSplatter(g, fb, device=0, band_rows=bands[r], band_pad_rows=pad, profile=(f == 0),
                                    band_cull=not a.no_cull, write_rgba=False,
                                    bin_global=a.bin_global)
                else:
                    s = GpuSplatter(g, fb, device=0, band_index=r, band_count=N, profile=(f == 0),
                                    band_interleaved=(N > 1 and not a.contiguous),
                                    band_cull=(N > 1 and not a.no_cull), write_rgba=False,
                                    bin_global=a.bin_global)
                s.set_view_wire(view)
                s.set_projection_wire(proj)
                s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
                s.set_profile_interval(1 << 30)  # no stage events in the timed loop
                R.append(s)
            for s in R:
                for v in (views or [None]):
                    if v is not None:
                        s.set_view_wire(v)
                    s.execute()

            def frame(k):
                if views is not None:
                    R[k % len(R)].set_view_wire(views[k % 120])
                if view_bands is not None:
                    t0, t1 = view_bands[(8 * (k // 8) - 4) % 120][r]
                    R[k % len(R)].set_band_rows(t0, t1)
                R[k % len(R)].execute_async()

            for k in range(a.warmup):
                frame(k)
            torch.cuda.synchronize()
            R[0].reset_kernel_times()
            t0 = time.perf_counter()
            for k in range(a.steps):
                frame(k)
            th = (time.perf_counter() - t0) / a.steps  # host enqueue (returns before the GPU is done)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            host.append(th * 1e6)
            for s in R:
                s.sync()
            per_band.append(dt * 1e6)
            # stage times: an isolated pass, one frame in flight, events on every frame
            R[0].set_profile_interval(1)
            R[0].reset_kernel_times()
            for k in range(12):
                if views is not None:
                    R[0].set_view_wire(views[k % 120])
                if view_bands is not None:
                    R[0].set_band_rows(*view_bands[(8 * (k // 8) - 4) % 120][r])
                R[0].execute_async()
            R[0].sync()
            stages.append({k: round(v[0] * 1e3, 1) for k, v in R[0].kernel_times().items()})
            pairs = R[0].stats()["n_pairs"]
            for s in R:
                s.close()
            del pairs
        worst = max(per_band)
        if base is None:
            base = worst
        i = per_band.index(worst)
        mean = sum(per_band) / len(per_band)
        print(json.dumps({"workload": "config5 8M/4K orbit" if a.config5 else f"config4 {a.n}/1080p",
                          "bands": N, "inflight": a.inflight,
                          "split": "rebalanced per 8 frames (4-frame-old histogram)" if view_bands else bands,
                          "us_per_frame_by_band": [round(v, 1) for v in per_band],
                          "slowest_us": round(worst, 1), "fastest_us": round(min(per_band), 1),
                          "skew_slowest_over_mean": round(worst / mean, 3),
                          "speedup": round(base / worst, 2),
                          "host_enqueue_us_by_band": [round(v, 1) for v in host],
                          "slowest_band_stage_us": stages[i]}), flush=True)


if __name__ == "__main__":
    main()
