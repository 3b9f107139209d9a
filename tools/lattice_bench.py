"""Time the lattice-migration emulator (GS_FLAG_LATTICE): GPU steps per
second of point_cloud_12 (or a synthetic scene) at the reference's geometry,
with the CPU oracle's step timed beside it.  Prints one JSON line.

    python tools/lattice_bench.py [--n 0] [--frames 200] [--scale-div 0.1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=0, help="synthetic Gaussians (0: point_cloud_12)")
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--cpu-frames", type=int, default=20)
    ap.add_argument("--scale-div", type=float, default=0.1)
    a = ap.parse_args()

    import numpy as np
    import torch

    from gaussian_splat_ipu_amd import camera, scene
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
    from oracle import oracle as O

    if a.n:
        g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=a.n, seed=1, sh_degree=0)))
    else:
        g, bb = scene.prepare_scene(scene.load_ply(os.path.join(ROOT, "tests", "golden", "point_cloud_12.ply")))
    view, proj = camera.headless(bb, 1280, 720)
    s = GpuSplatter(g, TiledFramebuffer(1280, 720, 32, 20), device=0, lattice=True)
    s.set_view_wire(view)
    s.set_projection_wire(proj)
    s.update_focal_lengths(camera.FOV_DEFAULT, a.scale_div)
    for _ in range(5):
        s.execute()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        s.execute_async()
    s.sync()
    gpu_s = (time.perf_counter() - t0) / a.frames
    st = s.lattice_stats()

    f = O.make_frame(view, proj, 1280, 720, 32, 20, camera.FOV_DEFAULT, a.scale_div)
    L = O.Lattice(g, f)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    for _ in range(5):
        L.step(f, threads)
    t0 = time.perf_counter()
    for _ in range(a.cpu_frames):
        L.step(f, threads)
    cpu_s = (time.perf_counter() - t0) / a.cpu_frames
    print(json.dumps({
        "workload": f"lattice emulator, {np.ascontiguousarray(g).shape[0]} Gaussians, 1280x720, 32x20 tiles, "
                    f"fxy[1]={a.scale_div}",
        "gpu_ms_per_step": round(gpu_s * 1e3, 4),
        "gpu_steps_per_sec": round(1.0 / gpu_s, 1),
        "cpu_oracle_ms_per_step": round(cpu_s * 1e3, 3),
        "cpu_threads": threads,
        "frames_after": st["frames"],
        "dropped_last_frame": st["dropped"],
        "send_failed_last_frame": st["send_failed"],
    }))


if __name__ == "__main__":
    main()
