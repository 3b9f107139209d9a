"""Headline benchmark: frames/sec + Gaussians-splatted/sec of the
project -> bin -> sort -> blend -> BGR8 frame path at 1920x1080 on a synthetic
1M-Gaussian SH-3 scene (BASELINE.json configs[2]; configs[3] for N > 1:
framebuffer tile rows split into N bands, one RCCL all-gather per frame).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.  A "step" is one full frame.  The timed region
covers K frames enqueued back to back (inputs resident in HBM), bracketed by a
barrier + device synchronise; the value is K / max-over-ranks elapsed.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--scale-div", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--sh-degree", type=int, default=3)
    ap.add_argument("--inflight", type=int, default=3,
                    help="frames in flight: independent renderers, each with its own buffers and "
                    "HIP stream, take frames round-robin, so one frame's latency-bound kernels "
                    "overlap the next frames' work (every frame is rendered in full)")
    ap.add_argument("--profile-frames", type=int, default=24,
                    help="frames of the isolated one-in-flight pass that times each kernel "
                    "(stage HIP events) for the kernel table and the roofline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--band-mode", choices=["balanced", "interleaved"], default="balanced",
                    help="N > 1: contiguous tile-row bands split by the work of a calibration "
                    "frame's row histogram (dist.balanced_bands; the band cull then skips ~7/8 "
                    "of the scene per rank), or interleaved tile rows (rank r: rows r, r + N, ...)")
    ap.add_argument("--gather-group", type=int, default=3,
                    help="N > 1: frames per all-gather = frames in flight x this (the collective's "
                    "host cost is paid once per group)")
    ap.add_argument("--split", type=int, default=0,
                    help="row bands of the split (default: the world size); with --gather on one "
                    "GPU, rank 0 renders band 0 of a --split way split (exercises the N > 1 path)")
    ap.add_argument("--config5", action="store_true",
                    help="BASELINE.json configs[4]: 8M Gaussians clustered around point_cloud_12's "
                    "positions (N(0, 0.02) jitter, seed 8), 3840x2160, orbit camera (frame k: "
                    "mvpStart * Ry(360 k / 120)); the tile load-imbalance stress")
    ap.add_argument("--gather", action="store_true",
                    help="run the band copy + RCCL all-gather path even at N = 1 (a one-rank "
                    "process group; exercises the multi-GPU frame path on one GPU)")
    ap.add_argument("--cpu-frames", type=int, default=2)
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    return ap.parse_args()


# the kernels behind each timed stage (rocprof short names)
STAGE_KERNELS = {
    "project": ["gs_project"],
    "scan": ["gs_count", "gs_colscan", "gs_scan"],
    "emit": ["gs_emit_chunk", "gs_emit"],
    "sort": ["gs_sort_tiles", "gs_sort_big"],
    "blend": ["gs_blend"],
}


def measured_copy_peak(torch) -> float:
    """Achievable HBM GB/s on this box: a 2 GiB device-to-device copy (read +
    write bytes), best of 5 (SURVEY §8 d asks for it beside the spec peak)."""
    n = 1 << 31
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    best = None
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst.copy_(src)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    del src, dst
    return round(2 * n / best / 1e9, 1)


def alg_bytes(kernel: str, st: dict, n: int, px: int) -> float:
    """Algorithmic HBM bytes per launch (SURVEY §8 d, restated in DESIGN.md).
    P = the pairs actually binned, sorted and blended (n_pairs_binned: the
    reference rectangle's pairs minus those the alpha box culls)."""
    T, P = st["n_tiles"], st["n_pairs_binned"]
    return {
        "project": n * (56 + 52),
        "scan": T * 12,
        "emit": n * 12 + P * 12,
        "sort": P * 24,
        "blend": T * 8 + P * (4 + 36) + px * (16 + 3),
    }[kernel]


def main():
    a = parse()
    if a.config5:
        a.n, a.width, a.height, a.seed, a.sh_degree = 8_000_000, 3840, 2160, 8, 0
        a.cpu_frames = 1
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("bench.py --gpus N>1 must be launched with torchrun / torch.distributed.run")
    torch.cuda.set_device(local)
    dist_on = world > 1 or a.gather
    if dist_on:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gaussian_splat_ipu_amd import camera, scene
    from gaussian_splat_ipu_amd.splatter import GpuSplatter
    from gaussian_splat_ipu_amd.tiles import TiledFramebuffer

    W, H, TW = a.width, a.height, a.tile
    if a.config5:
        src = scene.load_ply(os.path.join(ROOT, "tests", "golden", "point_cloud_12.ply"))
        centres = np.stack([src["x"], src["y"], src["z"]], 1)
        ply = scene.synthetic(scene.SynthSpec(n=a.n, seed=a.seed, sh_degree=a.sh_degree,
                                              cluster_xyz=centres, cluster_sigma=0.02))
        del src, centres
    else:
        ply = scene.synthetic(scene.SynthSpec(n=a.n, seed=a.seed, sh_degree=a.sh_degree))
    g, bb = scene.prepare_scene(ply)
    del ply
    view, proj = camera.headless(bb, W, H)
    fb = TiledFramebuffer(W, H, TW, TW)
    # N > 1: interleaved tile-row bands (rank r owns rows r, r + N, ...), so
    # every rank gets an equal share of the scene's dense centre rows.
    # F frames in flight: F renderers (own buffers, own non-blocking stream
    # created by libgsplat) take frames round-robin, so one frame's
    # latency-bound kernels (scans, list tails) overlap the next frames' work.
    # Every frame is rendered in full.
    F = max(1, a.inflight)
    # N > 1, balanced: one full frame on every rank gives the row histogram;
    # every rank derives the same work-balanced split from it
    bands, pad_rows = None, 0
    split = a.split if a.split > 0 else world
    if split > 1 and a.band_mode == "balanced":
        from gaussian_splat_ipu_amd import dist as gdist

        cal = GpuSplatter(g, fb, device=local, write_rgba=False)
        cal.set_view_wire(view)
        cal.set_projection_wire(proj)
        cal.update_focal_lengths(camera.FOV_DEFAULT, a.scale_div)
        cal.execute()
        bands = gdist.balanced_bands(gdist.row_work(cal.get_histogram(), fb), split)
        cal.close()
        pad_rows = max(t1 - t0 for t0, t1 in bands)
    R, streams = [], []
    for f in range(F):
        if bands is not None:
            r = GpuSplatter(g, fb, device=local, band_rows=bands[rank], band_pad_rows=pad_rows,
                            profile=(f == 0), band_cull=True)
        else:
            r = GpuSplatter(g, fb, device=local, band_index=rank, band_count=split, profile=(f == 0),
                            band_interleaved=split > 1, band_cull=split > 1)
        r.set_view_wire(view)
        r.set_projection_wire(proj)
        r.update_focal_lengths(camera.FOV_DEFAULT, a.scale_div)
        R.append(r)
        streams.append(torch.cuda.ExternalStream(r.get_stream()))
    s = R[0]
    # no stage events in the timed region (each costs host and device time);
    # the kernel table comes from the isolated pass after it
    s.set_profile_interval(1 << 30)

    # N > 1: each frame writes its padded band into a group buffer; the G
    # frames of a group (F renderers x --gather-group) are all-gathered by ONE RCCL call
    # on a communication stream while the next group renders.  Two group
    # buffers alternate.  (One gather per frame made the host loop the limit:
    # ~57 us of Python/launch work per frame against ~42 us of GPU work at 8
    # bands; a group amortises the collective's host cost over F frames.)
    band_bytes = (pad_rows * TW if bands is not None else fb.rows_per_band_padded(split)) * W * 3
    G = F * max(1, a.gather_group)
    gbuf = [torch.empty(G * band_bytes, dtype=torch.uint8, device="cuda") for _ in range(2)] if dist_on else []
    gout = ([torch.empty(world * G * band_bytes, dtype=torch.uint8, device="cuda") for _ in range(2)]
            if dist_on else [])
    comm = torch.cuda.Stream() if dist_on else None
    ev_copy = [torch.cuda.Event() for _ in range(F)]
    ev_free = [torch.cuda.Event() for _ in range(2)]
    nframe = [0]

    views = [camera.orbit_view(k) for k in range(120)] if a.config5 else None

    def gather_group(g):
        bsel = g % 2
        with torch.cuda.stream(comm):
            for e in ev_copy:
                comm.wait_event(e)
            dist.all_gather_into_tensor(gout[bsel], gbuf[bsel])  # (world, G, band) rank-major
            ev_free[bsel].record(comm)

    def one_frame():
        k = nframe[0]
        i, g, slot = k % F, k // G, k % G
        r, st = R[i], streams[i]
        if views is not None:  # orbit camera: a new view every frame
            r.set_view_wire(views[k % 120])
        if dist_on:
            # the frame writes its band straight into its group-buffer slot
            # (gs_set_bgr8_target), after the gather of group g - 2 read it:
            # a renderer's first frame of the group waits for that, and its
            # last one marks the end of its writes (in-stream order covers the
            # frames between)
            bsel = g % 2
            if slot < F:
                st.wait_event(ev_free[bsel])
            r.set_bgr8_target(gbuf[bsel].data_ptr() + slot * band_bytes, band_bytes)
        r.execute_async()
        if dist_on:
            if slot >= G - F:
                ev_copy[i].record(st)
            if slot == G - 1:
                gather_group(g)
        nframe[0] += 1

    def flush():  # a partial last group is gathered too
        if dist_on and nframe[0] % G:
            for e, st in zip(ev_copy, streams):
                e.record(st)
            gather_group(nframe[0] // G)

    # warm-up (the first blocking render sizes the pair buffers; with the
    # orbit camera every view once, so no timed frame can overflow them)
    for r in R:
        for v in (views if views is not None else [None]):
            if v is not None:
                r.set_view_wire(v)
            r.execute()
    for _ in range(a.warmup):
        one_frame()
    flush()
    nframe[0] = 0
    for r in R:
        r.sync()
    torch.cuda.synchronize()
    s.reset_kernel_times()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one_frame()
    flush()
    t_enq = time.perf_counter()  # host time to enqueue the K frames
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    t1 = time.perf_counter()
    for r in R:
        r.sync()  # raises on pair overflow
    elapsed = t1 - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = s.stats()
    for r in R:
        r.set_bgr8_target(None)
    # kernel table: the same frames with one in flight (renderer 0 alone,
    # stage HIP events on its stream around every kernel of every frame), so
    # each duration is the kernel's own, not shared with other frames' work
    s.set_profile_interval(1)
    s.execute()
    s.reset_kernel_times()
    for _ in range(a.profile_frames):
        s.execute_async()
    s.sync()
    kt = s.kernel_times()
    fps = a.steps / elapsed
    ms_per_step = 1e3 * elapsed / a.steps

    # per-kernel roofline of this rank's band (rank 0 reports)
    px = st["band_rows"] * W
    kern = {}
    for name, (avg_ms, cnt) in kt.items():
        b = alg_bytes(name, st, a.n, px)
        kern[name] = {
            "avg_ms": round(avg_ms, 5),
            "launches": int(cnt),
            "alg_bytes": int(b),
            "alg_GBps": round(b / (avg_ms * 1e-3) / 1e9, 1) if avg_ms > 0 else None,
        }
    dom = max(kern, key=lambda k: kern[k]["avg_ms"])
    # HBM bytes per launch of the same stage, from the committed PMC summary of
    # this workload (tools/profile.sh + tools/pmc_summary.py), when it matches
    pmc = None
    valu = None
    if os.path.exists(a.pmc_json):
        try:
            pm = json.load(open(a.pmc_json))
            ks = pm.get("kernels", {})
            names = [k for k in STAGE_KERNELS[dom] if k in ks]
            if pm.get("config") == f"{a.n}@{W}x{H}/t{TW}/w{world}" and names:
                pmc = int(sum(ks[k]["hbm_bytes_per_launch"] for k in names))
                # VALU issue-slot fraction beside the HBM fraction (SURVEY §8 d):
                # wave64 VALU instructions x 2 cycles over 1024 SIMDs x 2.4 GHz
                vi = sum(ks[k].get("SQ_INSTS_VALU", 0.0) for k in names)
                if vi:
                    valu = round(vi * 2.0 / (1024 * 2.4e9 * kern[dom]["avg_ms"] * 1e-3), 3)
        except Exception:
            pmc = None
    dk = kern[dom]
    achieved = dk["alg_GBps"]
    roofline = {
        "bound": "hbm",
        "kernel": dom,
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
        "traffic": pmc,
        "alg_bytes_per_launch": dk["alg_bytes"],
        "avg_launch_ms": dk["avg_ms"],
        "valu_issue_frac": valu,
        "peak_measured": measured_copy_peak(torch),
    }

    # single-frame latency (one frame in flight, blocking), for reference
    lat = []
    for _ in range(10):
        torch.cuda.synchronize()
        tl = time.perf_counter()
        R[-1].execute()
        lat.append(time.perf_counter() - tl)
    latency_ms = round(1e3 * sorted(lat)[len(lat) // 2], 4)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import oracle as O

        threads = min(16, os.cpu_count() or 1)
        f = O.make_frame(view, proj, W, H, TW, TW, camera.FOV_DEFAULT, a.scale_div)
        O.render(g, f, nthreads=threads, want_rgba=False)  # warm (page-in)
        tc0 = time.perf_counter()
        for _ in range(a.cpu_frames):
            O.render(g, f, nthreads=threads, want_rgba=False)
        tc = (time.perf_counter() - tc0) / a.cpu_frames
        cpu = {
            "value": round(1.0 / tc, 4),
            "unit": "frames/s",
            "cores": threads,
            "kind": "port",
            "sample": f"{a.cpu_frames} full frames of the same {a.n}-Gaussian {W}x{H} workload through the "
            f"CPU oracle Gaussian rasteriser (OpenMP, {threads} threads)",
            "gaussians_per_sec": round(a.n / tc, 1),
        }
        # the reference's own CPU path is a point splatter (cpu_rasteriser.cpp:
        # 9-92), restated in the oracle: reported beside, not comparable
        xyz = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[:, 0:3]
        O.point_splat(xyz, view, proj, W, H, TW, TW, nthreads=threads)
        tp0 = time.perf_counter()
        for _ in range(5):
            O.point_splat(xyz, view, proj, W, H, TW, TW, nthreads=threads)
        tp = (time.perf_counter() - tp0) / 5
        cpu["reference_cpu_path"] = {
            "value": round(1.0 / tp, 2),
            "unit": "frames/s",
            "kind": "port",
            "sample": f"5 frames of the reference's CPU point splatter (projectPoints + splatPoints + "
            f"buildTileHistogram) on the same {a.n} points, {threads} threads",
        }

    if rank == 0:
        out = {
            "metric": "frames/sec + Gaussians-splatted/sec at 1080p, 1M-Gaussian scene, 1/2/4/8 MI355X",
            "value": round(fps, 3),
            "unit": "frames/s",
            "gaussians_per_sec": round(fps * a.n, 1),
            "pairs_per_sec": round(fps * st["n_pairs"] * world, 1) if world == 1 else None,
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "frame_latency_ms": latency_ms,
            "host_enqueue_ms_per_step": round(1e3 * (t_enq - t0) / a.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded xoshiro256**, INRIA 3DGS layout, SH degree 3; parity semantics use DC only)",
            "config": {
                "workload": (f"synthetic {a.n} Gaussians clustered around point_cloud_12 (sigma 0.02), {W}x{H}, "
                             f"{TW}x{TW} tiles, orbit camera (120 views), fxy[1]={a.scale_div}" if a.config5 else
                             f"synthetic {a.n} Gaussians, {W}x{H}, {TW}x{TW} tiles, headless camera, fxy[1]={a.scale_div}"),
                "gaussians": a.n,
                "resolution": [W, H],
                "tile": [TW, TW],
                "frames_in_flight": F,
                "kernel_table": f"{a.profile_frames} frames, one in flight (stage HIP events)",
                "parallelism": f"row-band x{world}" + ((" (work-balanced contiguous bands " + str(bands) + ")"
                                                         if bands is not None else " (interleaved tile rows)")
                                                        + " + RCCL all-gather" if world > 1 else ""),
            },
            "frame": {k: st[k] for k in ("n_rendered", "n_pairs", "n_pairs_binned", "max_list", "n_tiles",
                                         "n_big_tiles")},
            "kernels": kern,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    for r in R:
        r.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
