"""Headline benchmark: frames/sec + Gaussians-splatted/sec of the
project -> bin -> sort -> blend -> BGR8 frame path at 1920x1080 on a synthetic
1M-Gaussian SH-3 scene (BASELINE.json configs[2]; configs[3] for N > 1: the
framebuffer's tile rows split into N bands, one per GPU, one RCCL all-gather
per frame inside gs_render -- the row-band group of gs_group.hip).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.  A "step" is one full frame.  The timed region
covers K frames enqueued back to back (inputs resident in HBM), bracketed by a
barrier + device synchronise; the value is K / max-over-ranks elapsed.

How the N GPUs are driven (launch_mode):
  N = 1 ("single"): F renderers (frames in flight) take frames round-robin on
      their own streams.
  N > 1, no launcher ("group"): ONE process drives the N devices as one
      row-band group (gs_create with num_gpus = N: ncclCommInitAll, one host
      thread per band enqueues its band and its ncclAllGather call).
  N > 1 under torchrun ("ranks"): each rank is one member of the group
      (gs_create_rank); torch.distributed (gloo, host only) carries the RCCL id,
      the barriers and the max-over-ranks reduction.
  --gather: the "group" path even at N = 1 (RCCL over one device).
  --split S: S bands emulated on this one GPU (device-copy gather).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

# the CPU baseline's OpenMP threads stay on their cores (SURVEY §8 d); set
# before any OpenMP runtime (torch's, the oracle's) starts
os.environ.setdefault("OMP_PROC_BIND", "close")
os.environ.setdefault("OMP_PLACES", "cores")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HEADLINE_METRIC = "frames/sec + Gaussians-splatted/sec at 1080p, 1M-Gaussian scene, 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=600)
    # ~200 frames (26 ms) of sustained load bring the GPU to its steady clocks:
    # 20 timed frames after 5 / 30 / 200 warm-up frames ran at 6 700 / 6 950 /
    # 7 600 frames/s (one box, interleaved)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--scale-div", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--sh-degree", type=int, default=3)
    ap.add_argument("--inflight", type=int, default=3,
                    help="frames in flight: independent renderers (N = 1) or band renderers per GPU "
                    "(group), each with its own buffers and HIP stream, take frames round-robin, so one "
                    "frame's latency-bound kernels overlap the next frames' work (every frame is "
                    "rendered in full)")
    ap.add_argument("--profile-frames", type=int, default=24,
                    help="frames of the isolated one-in-flight pass that times each kernel "
                    "(stage HIP events) for the kernel table and the roofline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-frames", type=int, default=120,
                    help="frames of the end-to-end pass after the timed region (each frame's BGR8 read back to "
                    "pinned host memory; reported as end_to_end, never as value); 0 = skip")
    ap.add_argument("--prewarm-ms", type=float, default=50.0,
                    help="untimed frames enqueued for this long (host time) before the --warmup steps, "
                    "reported in the line as prewarm: the GPU's clocks ramp over the first several hundred "
                    "frames, so without it a 20-frame window measures the ramp (DESIGN §7); 0 = none")
    ap.add_argument("--copy-peak-s", type=float, default=0.06,
                    help="seconds of 2 GiB copies for peak_measured (before the timed region; >= 6 copies)")
    ap.add_argument("--split", type=int, default=0,
                    help="one process: a row-band group of S bands emulated on this GPU (device ids "
                    "repeat, device-copy gather): the N > 1 frame path's total work on one GPU")
    ap.add_argument("--config5", action="store_true",
                    help="BASELINE.json configs[4]: 8M Gaussians clustered around point_cloud_12's "
                    "positions (N(0, 0.02) jitter, seed 8), 3840x2160, orbit camera (frame k: "
                    "mvpStart * Ry(360 k / 120)); the tile load-imbalance stress")
    ap.add_argument("--gather", action="store_true",
                    help="the in-process group path (gs_create with num_gpus = --gpus: ncclCommInitAll, one "
                    "ncclAllGather per frame) even at --gpus 1, to exercise the multi-GPU frame path on one GPU")
    ap.add_argument("--no-rebalance", action="store_true", help="group: keep the first (equal-rows) split")
    ap.add_argument("--sh", action="store_true",
                    help="opt-in view-dependent colour (gs_set_sh, SH degree 3 of the synthetic scene's f_dc / "
                    "f_rest) -- not the reference's DC-only colour, so not the headline mode")
    ap.add_argument("--fast-exp", action="store_true",
                    help="GS_FLAG_FAST_EXP (opt-in): the blend's exp from the hardware exp2, per-pixel RGBA within "
                    "the tolerance of tests/test_gpu_fast_exp.py instead of bit-exact (not the headline mode)")
    ap.add_argument("--cpu-frames", type=int, default=20, help="timed CPU baseline frames (median)")
    ap.add_argument("--cpu-warmup", type=int, default=3)
    ap.add_argument("--cpu-budget-s", type=float, default=30.0,
                    help="cap on the CPU baseline's timed frames (fewer frames if one takes longer)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    ap.add_argument("--cpi-json", default=os.path.join(ROOT, "profiles", "valu_cpi.json"),
                    help="VALU cycles per instruction of the kernels' hot loops (tools/valu_cpi.py)")
    return ap.parse_args()


# gs_frame_stats.paths bits (include/gsplat.h)
PATH_BIN_AGG, PATH_BLEND_SORT, PATH_BLEND_PX2, PATH_LAZY, PATH_BIG_LISTS = 1, 2, 4, 8, 16
PATH_PROJ_BAND, PATH_PROJ_ANY = 32, 64  # (ABI 13: which projection instantiation ran)
PATH_BIN_DIRECT = 128  # (ABI 14: a row band's direct binning -- no scan, no emit launch)


def binning_of(paths: int, bin_global: bool = False) -> str:
    """A frame's binning path, in words (gs_frame_stats.paths)."""
    if paths & PATH_BIN_DIRECT:
        return "direct: pairs placed by the projection into the layout of this view's last scan (no scan, no emit)"
    if paths & PATH_BIN_AGG:
        return "aggregated: counted in the projection, one-workgroup scan, emit"
    return "global atomics" if bin_global else "chunked: count, column scan, multi scan, emit"


def stage_kernels(stage: str, paths: int, bin_global: bool = False) -> list:
    """[(rocprof short name, launches per frame)] of the kernels a timed stage
    launched, from the frame's gs_frame_stats.paths (gs_kernels.hip launch_*):
    the roofline's PMC bytes and VALU are those kernels' per-launch counters
    weighted by their launches per frame -- never another path's kernel, never
    a per-launch average of several kernels summed."""
    agg, bsort, px2, lazy, big = (bool(paths & b) for b in (PATH_BIN_AGG, PATH_BLEND_SORT, PATH_BLEND_PX2,
                                                            PATH_LAZY, PATH_BIG_LISTS))
    buckets = [("gs_big_count", 1), ("gs_big_bscan", 1), ("gs_big_scatter", 1), ("gs_big_bsort", 1)]
    if stage == "project":
        if paths & PATH_BIN_DIRECT:
            return [("gs_project_direct", 1)]
        if paths & PATH_PROJ_BAND:
            return [("gs_project_band", 1)]
        return [("gs_project_any" if paths & PATH_PROJ_ANY else "gs_project", 1)]
    if stage in ("scan", "emit") and paths & PATH_BIN_DIRECT:
        return []  # (the projection placed the pairs; the blend's last workgroup wrote the counters)
    if stage == "scan":
        if agg:
            return [("gs_agg_scan", 1)]
        return [("gs_scan", 1)] if bin_global else [("gs_count", 1), ("gs_colscan", 1), ("gs_scan_multi", 1)]
    if stage == "emit":
        return [("gs_agg_emit", 1)] if agg else ([("gs_emit", 1)] if bin_global else [("gs_emit_chunk", 1)])
    if stage == "sort":
        ks = [] if bsort else [("gs_sort_tiles", 1)]
        if big:
            ks += [("gs_big_prefix", 1), ("gs_big_split", 1)]
            ks += [("gs_big_select", 1), ("gs_big_psort", 1)] if lazy else buckets
        return ks
    if stage == "blend":
        if paths & PATH_BIN_DIRECT:
            return [("gs_blend_direct", 1)]
        return [("gs_blend_px2" if px2 else ("gs_blend_sort" if bsort else "gs_blend"), 1)]
    if stage == "blend_cont":  # lazy big lists: window sort + continued blend, pass 2 (launch_blend_cont)
        return [("gs_big_cont", 1), ("gs_blend_cont", 2), ("gs_big_prefix", 1)] + buckets
    raise KeyError(stage)


def pmc_key_of(workload: str, n: int, W: int, H: int, TW: int, bands: int, band: int) -> str:
    """The PMC summary key of a renderer's launches: the workload and the band
    shape -- "whole" for a plain whole-frame renderer, "bands{B}/band{k}" for
    band k of a B-way row split (a group member; B = 1: the whole frame as a
    band, bench.py --gather).  Per-launch counters are kernel properties of
    that shape, not of the launch mode or the frames in flight."""
    shape = "whole" if bands <= 0 else f"bands{bands}/band{band}"
    return f"{workload}:{n}@{W}x{H}/t{TW}/{shape}"


def pmc_lookup(path: str, key: str):
    """The per-kernel PMC summary for `key` from a tools/pmc_summary.py file:
    {"summaries": {key: {"kernels": ...}}} (several band shapes), or the
    one-summary form {"config": key, "kernels": ...}; None when absent."""
    try:
        d = json.load(open(path))
    except Exception:
        return None
    if "summaries" in d:
        e = d["summaries"].get(key)
        return {"config": key, **e} if e else None
    return d if d.get("config") == key else None


def stage_pmc(stage: str, paths: int, kernels: dict, bin_global: bool = False):
    """(HBM bytes, wave64 VALU instructions, missing kernel names) per frame of
    a stage, from a PMC summary's per-launch counters (tools/pmc_summary.py)."""
    ks = stage_kernels(stage, paths, bin_global)
    missing = [k for k, _ in ks if k not in kernels]
    if missing or not ks:
        return None, None, missing
    hbm = sum(n * kernels[k]["hbm_bytes_per_launch"] for k, n in ks)
    valu = sum(n * kernels[k].get("SQ_INSTS_VALU", 0.0) for k, n in ks)
    return hbm, valu, []


def stage_valu_cycles(stage: str, paths: int, kernels: dict, cpi: dict, bin_global: bool = False):
    """(SIMD cycles of VALU issue per frame of a stage, the cpi used per
    kernel), or (None, missing names): each launched kernel's PMC
    SQ_INSTS_VALU x its hot loop's cycles per instruction (tools/valu_cpi.py:
    the MI355X issues a wave64 v_mul / v_add in ~2 cycles, a v_fma / v_cmp /
    v_cvt / v_pk_* in ~4, v_exp in ~8, tools/hip/valu_rate.hip)."""
    ks = stage_kernels(stage, paths, bin_global)
    missing = [k for k, _ in ks if k not in kernels or k not in cpi]
    if missing or not ks:
        return None, missing
    cyc = sum(n * kernels[k].get("SQ_INSTS_VALU", 0.0) * cpi[k]["cpi"] for k, n in ks)
    return cyc, {k: cpi[k]["cpi"] for k, _ in ks}


def measured_copy_peak(torch, min_s: float = 0.06) -> float:
    """Achievable HBM GB/s on this box: a 2 GiB device-to-device copy (read +
    write bytes), best of the copies made in >= min_s seconds (at least 6;
    SURVEY §8 d asks for it beside the spec peak).  bench.py measures it
    before the timed region, so the copies also bring the GPU to the clocks
    it holds under sustained load ("Warm-up and short runs")."""
    n = 1 << 31
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    best = None
    k = 0
    t_start = time.perf_counter()
    while k < 6 or time.perf_counter() - t_start < min_s:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst.copy_(src)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
        k += 1
    del src, dst
    torch.cuda.empty_cache()
    return round(2 * n / best / 1e9, 1)


def survey_bytes(kernel: str, T: int, P: int, n: int, px: int, rec: int, rec_cont: int, st: dict,
                 share: float = 1.0, band: bool = False, sort_in_blend: bool = False) -> float:
    """Algorithmic HBM bytes per launch by SURVEY §8(d)'s terms -- the
    roofline's `achieved`: project N x (56 read + 52 write);
    scan N x 8 plus the tile ranges P x 8 + T x 8; emit N x 12 + P x 12; sort
    one pass, P x 24; blend T x 8 + P x (4 + 36) + Px x 16 with the pack's
    Px x (16 + 3) fused in, where the blend's P is the records it staged (rec,
    gs_frame_stats.blend_records: a wave stops when its pixels have saturated;
    lazy big lists stage their sorted prefixes only).  P = the binned pairs;
    share / band = a row band's share of the frame (band cull: every
    Gaussian's 16-B cull record, the band's Gaussians in full).
    sort_in_blend (gs_frame_stats.paths GS_PATH_BLEND_SORT): the blend
    kernel's workgroups sort the lists of <= 2048 keys themselves, so that
    sort pass's P x 24 is the blend launch's and the sort stage keeps the big
    lists' (st["big_pairs"])."""
    rendered = st["n_rendered"] * share
    in_blend = P - st["big_pairs"] if sort_in_blend else 0
    return {
        "project": n * 16 + rendered * 108 if band else n * 108,
        "scan": n * 8 + P * 8 + T * 8,
        "emit": n * 12 + P * 12,
        "sort": (P - in_blend) * 24,
        "blend": T * 8 + rec * (4 + 36) + px * (16 + 3) + in_blend * 24,
        "blend_cont": rec_cont * (4 + 36) + st["cont_keys"] * 24,
    }[kernel]


def layout_bytes(kernel: str, T: int, P: int, n: int, px: int, rec: int, rec_cont: int, st: dict,
                 n_chunks: int, rect_b: int, share: float = 1.0, band: bool = False,
                 sort_in_blend: bool = False) -> float:
    """HBM bytes per launch of the layouts the kernels actually move (DESIGN
    §3): the figure to hold against the PMC bytes of the same launch (reported
    beside survey_bytes, labelled).
    P = the pairs binned and sorted (the reference rectangle's pairs minus
    those the alpha box culls); T = tiles; px = pixels written; rec = the
    tile-list records the blend staged; rec_cont = the records the
    continuation staged; st = the frame stats (big-list pairs, prefix / window
    keys); rect_b = the bytes of a Gaussian's two rectangles (8 with 8-bit
    bounds, else 16); share / band = a row band's share of the frame's pairs
    (the group); sort_in_blend: the small / medium lists' sort runs in the
    blend's workgroups (its bytes move from the sort stage to the blend)."""
    rendered = st["n_rendered"] * share
    big = st["big_pairs"]
    in_blend = (P - big) * 12 if sort_in_blend else 0
    pre, win = st["big_prefix_keys"], st["big_window_keys"]
    if band:  # band cull: every Gaussian's 16-B cull record and scales + gid, the band's Gaussians in
        # full (mean + opacity, the cached 3D covariance); rectangles, depth key, records
        project = n * (16 + 16) + rendered * (16 + 36 + 4 + 32) + n * rect_b
    else:  # mean + opacity, the cached 3D covariance (52 B); rectangles, depth key; the binned records
        project = n * (52 + rect_b + 4) + rendered * 32
    chunk_matrix = n_chunks * T * 4
    if pre or win:  # lazy big lists: the select reads every big-list key once,
        # writes the prefixes and windows, and the prefixes are sorted into the lists
        big_sort = big * 8 + (pre + win) * 8 + pre * 12
    else:  # the sample sort over every big-list key
        big_sort = big * (8 + 8 + 16 + 12)
    return {
        "project": project,
        # count: both rectangles; count writes the chunk matrix, colscan reads
        # and rewrites it; tile starts, queues and counters
        "scan": n * rect_b + 3 * chunk_matrix + T * 12,
        # emit: the binned rectangle and depth key, its chunk row, the pairs
        "emit": n * (rect_b // 2 + 4) + chunk_matrix + P * 8,
        # small / medium lists: read the 8-B keys, write the 4-B list
        "sort": (P - big) * 12 + big_sort - in_blend,
        # the tile's list bounds; per staged record its 4-B list entry, the
        # 32-B record and the 16-B colour + opacity; RGBA f32 + BGR8 per pixel
        "blend": T * 8 + rec * (4 + 32 + 16) + px * (16 + 3) + in_blend,
        # the continued records, and the window keys the continuation sorted
        "blend_cont": rec_cont * (4 + 32 + 16) + st["cont_keys"] * 12,
    }[kernel]


def bench_chunks(n: int) -> int:
    """The renderer's binning chunk count for a whole frame (gs_renderer.hip:
    chunks of max(4096, n / 256) Gaussians, at most 65 535)."""
    cs = min(65535, max(4096, -(-n // 256)))
    return -(-n // cs)


def core_map():
    """CPU id -> (core, socket) from lscpu (empty if lscpu is unavailable)."""
    core_of = {}
    try:
        out = subprocess.run(["lscpu", "-p=CPU,CORE,SOCKET"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line and not line.startswith("#"):
                c, core, sock = line.split(",")[:3]
                core_of[int(c)] = (core, sock)
    except Exception:
        pass
    return core_of


def host_cpus():
    """(usable CPUs, physical cores among them) from the affinity mask and lscpu."""
    cpus = sorted(os.sched_getaffinity(0))
    core_of = core_map()
    phys = len({core_of[c] for c in cpus if c in core_of}) or None
    return len(cpus), phys


def launch_mode(gpus: int, world_env: int, split: int = 0, gather: bool = False) -> str:
    """How bench.py forms the frame path for --gpus N (module docstring):
    "ranks" (one process per GPU, torchrun set WORLD_SIZE), "group" (one
    process, N devices, ncclCommInitAll), "emulated" (--split S bands on one
    GPU) or "single" (one GPU, independent renderers)."""
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if world_env > 1:
        if world_env != gpus:
            raise SystemExit(f"bench.py: launched with WORLD_SIZE={world_env} ranks but --gpus {gpus}")
        return "ranks"
    if split > 1:
        if gpus > 1:
            raise SystemExit("bench.py: --split emulates the bands on one GPU (use --gpus 1)")
        return "emulated"
    if gpus > 1 or gather:
        return "group"
    return "single"


def frame_digest(bgr) -> str:
    return hashlib.sha1(bgr.tobytes()).hexdigest()[:16]


def main():
    a = parse()
    if a.config5:
        a.n, a.width, a.height, a.seed, a.sh_degree = 8_000_000, 3840, 2160, 8, 0
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    mode = launch_mode(a.gpus, world, a.split, a.gather)
    # GPUs of the job: ranks x 1, or the devices one process drives
    ngpu = world if mode == "ranks" else (a.gpus if mode == "group" else 1)
    if mode == "group":
        have = torch.cuda.device_count()  # (counts without initialising HIP)
        if have < a.gpus:
            raise SystemExit(f"bench.py --gpus {a.gpus}: only {have} HIP device(s) visible")
    torch.cuda.set_device(local)
    if world > 1:
        # host-side plumbing only (RCCL id, barriers, max over ranks); the
        # frame's all-gather is libgsplat's own RCCL call inside gs_render
        dist.init_process_group("gloo")
    group = mode != "single"

    from gaussian_splat_ipu_amd import camera, scene
    from gaussian_splat_ipu_amd._lib import GsError
    from gaussian_splat_ipu_amd.splatter import GpuSplatter, comm_id_create
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
    sh = scene.sh_arrays(ply) if a.sh else None
    if a.sh and sh[1] is None:
        raise SystemExit("--sh needs a scene with f_rest (SH degree 3)")
    del ply
    view, proj = camera.headless(bb, W, H)
    fb = TiledFramebuffer(W, H, TW, TW)
    F = max(1, a.inflight)
    views = [camera.orbit_view(k) for k in range(120)] if a.config5 else [view]

    def setup(r):
        r.set_view_wire(view)
        r.set_projection_wire(proj)
        r.update_focal_lengths(camera.FOV_DEFAULT, a.scale_div)
        if sh is not None:
            r.set_sh(sh[0], sh[1], 3)

    # ------------------------------------------------------------ renderers
    split = a.split if mode == "emulated" else ngpu
    if group:
        if mode == "ranks":  # one process per GPU: ncclCommInitRank
            from gaussian_splat_ipu_amd import dist as gdist

            cid = gdist.share_comm_id(rank, comm_id_create)
            R = [GpuSplatter(g, fb, device=local, comm_id=cid, rank=rank, world=world, frames_in_flight=F,
                             profile=True, rebalance=not a.no_rebalance, fast_exp=a.fast_exp)]
        elif mode == "group":  # one process, N devices: ncclCommInitAll, a host thread per band
            R = [GpuSplatter(g, fb, num_gpus=ngpu, device_ids=list(range(ngpu)), frames_in_flight=F,
                             profile=True, rebalance=not a.no_rebalance, fast_exp=a.fast_exp)]
        else:  # --split S: S bands emulated on this GPU
            R = [GpuSplatter(g, fb, num_gpus=split, device_ids=[local] * split, frames_in_flight=F,
                             profile=True, rebalance=not a.no_rebalance, fast_exp=a.fast_exp)]
    else:
        R = [GpuSplatter(g, fb, device=local, profile=(f == 0), fast_exp=a.fast_exp) for f in range(F)]
    for r in R:
        setup(r)
    s = R[0]
    # no stage events in the timed region (each costs host and device time);
    # the kernel table comes from the isolated pass after it
    s.set_profile_interval(1 << 30)

    nframe = [0]

    def one_frame():
        k = nframe[0]
        r = R[k % len(R)]
        if a.config5:  # orbit camera: a new view every frame
            r.set_view_wire(views[k % 120])
        r.execute_async()
        nframe[0] += 1

    # warm-up: a blocking frame of every view sizes the pair buffers (no timed
    # frame can overflow them); the group's split settles on the headline view
    for r in R:
        for v in views:
            r.set_view_wire(v)
            r.execute()
        r.set_view_wire(views[0])
    def sync_all():
        """Every renderer's gs_sync, then the status agreed over ranks BEFORE any
        barrier: a rank that raised alone would leave the others waiting in
        the barrier (the group decides overflow from the gathered footers, the
        same on every rank; this is the belt to those braces)."""
        err = None
        for r in R:
            try:
                r.sync()
            except GsError as e:
                err = err or e
        if world > 1:
            t = torch.tensor([0 if err is None else 1], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if t.item() and err is None:
                err = RuntimeError("another rank's frames overflowed their pair capacity")
        if err is not None:
            raise err

    # the achievable copy rate, measured before the timed region (its copies
    # keep the GPU busy for ~0.1 s, as a long run's first frames would)
    peak_measured = measured_copy_peak(torch, a.copy_peak_s)
    # pre-warm: untimed frames for --prewarm-ms (beyond the --warmup steps),
    # reported in the line
    prewarm = {"ms": a.prewarm_ms, "frames": 0,
               "note": "untimed frames enqueued before the warm-up steps (the GPU clocks' ramp, DESIGN §7); "
                       "the timed region is exactly --steps frames between barriers"}
    if a.prewarm_ms > 0:
        tp = time.perf_counter()
        while (time.perf_counter() - tp) * 1e3 < a.prewarm_ms:
            for _ in range(8):
                one_frame()
            prewarm["frames"] += 8
    for _ in range(a.warmup):
        one_frame()
    sync_all()
    nframe[0] = 0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enq = []
    for _ in range(a.steps):
        te = time.perf_counter()
        one_frame()
        enq.append(time.perf_counter() - te)
    t_enq = time.perf_counter()  # host time to enqueue the K frames
    sync_all()  # raises (on every rank) on pair overflow
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    fps = a.steps / elapsed
    ms_per_step = 1e3 * elapsed / a.steps

    # the timed frames did the work: each renderer's last timed frame equals a
    # blocking render of the same view on it
    check = []
    for i, r in enumerate(R):
        last_k = max(k for k in range(a.steps) if k % len(R) == i) if a.steps > i else None
        if last_k is None:
            continue
        d0 = frame_digest(r.get_frame_buffer())
        r.set_view_wire(views[last_k % 120] if a.config5 else view)
        r.execute()
        d1 = frame_digest(r.get_frame_buffer())
        check.append(d0 == d1)
    frame_check = {"renderers": len(check), "last_timed_frame_equals_blocking_render": all(check)}

    # end to end with the readback (the reference's frame timer
    # includes getFrameBuffer, splat.cpp:246-268): every frame's BGR8 copied
    # to pinned host memory (gs_read_bgr8) while the next frames render.
    # Reported beside the headline, never as `value` (one GPU, one process)
    e2e = None
    if not group and a.e2e_frames > 0:
        nbytes = H * W * 3
        hosts = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(2)]
        F_ = len(R)
        sync_all()
        torch.cuda.synchronize()
        te0 = time.perf_counter()
        for k in range(a.e2e_frames + F_ - 1):
            if k < a.e2e_frames:
                r = R[k % F_]
                if a.config5:
                    r.set_view_wire(views[k % 120])
                r.execute_async()
            j = k - (F_ - 1)  # the oldest frame in flight: read it back
            if j >= 0:
                R[j % F_].get_frame_buffer(out=hosts[j % 2])
        te1 = time.perf_counter()
        e2e = {
            "frames_per_s": round(a.e2e_frames / (te1 - te0), 1),
            "frames": a.e2e_frames,
            "readback": f"BGR8 {H}x{W}x3 ({nbytes} B) per frame into pinned host memory (gs_read_bgr8), "
                        f"{F_} frames in flight",
            "note": "PCIe-inclusive rate, the reference's timing definition (its timer includes the readback); "
                    "not the headline value (inputs and outputs resident in HBM)",
        }
    st = s.stats()
    bands = s.bands() if group else None

    # kernel table: the same frames with one in flight (renderer 0 alone,
    # stage HIP events on its stream around every kernel of every frame), so
    # each duration is the kernel's own, not shared with other frames' work
    s.set_view_wire(view)
    s.set_profile_interval(1)
    s.execute()
    s.reset_kernel_times()
    for _ in range(a.profile_frames):
        s.execute()  # blocking: one frame in flight (a group's band + its all-gather)
    kt = s.kernel_times()
    st_view = s.stats()

    # algorithmic bytes of the band renderer the table timed (group: rank 0's
    # band, its pairs estimated from the gathered histogram)
    if group:
        hist = s.get_histogram().reshape(fb.tiles_down, fb.tiles_across).astype(np.float64)
        b0, b1 = bands[rank] if world > 1 else bands[0]
        share = hist[b0:b1].sum() / max(1.0, hist.sum())
        T_b = (b1 - b0) * fb.tiles_across
        P_b = int(round(st_view["n_pairs_binned"] * share))
        px = (min(H, b1 * TW) - b0 * TW) * W
    else:
        T_b, P_b, px = st_view["n_tiles"], st_view["n_pairs_binned"], st_view["band_rows"] * W
    # two rectangles per Gaussian, 8-bit bounds when the grid has <= 256 tile
    # columns and band rows (FrameParams::rect8)
    rect_b = 8 if (fb.tiles_across <= 256 and fb.tiles_down <= 256) else 16
    rec, rec_cont = st_view["blend_records"], st_view["blend_cont_records"]
    # the tile sort ran inside the blend's workgroups (gs_frame_stats.paths)
    sib = bool(st_view.get("paths", 0) & 2)
    kern = {}
    for name, (avg_ms, cnt) in kt.items():
        if name in ("scan", "emit") and int(st_view.get("paths", 0)) & PATH_BIN_DIRECT:
            continue  # (direct binning: no such launch; its stage events are back to back)
        if name == "gather":
            if group:
                kern[name] = {"avg_ms": round(avg_ms, 5), "launches": int(cnt),
                              "note": "ncclAllGather on the comm stream, local band done -> frame gathered "
                                      "(includes waiting for the slowest rank)"}
            continue
        if name == "blend_cont" and (not cnt or not rec_cont):
            continue  # (no lazy continuation ran: its stage is two back-to-back events)
        b = survey_bytes(name, T_b, P_b, a.n, px, rec, rec_cont, st_view, share if group else 1.0, group,
                         sort_in_blend=sib)
        lb = layout_bytes(name, T_b, P_b, a.n, px, rec, rec_cont, st_view,
                          0 if group else bench_chunks(a.n), rect_b, share if group else 1.0, group,
                          sort_in_blend=sib)
        kern[name] = {
            "avg_ms": round(avg_ms, 5),
            "launches": int(cnt),
            "alg_bytes": int(b),
            "alg_GBps": round(b / (avg_ms * 1e-3) / 1e9, 1) if avg_ms > 0 else None,
            "layout_bytes": int(lb),
        }
    if "blend" in kern:
        kern["blend"]["records_staged"] = int(rec)
        kern["blend"]["pairs_binned"] = int(P_b)
        # pairs the blend's workgroups sorted (sort inside the blend), in its alg_bytes at 24 B
        kern["blend"]["pairs_sorted"] = int(P_b - st_view["big_pairs"]) if sib else 0
    if "blend_cont" in kern:
        kern["blend_cont"]["records_staged"] = int(rec_cont)
        kern["blend_cont"]["lists"] = int(st_view["cont_lists"])
        kern["blend_cont"]["keys_sorted"] = int(st_view["cont_keys"])
        kern["blend_cont"]["longest_list"] = int(st_view["cont_max"])
        kern["blend_cont"]["prefix_overflows"] = int(st_view["prefix_overflows"])
        kern["blend_cont"]["full_sorts"] = int(st_view["cont_full_sorts"])
        kern["blend_cont"]["note"] = ("the flagged big lists' windows sorted, the continued blend, and the full "
                                      "sample sort of the lists that outlive their window (8 launches, a latency "
                                      "chain); alg_bytes: the continued records and the window keys sorted")
    # the dominant kernel's stage: the longest stage of the one-in-flight
    # kernel table, every stage included.  The lazy continuation (blend_cont,
    # config 5: the flagged big lists' window sort, the continued blend and the
    # full sort of the lists that outlive their window) is a chain of short
    # launches: when it is the longest, the line says it is latency-bound and
    # carries the blend's own figure beside it.
    stage = {k: v for k, v in kern.items() if k != "gather"}
    dom = max(stage, key=lambda k: stage[k]["avg_ms"])
    # PMC counters are per launch (kernel properties): the key names the
    # workload, the split and the band, not the frames in flight
    # (the band shape, not the launch: a --gpus N line's rank 0 renders band 0
    # of N, as band 0 of an N-way split emulated on one GPU does)
    pmc_key = pmc_key_of("c5" if a.config5 else "c3", a.n, W, H, TW, split if group else 0, 0)
    # HBM bytes per launch of the same stage, from the committed PMC summary of
    # this exact workload and band shape (tools/profile.sh, tools/r6/pmc_bands.sh
    # + tools/pmc_summary.py), if any
    pm = pmc_lookup(a.pmc_json, pmc_key)

    paths = int(st_view.get("paths", 0))
    bin_global = bool(st_view.get("bin_global", 0))
    cpi = {}
    if os.path.exists(a.cpi_json):
        try:
            cpi = json.load(open(a.cpi_json))
        except Exception:
            cpi = {}

    def roof(name):
        k = kern[name]
        pmc = valu = valu2 = valu_cpi = valu_note = None
        launched = [x for x, _ in stage_kernels(name, paths, bin_global)]
        if pm is None:
            note = f"no PMC summary for {pmc_key} in {os.path.relpath(a.pmc_json, ROOT)}"
        else:
            hb, vi, missing = stage_pmc(name, paths, pm.get("kernels", {}), bin_global)
            if missing:
                note = f"the PMC summary lacks {', '.join(missing)}, which this stage launched"
            else:
                note = None
                pmc = int(hb)
                # VALU pipe fraction beside the HBM fraction (SURVEY §8 d): the
                # stage's wave64 VALU instructions x their hot loops' measured
                # cycles per instruction over 1024 SIMDs x 2.4 GHz x the launch
                cyc, used = stage_valu_cycles(name, paths, pm.get("kernels", {}), cpi, bin_global)
                if vi:
                    # ... and at a flat 2 SIMD cycles per wave64 instruction
                    # (MI355X_MICROARCH.md's v_fma_f32 row; DESIGN §4 on why
                    # the measured costs differ)
                    valu2 = round(min(1.0, vi * 2.0 / (1024 * 2.4e9 * k["avg_ms"] * 1e-3)), 3)
                if cyc is not None:
                    valu = round(min(1.0, cyc / (1024 * 2.4e9 * k["avg_ms"] * 1e-3)), 3)
                    valu_cpi = used
                elif vi:
                    valu_note = f"no measured VALU cost for {', '.join(used)} in {os.path.relpath(a.cpi_json, ROOT)}"
        ach = k["alg_GBps"]
        out = {
            "kernel": name,
            "launched": launched,
            "achieved": ach,
            "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
            "traffic": pmc,
            "traffic_over_alg": round(pmc / k["alg_bytes"], 3) if pmc and k["alg_bytes"] else None,
            "alg_bytes_per_launch": k["alg_bytes"],
            "layout_bytes_per_launch": k["layout_bytes"],
            "layout_frac": round(k["layout_bytes"] / (k["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            if k["avg_ms"] > 0 else None,
            "avg_launch_ms": k["avg_ms"],
            "valu_issue_frac": valu,
            "valu_issue_frac_2cyc": valu2,
            "valu_cpi": valu_cpi,
        }
        if note:
            out["traffic_note"] = note
        if valu_note:
            out["valu_note"] = valu_note
        return out

    rd = roof(dom)
    roofline = {
        "bound": "hbm",
        "kernel": dom,
        "achieved": rd["achieved"],
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": rd["frac"],
        "traffic": rd["traffic"],
        "traffic_key": pmc_key,
        "traffic_kernels": rd["launched"],
        "traffic_over_alg": rd["traffic_over_alg"],
        "alg_bytes_per_launch": rd["alg_bytes_per_launch"],
        "alg_bytes_model": "SURVEY §8(d) terms (bench.survey_bytes); the blend's P = the records it staged, "
                           "40 B each (4-B list entry + 36-B 2D record), plus T x 8 and Px x (16 + 3)",
        "layout_bytes_per_launch": rd["layout_bytes_per_launch"],
        "layout_frac": rd["layout_frac"],
        "layout_bytes_model": "the bytes the kernels' layouts move (bench.layout_bytes; the blend: 52 B per staged "
                              "record = list entry + 32-B record + 16-B colour)",
        "avg_launch_ms": rd["avg_launch_ms"],
        "valu_issue_frac": rd["valu_issue_frac"],
        "valu_issue_frac_2cyc": rd["valu_issue_frac_2cyc"],
        "valu_cpi": rd["valu_cpi"],
        "valu_model": "SQ_INSTS_VALU of the launched kernels x their hot loops' SIMD cycles per wave64 instruction "
                      "(tools/valu_cpi.py from the measured per-instruction costs, tools/hip/valu_rate.hip: "
                      "v_mul/v_add 2, v_fma/v_cmp/v_cvt/v_pk 4, v_exp 8) over 1024 SIMDs x 2.4 GHz x the launch; "
                      "valu_issue_frac_2cyc: the same instructions at a flat 2 cycles (the guide's v_fma_f32 row)",
        "traffic_model": "PMC HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE) and VALU of the kernels this stage launched in "
                         "the timed frames (gs_frame_stats.paths -> bench.stage_kernels), per launch x launches per "
                         "frame; null with traffic_note when the summary lacks one of them",
        "selection": "longest stage of the one-in-flight kernel table (every stage, the lazy continuation included)",
        "latency_bound": dom == "blend_cont",
        "peak_measured": peak_measured,
    }
    if rd.get("traffic_note"):
        roofline["traffic_note"] = rd["traffic_note"]
    if dom == "blend_cont":
        roofline["note"] = ("the longest stage is the lazy continuation, a chain of short launches (latency-bound); "
                            "the blend's own roofline is in roofline.blend")
    if dom != "blend" and "blend" in kern:
        roofline["blend"] = roof("blend")

    # single-frame latency (one frame in flight, blocking), for reference
    lat = []
    for _ in range(10):
        torch.cuda.synchronize()
        tl = time.perf_counter()
        R[-1].execute()
        lat.append(time.perf_counter() - tl)
    latency_ms = round(1e3 * sorted(lat)[len(lat) // 2], 4)

    cpu = None
    # the group's own account of its bands (RCCL rank count, host threads,
    # per-band HIP-event times of the kernel-table frames and their skew)
    ginfo = None
    if group:
        gi = s.group_info()
        band_ms = gi["band_ms"]
        gather_ms = gi["gather_ms"]
        if world > 1:  # one band per rank: collect them on every rank
            allb = [None] * world
            dist.all_gather_object(allb, (band_ms, gather_ms))
            band_ms = [v for b in allb for v in b[0]]
            gather_ms = [v for b in allb for v in b[1]]
        mean_b = sum(band_ms) / max(1, len(band_ms))
        ginfo = {
            "mode": mode,
            "world": gi["world"],
            "rccl_comm_ranks": gi["comm_ranks"],
            "threaded_enqueue": gi["threaded"],
            "bounds": gi["bounds"],
            "rebalances": gi["rebalances"],
            "timed_frames": gi["timed_frames"],
            "band_ms": [round(v, 5) for v in band_ms],
            "band_skew_max_over_mean": round(max(band_ms) / mean_b, 3) if mean_b > 0 else None,
            "gather_ms": [round(v, 5) for v in gather_ms],
            "note": "per-band HIP events over the kernel-table frames (one in flight): band = its first kernel "
                    "to its last; gather = band written to frame gathered (includes waiting for the slowest band)",
        }

    if rank == 0 and ngpu == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a, g, view, proj, W, H, TW, np)

    if rank == 0:
        if a.config5:
            metric = "frames/sec + Gaussians-splatted/sec at 4K, 8M-Gaussian clustered scene, orbit camera, 1/8 MI355X"
            workload = (f"synthetic {a.n} Gaussians clustered around point_cloud_12 (sigma 0.02), {W}x{H}, "
                        f"{TW}x{TW} tiles, orbit camera (120 views), fxy[1]={a.scale_div}")
        else:
            metric = HEADLINE_METRIC
            workload = f"synthetic {a.n} Gaussians, {W}x{H}, {TW}x{TW} tiles, headless camera, fxy[1]={a.scale_div}"
        if a.split > 1:
            metric = f"frames/sec, {a.split} row bands emulated on one MI355X (group path, device-copy gather)"
        if a.fast_exp:
            metric += " [GS_FLAG_FAST_EXP: RGBA within tolerance, not bit-exact]"
        if a.sh:
            metric += " [gs_set_sh: view-dependent SH-3 colour]"
        if mode == "ranks":
            par = f"row-band x{world}: one process per GPU, work-balanced contiguous bands, one ncclAllGather/frame"
        elif mode == "group":
            par = (f"row-band x{ngpu}: one process, {ngpu} devices (ncclCommInitAll, one host thread per band), "
                   f"work-balanced contiguous bands, one ncclAllGather/frame")
        elif mode == "emulated":
            par = f"row-band x{a.split} emulated on one GPU (copy gather)"
        else:
            par = "single GPU"
        out = {
            "metric": metric,
            "value": round(fps, 3),
            "unit": "frames/s",
            "gaussians_per_sec": round(fps * a.n, 1),
            "pairs_per_sec": round(fps * st["n_pairs"], 1),
            "n_gpus": ngpu,
            "steps": a.steps,
            "warmup": a.warmup,
            "prewarm": prewarm,
            "ms_per_step": round(ms_per_step, 4),
            "frame_latency_ms": latency_ms,
            "host_enqueue_ms_per_step": round(1e3 * (t_enq - t0) / a.steps, 4),
            # per-frame enqueue time percentiles (a long tail = the host waited on the GPU)
            "host_enqueue_ms_p50_p90_max": [round(1e3 * float(np.percentile(enq, q)), 4) for q in (50, 90, 100)],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded xoshiro256**, INRIA 3DGS layout"
                    + (", SH degree 3; parity semantics use DC only)" if a.sh_degree == 3 else ", SH degree 0)"),
            "config": {
                "workload": workload,
                "gaussians": a.n,
                "resolution": [W, H],
                "tile": [TW, TW],
                "frames_in_flight": F,
                "kernel_table": f"{a.profile_frames} blocking frames, one in flight (stage HIP events)",
                "parallelism": par,
                "bands": bands,
                "pmc_key": pmc_key,
                # (the last timed frame's binning; a fixed camera's band frames after the first
                # place their pairs into the layout of that view's last scan: DESIGN.md section 4)
                "binning": binning_of(int(st["paths"]), bool(st.get("bin_global"))),
            },
            "frame": {k: st[k] for k in ("n_rendered", "n_pairs", "n_pairs_binned", "max_list", "n_tiles",
                                         "n_big_tiles", "paths", "bin_global")},
            "frame_check": frame_check,
            "end_to_end": e2e,
            "kernels": kern,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if group:
            out["gather_ms_per_frame"] = kern.get("gather", {}).get("avg_ms")
            out["group"] = ginfo
        print(json.dumps(out), flush=True)
    for r in R:
        r.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(a, g, view, proj, W, H, TW, np):
    """The oracle Gaussian rasteriser on the same frame (the apples-to-apples
    CPU baseline, SURVEY §8 d) and the reference's own CPU point splatter
    restated (cpu_rasteriser.cpp:9-92): OpenMP over the host's cores, pinned
    close, median of --cpu-frames after --cpu-warmup frames, bounded by
    --cpu-budget-s."""
    from gaussian_splat_ipu_amd import camera
    from oracle import oracle as O

    n_cpus, phys = host_cpus()
    omp_env = os.environ.get("OMP_NUM_THREADS")
    # the GPU box sets OMP_NUM_THREADS to its CPU share (16 per GPU); the
    # affinity mask of this (torch-initialised) thread can be narrower than
    # the cores the OpenMP team actually gets, so it does not cap the count
    threads = int(omp_env) if omp_env and omp_env.isdigit() else (phys or n_cpus)
    threads = max(1, threads)
    # where the OpenMP team really runs: each thread reads its CPU inside a
    # parallel region (the affinity mask of this thread says nothing about it)
    team = O.omp_team_cpus(threads, spin_ms=100.0)
    core_of = core_map()
    team_cpus = len(set(team))
    team_cores = len({core_of[c] for c in team if c in core_of}) or None
    f = O.make_frame(view, proj, W, H, TW, TW, camera.FOV_DEFAULT, a.scale_div)

    def timed(fn, frames, warm):
        for _ in range(warm):
            fn()
        ts = []
        tb = time.perf_counter()
        for _ in range(frames):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            if time.perf_counter() - tb > a.cpu_budget_s:
                break
        return float(np.median(ts)), len(ts)

    tc, nf = timed(lambda: O.render(g, f, nthreads=threads, want_rgba=False), a.cpu_frames, a.cpu_warmup)
    xyz = np.ascontiguousarray(g).view(np.float32).reshape(-1, 16)[:, 0:3]
    tp, npf = timed(lambda: O.point_splat(xyz, view, proj, W, H, TW, TW, nthreads=threads), a.cpu_frames,
                    a.cpu_warmup)
    # BASELINE configs[0] (bonsai-7k-mini.ply at 720p on the CPU rasteriser; the
    # file is absent): its SURVEY §8 d substitute, the seeded synthetic 7k scene
    # and point_cloud_12 at 1280x720 / 32x20 through the same CPU point splatter
    from gaussian_splat_ipu_amd import scene as gscene

    c1 = {}
    for name, ply in (("synthetic_7k_seed7", gscene.synthetic(gscene.SynthSpec(n=7000, seed=7, sh_degree=3))),
                      ("point_cloud_12", gscene.load_ply(os.path.join(ROOT, "tests", "golden", "point_cloud_12.ply")))):
        g1, bb1 = gscene.prepare_scene(ply)
        v1, p1 = camera.headless(bb1, 1280, 720)
        x1 = np.ascontiguousarray(g1).view(np.float32).reshape(-1, 16)[:, 0:3].copy()
        t1, n1 = timed(lambda: O.point_splat(x1, v1, p1, 1280, 720, 32, 20, nthreads=threads), 50, 3)
        c1[name] = {"points": int(len(x1)), "frames_per_s": round(1.0 / t1, 1), "median_of": n1}
    host = (f"{os.cpu_count()} CPUs on the host, {n_cpus} in this thread's affinity mask, {phys} physical "
            f"cores among those (lscpu); "
            f"OMP_NUM_THREADS={omp_env} (the GPU box's CPU share), OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')}; "
            f"the {threads}-thread OpenMP team ran on {team_cpus} distinct CPUs = {team_cores} physical cores "
            f"(sched_getcpu inside a parallel region)")
    return {
        "value": round(1.0 / tc, 4),
        "unit": "frames/s",
        "cores": team_cores or team_cpus,
        "threads": threads,
        "team_cpus": team_cpus,
        "team_physical_cores": team_cores,
        "kind": "port",
        "sample": f"median of {nf} full frames (after {a.cpu_warmup} warm-up) of the same {a.n}-Gaussian {W}x{H} "
                  f"workload through the CPU oracle Gaussian rasteriser (OpenMP, {threads} threads)",
        "host": host,
        "gaussians_per_sec": round(a.n / tc, 1),
        "config1_substitute": {
            "workload": "BASELINE configs[0] substitute (bonsai-7k-mini.ply is absent): 1280x720, 32x20 tiles, "
                        "the reference's CPU point splatter (cpu_rasteriser.cpp:9-92) restated",
            "threads": threads, **c1},
        "reference_cpu_path": {
            "value": round(1.0 / tp, 2),
            "unit": "frames/s",
            "kind": "port",
            "sample": f"median of {npf} frames of the reference's CPU point splatter (projectPoints + "
                      f"splatPoints + buildTileHistogram) on the same {a.n} points, {threads} threads",
        },
    }


if __name__ == "__main__":
    main()
