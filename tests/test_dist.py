"""Multi-process path on CPU (gloo, world size 2 and 3): every rank renders
its row band (here with the CPU oracle -- the GPU path's bands are checked
against the same oracle in test_gpu_parity.py), pads it, and one all_gather
assembles the frame.  The assembled frame must equal the single-process
frame bit for bit, and the max-over-ranks timing reduction must work."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, interleaved=False, balanced=False):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gaussian_splat_ipu_amd import camera, dist as gdist, scene
        from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
        from oracle import oracle as O

        g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=20000, seed=4, sh_degree=0)))
        W, H, T = 640, 360, 16
        fb = TiledFramebuffer(W, H, T, T)
        view, proj = camera.headless(bb, W, H)
        if balanced:
            # work-balanced contiguous bands from the full frame's histogram
            # (every rank computes the same split), padded to the tallest band
            full0 = O.render(g, O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0), nthreads=2)
            bands = gdist.balanced_bands(gdist.row_work(full0["hist"], fb), world)
            ty0, ty1 = bands[rank]
            f = O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0, band=(ty0, ty1))
            band = O.render(g, f, nthreads=2)["bgr"]
            pad = max(b1 - b0 for b0, b1 in bands) * T
            padded_np = np.zeros((pad, W, 3), np.uint8)
            padded_np[: band.shape[0]] = band
            padded = torch.from_numpy(padded_np.reshape(-1))
            out = torch.empty(padded.numel() * world, dtype=torch.uint8)
            dist.all_gather_into_tensor(out, padded)
            frame = gdist.assemble_bands(out.numpy(), fb, bands)
            if rank == 0:
                q.put((np.array_equal(frame, full0["bgr"]), float(world), frame.shape))
            return
        if interleaved:
            # tile rows rank, rank + world, ...: each rendered as a one-row
            # oracle band (the GPU renders them in one pass; test_gpu_parity)
            parts = []
            for ty in fb.interleaved_tile_rows(world, rank):
                f = O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0, band=(ty, ty + 1))
                b1 = O.render(g, f, nthreads=2)["bgr"]
                parts.append(np.concatenate([b1, np.zeros((T - b1.shape[0],) + b1.shape[1:], b1.dtype)]))
            band = np.concatenate(parts) if parts else np.zeros((0, W, 3), np.uint8)
        else:
            ty0, ty1, _, rows = fb.band_rows(world)[rank]
            f = O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0, band=(ty0, ty1))
            band = O.render(g, f, nthreads=2)["bgr"]
            assert band.shape[0] == rows
        padded = torch.from_numpy(gdist.pad_band(band, fb, world).reshape(-1))
        out = torch.empty(padded.numel() * world, dtype=torch.uint8)
        dist.all_gather_into_tensor(out, padded)
        frame = gdist.assemble(out.numpy(), fb, world, interleaved=interleaved)
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            full = O.render(g, O.make_frame(view, proj, W, H, T, T, camera.FOV_DEFAULT, 1.0), nthreads=2)["bgr"]
            q.put((np.array_equal(frame, full), float(t.item()), frame.shape))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,interleaved,balanced", [(2, False, False), (3, False, False), (3, True, False),
                                                       (3, False, True)])
def test_band_allgather_equals_single_frame(built, world, interleaved, balanced):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, interleaved, balanced)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    same, tmax, shape = q.get(timeout=10)
    assert same
    assert tmax == float(world)
    assert shape == (360, 640, 3)


def test_balanced_bands_partition():
    """dist.balanced_bands: contiguous, covering, non-empty, and its heaviest
    band exceeds the ideal share by at most two rows' work."""
    from gaussian_splat_ipu_amd import dist as gdist

    rng = np.random.default_rng(3)
    for T, world in [(68, 8), (68, 2), (8, 8), (135, 7), (30, 4)]:
        w = rng.gamma(0.5, 100.0, T) + 1.0
        w[T // 3: T // 2] *= 20.0  # a dense centre
        bands = gdist.balanced_bands(w, world)
        assert bands[0][0] == 0 and bands[-1][1] == T
        assert all(b0 < b1 for b0, b1 in bands)
        assert all(bands[i][1] == bands[i + 1][0] for i in range(world - 1))
        loads = [w[b0:b1].sum() for b0, b1 in bands]
        assert max(loads) <= w.sum() / world + 2.0 * w.max() + 1e-9
    with pytest.raises(ValueError):
        gdist.balanced_bands(np.ones(3), 4)


def _id_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gaussian_splat_ipu_amd import dist as gdist

        made = []

        def make():
            made.append(rank)
            return bytes(range(128))

        cid = gdist.share_comm_id(rank, make)
        q.put((rank, cid == bytes(range(128)), made))
    finally:
        dist.destroy_process_group()


def test_share_comm_id_world_3():
    """bench.py's RCCL-id hand-off for the row-band group (gs_create_rank):
    only rank 0 makes the id, every rank receives the same 128 bytes."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_id_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = sorted(q.get(timeout=10) for _ in range(3))
    assert all(ok for _, ok, _ in got)
    assert [m for _, _, m in got] == [[0], [], []]
