"""The row-band group's decisions (gs_group.hip: decide(), exported as
gs_group_decide) on CPU: every rank applies the same rule to the same
gathered footers, so every rank returns the same status, grows to the same
capacity and moves to the same split.  A rank-local overflow (one band, one
earlier in-flight frame) reaches every rank through the footer's sticky word
(word 15), never through a rank-local flag -- the reference's blocking
execute contract (ipu_rasteriser.cpp:408-420) holds on every rank or none.

The world-3 test runs the real data flow with gloo in place of RCCL: each
rank writes its band's footer, one all_gather moves the footers, each rank
decides, and the decisions are compared across ranks."""
import ctypes
import os
import socket

import numpy as np
import pytest

GS_OK, GS_EOVERFLOW = 0, 4


def _decide(footers, foot_words, world, tiles_x, tiles_y, frame_bounds, cur_bounds, rebalance=True):
    from gaussian_splat_ipu_amd import _lib

    L = _lib.lib()
    f = np.ascontiguousarray(footers, dtype=np.uint32)
    fb = np.ascontiguousarray(frame_bounds, dtype=np.uint32)
    cb = np.ascontiguousarray(cur_bounds, dtype=np.uint32)
    nb = np.zeros(world + 1, np.uint32)
    need = ctypes.c_uint64(0)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    rc = L.gs_group_decide(f.ctypes.data_as(u32p), foot_words, world, tiles_x, tiles_y, fb.ctypes.data_as(u32p),
                           cb.ctypes.data_as(u32p), int(rebalance), nb.ctypes.data_as(u32p), ctypes.byref(need))
    return rc, [int(v) for v in nb], int(need.value)


def _band_footer(rng, foot_words, tiles_x, rows, *, ovf=0, sticky=0, weight=1.0):
    """One band's footer as the scan writes it: counters[16] then the band's
    reference list lengths (rows x tiles_x)."""
    f = np.zeros(foot_words, np.uint32)
    lens = (rng.gamma(0.7, 200.0 * weight, rows * tiles_x)).astype(np.uint32)
    pairs = int(lens.sum())
    f[0] = int((lens > 2048).sum())
    f[2] = 1000
    f[3] = ovf
    f[5], f[6] = pairs & 0xFFFFFFFF, pairs >> 32
    f[10], f[11] = f[5], f[6]
    f[15] = sticky
    f[16:16 + lens.size] = lens
    return f


def _frame(rng, world, tiles_x, tiles_y, bounds, heavy_rows=(), ovf=None, sticky=None):
    T = tiles_x * tiles_y
    fw = 16 + T
    out = np.zeros((world, fw), np.uint32)
    for r in range(world):
        rows = bounds[r + 1] - bounds[r]
        w = 1.0 + 30.0 * sum(1 for y in range(bounds[r], bounds[r + 1]) if y in heavy_rows) / rows
        out[r] = _band_footer(rng, fw, tiles_x, rows, ovf=int(ovf == r), sticky=int(sticky == r), weight=w)
    return out, fw


def test_identical_footers_identical_decisions(built):
    rng = np.random.default_rng(5)
    tx, ty, world = 120, 68, 8
    bounds = [0, 9, 18, 27, 36, 45, 54, 62, 68]
    foot, fw = _frame(rng, world, tx, ty, bounds, heavy_rows=set(range(20, 34)))
    a = _decide(foot, fw, world, tx, ty, bounds, bounds)
    b = _decide(foot.copy(), fw, world, tx, ty, bounds, bounds)
    assert a == b
    rc, nb, need = a
    assert rc == GS_OK
    assert nb != bounds  # the heavy rows moved the split
    assert nb[0] == 0 and nb[-1] == ty and all(x < y for x, y in zip(nb, nb[1:]))
    lens = [int(foot[r, 5]) for r in range(world)]
    assert need == max(lens)
    # the split is the Python rule's on the gathered histogram
    from gaussian_splat_ipu_amd import dist

    hist = np.concatenate([foot[r, 16:16 + (bounds[r + 1] - bounds[r]) * tx] for r in range(world)]).astype(np.float64)
    w = hist.reshape(ty, tx).sum(1) + 128.0 * tx
    want = dist.balanced_bands(w, world)
    assert [b0 for b0, _ in want] + [ty] == nb


@pytest.mark.parametrize("word", ["frame", "sticky"])
def test_one_band_overflow_is_everyones(built, word):
    """Only band 1 of 3 overflowed -- in the last frame (word 3) or in an
    earlier in-flight frame (word 15): the status is GS_EOVERFLOW, and the
    split does not move on an overflowed frame."""
    rng = np.random.default_rng(7)
    tx, ty, world = 40, 23, 3
    bounds = [0, 8, 16, 23]
    kw = {"ovf": 1} if word == "frame" else {"sticky": 1}
    foot, fw = _frame(rng, world, tx, ty, bounds, heavy_rows={2, 3, 4}, **kw)
    rc, nb, _ = _decide(foot, fw, world, tx, ty, bounds, bounds)
    assert rc == GS_EOVERFLOW
    assert nb == bounds
    foot[1, 3] = foot[1, 15] = 0
    rc, nb2, _ = _decide(foot, fw, world, tx, ty, bounds, bounds)
    assert rc == GS_OK
    assert nb2 != bounds


def test_no_rebalance_keeps_the_split_and_bad_input_is_refused(built):
    from gaussian_splat_ipu_amd import _lib

    rng = np.random.default_rng(9)
    tx, ty, world = 30, 17, 2
    bounds = [0, 9, 17]
    foot, fw = _frame(rng, world, tx, ty, bounds, heavy_rows={1, 2})
    rc, nb, _ = _decide(foot, fw, world, tx, ty, bounds, bounds, rebalance=False)
    assert rc == GS_OK and nb == bounds
    assert _decide(foot, fw, world, tx, ty, [0, 9, 16], bounds)[0] == _lib.GS_EINVAL  # does not cover the rows
    assert _decide(foot, 16 + 5, world, tx, ty, bounds, bounds)[0] == _lib.GS_EINVAL  # footer too short


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tx, ty = 48, 30
        T = tx * ty
        fw = 16 + T
        bounds = [0, 10, 20, 30]
        decisions = []
        # three frames; rank 1 overflows in frame 1 only: its sticky word stays
        # set in frames 1 and 2 (until the collective sync after frame 2)
        sticky = 0
        for k in range(3):
            rng = np.random.default_rng(100 * k + rank)
            rows = bounds[rank + 1] - bounds[rank]
            ovf = int(rank == 1 and k == 1)
            sticky = sticky | ovf
            mine = _band_footer(rng, fw, tx, rows, ovf=ovf, sticky=sticky, weight=1.0 + 5.0 * (rank == 0))
            t = torch.from_numpy(mine.view(np.int32).copy())
            out = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(out, t)  # the all-gather (RCCL in the group)
            foot = np.stack([o.numpy().view(np.uint32) for o in out])
            decisions.append(_decide(foot, fw, world, tx, ty, bounds, bounds))
        # every rank's decisions, compared on rank 0
        got = [None] * world
        dist.all_gather_object(got, decisions)
        if rank == 0:
            q.put(got)
    finally:
        dist.destroy_process_group()


def test_world3_ranks_decide_alike(built):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = q.get(timeout=10)
    assert got[0] == got[1] == got[2]
    status = [d[0] for d in got[0]]
    # frame 0 fine; frame 1 overflowed on band 1; frame 2 carries band 1's
    # sticky bit, so the sync after it reports the overflow on every rank
    assert status == [GS_OK, GS_EOVERFLOW, GS_EOVERFLOW]
