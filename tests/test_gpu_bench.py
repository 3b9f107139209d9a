"""bench.py's multi-GPU launch paths on the one-GPU test box (VERDICT r3 item
1): the in-process row-band group (gs_create with num_gpus: ncclCommInitAll,
one host thread per band) runs with no launcher and emits a valid line.  At
--gpus 1 that is `--gather` (RCCL over one device); the same code path serves
--gpus N on an N-GPU node.  One subprocess per case, one at a time."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(*args, timeout=240):
    env = dict(os.environ)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                         timeout=timeout, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_in_process_group_over_rccl():
    d = _bench("--gather", "--n", "200000", "--steps", "60", "--warmup", "20", "--profile-frames", "6",
               "--no-cpu-baseline")
    assert d["n_gpus"] == 1
    assert d["value"] > 0 and d["unit"] == "frames/s"
    assert d["frame_check"]["last_timed_frame_equals_blocking_render"]
    gr = d["group"]
    assert gr["mode"] == "group"
    assert gr["world"] == 1
    assert gr["rccl_comm_ranks"] == 1  # ncclCommCount of the one-device communicator
    assert gr["timed_frames"] >= 6
    assert len(gr["band_ms"]) == 1 and gr["band_ms"][0] > 0
    assert gr["gather_ms"][0] >= 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["frac"] > 0 and r["alg_bytes_per_launch"] > 0
    # the group's stats carry the kernels its band renderer launched (a
    # one-band group renders the whole frame: the two-pixel blend), so the
    # line's PMC lookup asks for the right kernels
    assert r["traffic_kernels"] == ["gs_blend_px2"], r


def test_bench_refuses_more_gpus_than_visible():
    """--gpus N with fewer devices: a clear error before any frame."""
    import torch

    n = torch.cuda.device_count()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "2"],
                         capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode != 0
    assert "HIP device" in out.stderr


def test_bench_single_gpu_line_reports_end_to_end():
    """The one-GPU line: `value` from the device-resident frames, and beside it
    the end-to-end rate with every frame's BGR8 read back to pinned host
    memory (the reference's timer includes its readback)."""
    d = _bench("--n", "200000", "--steps", "60", "--warmup", "20", "--profile-frames", "6", "--e2e-frames", "30",
               "--no-cpu-baseline")
    assert d["n_gpus"] == 1 and d["value"] > 0
    e = d["end_to_end"]
    assert e["frames"] == 30 and 0 < e["frames_per_s"]
    assert d["roofline"]["traffic_kernels"] == ["gs_blend_px2"]
