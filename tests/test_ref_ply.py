"""The product's PLY reader (gs_ply_load, csrc/host/gs_scene.cpp) against the
reference's own parser: oracle/_ref/ply_dump is the reference's vendored
happly.h compiled from /root/reference/include (oracle/Makefile), called as
splat::fillPlyProperties calls it (src/splat/file_io.cpp:57-77).  Every one of
the 14 properties of every data file the reference ships must come out bit
for bit the same.  CPU only; skipped where /root/reference is absent (the
GPU box)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

REF = "/root/reference"
TOOL = os.path.join(ROOT, "oracle", "_ref", "ply_dump")
PROPS = ["x", "y", "z", "f_dc_0", "f_dc_1", "f_dc_2", "opacity", "scale_0", "scale_1", "scale_2",
         "rot_0", "rot_1", "rot_2", "rot_3"]


def _files():
    out = [os.path.join(REF, "data", f"point_cloud_{k}.ply") for k in (9, 10, 11, 12)]
    return [p for p in out if os.path.exists(p)] + [os.path.join(GOLDEN, "point_cloud_12.ply")]


@pytest.fixture(scope="module")
def tool(built):
    if not os.path.isdir(REF):
        pytest.skip("/root/reference is not present (the reference parser is built here only)")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref-tools"], check=True)
    if not os.path.exists(TOOL):
        pytest.skip("oracle/_ref/ply_dump was not built (happly.h absent)")
    return TOOL


@pytest.mark.parametrize("path", _files(), ids=os.path.basename)
def test_ply_reader_matches_the_reference_parser(tool, tmp_path, path):
    from gaussian_splat_ipu_amd import scene

    dump = tmp_path / "ref.bin"
    subprocess.run([tool, path, str(dump)], check=True)
    raw = dump.read_bytes()
    n = int(np.frombuffer(raw[:8], np.int64)[0])
    ref = np.frombuffer(raw[8:], np.float32).reshape(len(PROPS), n)
    ply = scene.load_ply(path)
    assert len(ply) == n
    for k, name in enumerate(PROPS):
        got = np.asarray(ply[name], np.float32)
        np.testing.assert_array_equal(got.view(np.uint32), ref[k].view(np.uint32), err_msg=name)
