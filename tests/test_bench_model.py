"""bench.py's algorithmic-byte model (SURVEY §8 d) on CPU: the
per-stage bytes follow the layouts the kernels move, and the committed
round-end bench lines stay within 1.1x of the PMC bytes of the same stages
("algorithmic bytes <= PMC bytes x 1.1, or the difference is
explained")."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles", "r03_end")


def _stats(**kw):
    st = {"n_rendered": 1_000_000, "big_pairs": 0, "big_prefix_keys": 0, "big_window_keys": 0, "cont_keys": 0}
    st.update(kw)
    return st


def test_chunk_count_matches_the_renderer_rule():
    # gs_renderer.hip: chunks of max(4096, n / 256) Gaussians, at most 65 535
    assert bench.bench_chunks(1_000_000) == 245
    assert bench.bench_chunks(8_000_000) == 256
    assert bench.bench_chunks(20_000_000) == 306
    assert bench.bench_chunks(1000) == 1


def test_stage_bytes_from_the_layouts():
    n, T, P, px, rec = 1_000_000, 8160, 1_990_107, 1920 * 1080, 1_334_875
    nc = bench.bench_chunks(n)
    st = _stats()

    def ab(k, **kw):
        return bench.alg_bytes(k, T, P, n, px, rec, 0, st, nc, 8, **kw)

    # mean + opacity, scales + gid, rotation; two 4-B rectangles, depth key; 32-B records
    assert ab("project") == n * (48 + 8 + 4) + n * 32
    assert ab("scan") == n * 8 + 3 * nc * T * 4 + T * 12
    assert ab("emit") == n * (4 + 4) + nc * T * 4 + P * 8
    assert ab("sort") == P * 12  # no big lists: read the key, write the list entry
    assert ab("blend") == T * 8 + rec * 52 + px * 19
    # a band: every Gaussian's 16-B cull record, the band's share in full
    assert ab("project", share=0.25, band=True) == n * 16 + 0.25 * n * (48 + 4 + 32) + n * 8


def test_lazy_big_list_sort_bytes():
    n, T, P = 8_000_000, 32400, 26_000_000
    st = _stats(n_rendered=8_000_000, big_pairs=24_000_000, big_prefix_keys=1_800_000, big_window_keys=2_700_000)
    b = bench.alg_bytes("sort", T, P, n, 3840 * 2160, 0, 0, st, 256, 8)
    # small / medium lists; the select reads every big-list key once, writes the
    # prefixes and windows; the prefixes are sorted into the lists
    assert b == (P - 24_000_000) * 12 + 24_000_000 * 8 + (1_800_000 + 2_700_000) * 8 + 1_800_000 * 12
    # without lazy prefixes: the full sample sort of every big-list key
    st0 = _stats(big_pairs=24_000_000)
    assert bench.alg_bytes("sort", T, P, n, 0, 0, 0, st0, 256, 8) == (P - 24_000_000) * 12 + 24_000_000 * 44


@pytest.mark.parametrize("line,pmc", [("bench_c3_pmc.json", "pmc_c3.json"), ("bench_c5.json", "pmc_c5.json")])
def test_committed_lines_within_pmc(line, pmc):
    lp, pp = os.path.join(PROF, line), os.path.join(PROF, pmc)
    if not (os.path.exists(lp) and os.path.exists(pp)):
        pytest.skip("round-end profiles not present")
    d = json.loads(open(lp).read().strip().splitlines()[-1])
    kernels = json.load(open(pp))["kernels"]
    for stage, k in d["kernels"].items():
        if "alg_bytes" not in k:
            continue
        names = [x for x in bench.STAGE_KERNELS.get(stage, []) if x in kernels]
        if not names:
            continue
        hbm = sum(kernels[x]["hbm_bytes_per_launch"] for x in names)
        assert k["alg_bytes"] <= 1.1 * hbm, (stage, k["alg_bytes"], hbm)
