"""bench.py's byte models (SURVEY §8 d) and launch modes on
CPU: the roofline's algorithmic bytes are SURVEY §8(d)'s terms
(survey_bytes), the layout bytes follow the layouts the kernels move and stay
within 1.1x of the PMC bytes of the same stages in the committed round-end
lines, and the committed lines' roofline is recomputable from their own
fields."""
import glob
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _newest_profiles() -> str:
    """The newest round's profile directory holding the round-end PMC summaries
    of configs 3 and 5 (profiles/r0N_*/pmc_c3.json, pmc_c5.json)."""
    ds = sorted(os.path.dirname(p) for p in glob.glob(os.path.join(ROOT, "profiles", "r0*", "pmc_c3.json"))
                if os.path.exists(os.path.join(os.path.dirname(p), "pmc_c5.json")))
    # (the newest round first; within a round, its end set over earlier ones)
    ds.sort(key=lambda d: (os.path.basename(d)[:3], os.path.basename(d).endswith(("final", "end"))))
    return ds[-1] if ds else os.path.join(ROOT, "profiles", "r04_final")


PROF = _newest_profiles()
# the paths the default frames take (gs_frame_stats.paths): config 3 whole
# frames blend two pixels per lane; config 5 (big lists) the lazy one-pixel blend
C3_PATHS = bench.PATH_BLEND_PX2
C5_PATHS = bench.PATH_LAZY | bench.PATH_BIG_LISTS


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
        return bench.layout_bytes(k, T, P, n, px, rec, 0, st, nc, 8, **kw)

    # mean + opacity, the cached 3D covariance + gid; two 4-B rectangles, depth key; 32-B records
    assert ab("project") == n * (52 + 8 + 4) + n * 32
    assert ab("scan") == n * 8 + 3 * nc * T * 4 + T * 12
    assert ab("emit") == n * (4 + 4) + nc * T * 4 + P * 8
    assert ab("sort") == P * 12  # no big lists: read the key, write the list entry
    assert ab("blend") == T * 8 + rec * 52 + px * 19
    # a band: every Gaussian's 16-B cull record and scales + gid, the band's share in full
    assert ab("project", share=0.25, band=True) == n * 32 + 0.25 * n * (16 + 36 + 4 + 32) + n * 8


def test_lazy_big_list_sort_bytes():
    n, T, P = 8_000_000, 32400, 26_000_000
    st = _stats(n_rendered=8_000_000, big_pairs=24_000_000, big_prefix_keys=1_800_000, big_window_keys=2_700_000)
    b = bench.layout_bytes("sort", T, P, n, 3840 * 2160, 0, 0, st, 256, 8)
    # small / medium lists; the select reads every big-list key once, writes the
    # prefixes and windows; the prefixes are sorted into the lists
    assert b == (P - 24_000_000) * 12 + 24_000_000 * 8 + (1_800_000 + 2_700_000) * 8 + 1_800_000 * 12
    # without lazy prefixes: the full sample sort of every big-list key
    st0 = _stats(big_pairs=24_000_000)
    assert bench.layout_bytes("sort", T, P, n, 0, 0, 0, st0, 256, 8) == (P - 24_000_000) * 12 + 24_000_000 * 44


def test_survey_bytes_are_section_8d_terms():
    """project N x (56 + 52); scan N x 8 + ranges P x 8 + T x 8;
    emit N x 12 + P x 12; sort P x 24 (one pass); blend T x 8 + P x (4 + 36)
    + Px x 16 with the pack's Px x (16 + 3) fused (P = the records staged)."""
    n, T, P, px, rec = 1_000_000, 8160, 1_990_107, 1920 * 1080, 1_334_875
    st = _stats(cont_keys=1000)

    def sb(k, **kw):
        return bench.survey_bytes(k, T, P, n, px, rec, 77, st, **kw)

    assert sb("project") == n * 108
    assert sb("scan") == n * 8 + P * 8 + T * 8
    assert sb("emit") == n * 12 + P * 12
    assert sb("sort") == P * 24
    assert sb("blend") == T * 8 + rec * 40 + px * 19
    # the round-3 verdict's figure for config 3: 92.86 MB per blend launch
    assert abs(sb("blend") - 92.86e6) < 0.01e6
    assert sb("blend_cont") == 77 * 40 + 1000 * 24
    assert sb("project", share=0.25, band=True) == n * 16 + 0.25 * n * 108
    # the sort inside the blend: the small / medium lists' pass moves to the blend
    st["big_pairs"] = 1000
    assert sb("blend", sort_in_blend=True) == T * 8 + rec * 40 + px * 19 + (P - 1000) * 24
    assert sb("sort", sort_in_blend=True) == 1000 * 24


def test_launch_modes():
    assert bench.launch_mode(1, 1) == "single"
    assert bench.launch_mode(1, 1, gather=True) == "group"
    # no launcher: one process drives the N devices (ncclCommInitAll)
    assert bench.launch_mode(8, 1) == "group"
    assert bench.launch_mode(2, 1) == "group"
    # torchrun: one rank per GPU
    assert bench.launch_mode(8, 8) == "ranks"
    assert bench.launch_mode(1, 1, split=8) == "emulated"
    for bad in [(4, 8), (0, 1)]:
        with pytest.raises(SystemExit):
            bench.launch_mode(*bad)
    with pytest.raises(SystemExit):
        bench.launch_mode(2, 1, split=4)


@pytest.mark.parametrize("line,pmc,paths", [("bench_c3_pmc.json", "pmc_c3.json", C3_PATHS),
                                             ("bench_c5.json", "pmc_c5.json", C5_PATHS)])
def test_committed_lines_within_pmc(line, pmc, paths):
    lp, pp = os.path.join(PROF, line), os.path.join(PROF, pmc)
    if not (os.path.exists(lp) and os.path.exists(pp)):
        pytest.skip("round-end profiles not present")
    d = json.loads(open(lp).read().strip().splitlines()[-1])
    kernels = json.load(open(pp))["kernels"]
    paths = d["frame"].get("paths", paths)
    for stage, k in d["kernels"].items():
        lb = k.get("layout_bytes", k.get("alg_bytes"))  # (round-3 lines: alg_bytes was the layout model)
        if lb is None:
            continue
        hbm, _, missing = bench.stage_pmc(stage, paths, kernels)
        assert not missing, (stage, missing)
        assert lb <= 1.1 * hbm, (stage, lb, hbm)


def test_stage_kernels_follow_the_frame_paths():
    """The roofline's PMC figures come from the kernels the timed frames
    launched (a line read another path's kernel)."""
    sk = bench.stage_kernels
    assert sk("blend", C3_PATHS) == [("gs_blend_px2", 1)]
    assert sk("blend", C5_PATHS) == [("gs_blend", 1)]
    assert sk("blend", bench.PATH_BLEND_SORT | bench.PATH_BIN_AGG) == [("gs_blend_sort", 1)]
    assert sk("scan", bench.PATH_BIN_AGG) == [("gs_agg_scan", 1)]
    assert sk("scan", 0) == [("gs_count", 1), ("gs_colscan", 1), ("gs_scan_multi", 1)]
    assert [k for k, _ in sk("sort", C5_PATHS)] == ["gs_sort_tiles", "gs_big_prefix", "gs_big_split",
                                                   "gs_big_select", "gs_big_psort"]
    assert ("gs_blend_cont", 2) in sk("blend_cont", C5_PATHS)
    # launches per frame weight the per-launch counters; a missing kernel is reported
    ks = {"gs_big_cont": {"hbm_bytes_per_launch": 10.0, "SQ_INSTS_VALU": 1.0},
          "gs_blend_cont": {"hbm_bytes_per_launch": 3.0, "SQ_INSTS_VALU": 2.0}}
    hb, vi, missing = bench.stage_pmc("blend_cont", C5_PATHS, ks)
    assert hb is None and "gs_big_bsort" in missing
    for k in ("gs_big_prefix", "gs_big_count", "gs_big_bscan", "gs_big_scatter", "gs_big_bsort"):
        ks[k] = {"hbm_bytes_per_launch": 1.0, "SQ_INSTS_VALU": 0.0}
    hb, vi, missing = bench.stage_pmc("blend_cont", C5_PATHS, ks)
    assert (hb, vi, missing) == (10.0 + 2 * 3.0 + 5.0, 1.0 + 2 * 2.0, [])


def test_valu_cycles_weigh_each_kernel_by_its_measured_cost():
    """The roofline's VALU fraction: each launched kernel's SQ_INSTS_VALU x
    its hot loop's measured cycles per instruction (profiles/valu_cpi.json,
    tools/valu_cpi.py), x its launches per frame; a kernel without a measured
    cost makes it unknown, not a guess."""
    ks = {"gs_blend_px2": {"hbm_bytes_per_launch": 1.0, "SQ_INSTS_VALU": 100.0}}
    cyc, used = bench.stage_valu_cycles("blend", C3_PATHS, ks, {"gs_blend_px2": {"cpi": 2.5}})
    assert (cyc, used) == (250.0, {"gs_blend_px2": 2.5})
    cyc, missing = bench.stage_valu_cycles("blend", C3_PATHS, ks, {})
    assert cyc is None and missing == ["gs_blend_px2"]
    cpi = json.load(open(os.path.join(ROOT, "profiles", "valu_cpi.json")))
    for k in ("gs_blend_px2", "gs_blend", "gs_blend_sort"):
        # between the full-rate (v_mul / v_add: 2) and half-rate (v_fma / v_cmp: 4)
        # costs, and the rates it came from are committed
        assert 2.0 <= cpi[k]["cpi"] <= 4.0 and cpi[k]["loop_valu"] > 0, k
    rates = json.load(open(os.path.join(ROOT, "profiles", "r05_valu", "valu_rate.json")))
    assert any(e["op"] == "v_fma_f32" and e["waves_per_simd"] == 8 for e in rates)


@pytest.mark.parametrize("pmc,paths", [("pmc_c3.json", C3_PATHS), ("pmc_c5.json", C5_PATHS)])
def test_round_pmc_holds_the_default_kernels(pmc, paths):
    """The newest round-end PMC summaries (and profiles/pmc_latest.json, the
    bench's default for config 3) hold every kernel the default frames launch."""
    pp = os.path.join(PROF, pmc)
    if not os.path.exists(pp):
        pytest.skip("round-end profiles not present")
    files = [pp] + ([os.path.join(ROOT, "profiles", "pmc_latest.json")] if pmc == "pmc_c3.json" else [])
    key = bench.pmc_key_of("c3" if pmc == "pmc_c3.json" else "c5", 1_000_000 if pmc == "pmc_c3.json" else 8_000_000,
                           1920 if pmc == "pmc_c3.json" else 3840, 1080 if pmc == "pmc_c3.json" else 2160, 16, 0, 0)
    for f in files:
        d = json.load(open(f))
        # (the several-shape form keyed by bench.pmc_key_of, or round 5's one-summary form)
        kernels = bench.pmc_lookup(f, key)["kernels"] if "summaries" in d else d["kernels"]
        for stage in ("project", "scan", "emit", "sort", "blend") + (("blend_cont",) if paths & bench.PATH_LAZY else ()):
            _, _, missing = bench.stage_pmc(stage, paths, kernels)
            assert not missing, (f, stage, missing)


def _lines_with_survey_model():
    out = []
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r0[4-9]*", "*.json"))):
        try:
            d = json.loads(open(p).read().strip().splitlines()[-1])
        except Exception:
            continue
        if isinstance(d, dict) and "alg_bytes_model" in d.get("roofline", {}):
            out.append((p, d))
    return out


def test_committed_lines_use_the_survey_terms():
    """Every committed bench line of round 4 on: the blend's alg_bytes are
    §8(d)'s T x 8 + rec x 40 + Px x 19 from the line's own fields, and the
    roofline's frac = alg_bytes / avg launch time / 8 TB/s."""
    lines = _lines_with_survey_model()
    if not lines:
        pytest.skip("no round-4 bench line committed yet")
    for p, d in lines:
        k = d["kernels"]["blend"]
        W, H = d["config"]["resolution"]
        if d["config"].get("bands") is None:
            T = d["frame"]["n_tiles"]
            px = W * H
            # (+ the pairs the blend's workgroups sorted, when the sort ran inside it)
            assert k["alg_bytes"] == T * 8 + k["records_staged"] * 40 + px * 19 + k.get("pairs_sorted", 0) * 24, p
        r = d["roofline"]
        dk = d["kernels"][r["kernel"]]
        assert r["alg_bytes_per_launch"] == dk["alg_bytes"], p
        assert abs(r["frac"] - dk["alg_bytes"] / (dk["avg_ms"] * 1e-3) / 8e12) < 2e-3, p


@pytest.mark.parametrize("bands,paths", [
    (8, bench.PATH_BIN_AGG | bench.PATH_BLEND_SORT | bench.PATH_PROJ_BAND),
    (4, bench.PATH_BIN_AGG | bench.PATH_BLEND_SORT | bench.PATH_PROJ_BAND),
    (2, bench.PATH_BIN_AGG | bench.PATH_BLEND_SORT | bench.PATH_PROJ_BAND),
    # a band renderer's frames after its first (direct binning: no scan or emit launch)
    (8, bench.PATH_BIN_AGG | bench.PATH_BLEND_SORT | bench.PATH_BIN_DIRECT),
    (4, bench.PATH_BIN_AGG | bench.PATH_BLEND_SORT | bench.PATH_BIN_DIRECT),
    (2, bench.PATH_BIN_AGG | bench.PATH_BLEND_SORT | bench.PATH_BIN_DIRECT),
    (1, bench.PATH_BLEND_PX2),  # bench.py --gather: the one-GPU group renders the whole frame as band 0 of 1
])
def test_group_line_shapes_resolve_traffic_and_valu(bands, paths):
    """A --gpus N line (rank 0 renders band 0 of N) and the one-GPU group line
    (--gather) find their band shape's PMC summary in the bench's default file
    (bench.pmc_key_of, profiles/pmc_latest.json from tools/r6/pmc_bands.sh), so
    every launched stage has non-null traffic and the blend a VALU fraction."""
    key = bench.pmc_key_of("c3", 1_000_000, 1920, 1080, 16, bands, 0)
    pm = bench.pmc_lookup(os.path.join(ROOT, "profiles", "pmc_latest.json"), key)
    assert pm is not None, key
    kernels = pm["kernels"]
    for stage in ("project", "scan", "emit", "sort", "blend"):
        if not bench.stage_kernels(stage, paths):
            continue  # (a band's tile sort runs inside its blend)
        hb, vi, missing = bench.stage_pmc(stage, paths, kernels)
        assert not missing and hb and hb > 0 and vi, (key, stage, missing)
    cpi = json.load(open(os.path.join(ROOT, "profiles", "valu_cpi.json")))
    cyc, used = bench.stage_valu_cycles("blend", paths, kernels, cpi)
    assert cyc is not None and cyc > 0, (key, used)


def test_binning_named_from_the_frame_paths():
    """The line's config.binning follows gs_frame_stats.paths (a fixed view's
    band frames after the first take the direct binning)."""
    assert bench.binning_of(bench.PATH_BIN_AGG | bench.PATH_BIN_DIRECT).startswith("direct")
    assert bench.binning_of(bench.PATH_BIN_AGG).startswith("aggregated")
    assert bench.binning_of(bench.PATH_BLEND_PX2).startswith("chunked")
    assert bench.binning_of(0, bin_global=True) == "global atomics"
