"""Per-stage bytes of a bench line against the PMC HBM bytes of the same
stage's kernels: the SURVEY §8(d) algorithmic bytes (the roofline's, bench.
survey_bytes) and the layout bytes the kernels move (bench.layout_bytes,
which should stay within 1.1x of the PMC bytes).

  python tools/alg_vs_pmc.py <bench line .json> <pmc summary .json>
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bench import stage_pmc, stage_kernels  # noqa: E402


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    pmc = json.load(open(sys.argv[2]))["kernels"]
    print(f"{'stage':12s} {'avg_us':>8s} {'8d MB':>9s} {'layout MB':>10s} {'PMC MB':>9s} {'PMC/8d':>8s} "
          f"{'layout/PMC':>10s}")
    for stage, k in line["kernels"].items():
        if "alg_bytes" not in k:
            continue
        lb = k.get("layout_bytes", k["alg_bytes"])
        paths, bg = line["frame"].get("paths", 0), bool(line["frame"].get("bin_global", 0))
        hbm, _, missing = stage_pmc(stage, paths, pmc, bg)
        names = [f"{n} x{c}" for n, c in stage_kernels(stage, paths, bg)]
        if missing:
            print(f"{stage:12s} PMC summary lacks {', '.join(missing)}")
            continue
        r8 = hbm / k["alg_bytes"] if k["alg_bytes"] else float("nan")
        rl = lb / hbm if hbm else float("nan")
        print(f"{stage:12s} {1e3 * k['avg_ms']:8.1f} {k['alg_bytes'] / 1e6:9.1f} {lb / 1e6:10.1f} {hbm / 1e6:9.1f} "
              f"{r8:8.2f} {rl:10.2f}  ({', '.join(names)})")


if __name__ == "__main__":
    main()
