"""Per-stage algorithmic bytes of a bench line against the PMC HBM bytes of
the same stage's kernels (algorithmic bytes <= PMC bytes x 1.1,
or the difference explained).

  python tools/alg_vs_pmc.py <bench line .json> <pmc summary .json>
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bench import STAGE_KERNELS  # noqa: E402


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    pmc = json.load(open(sys.argv[2]))["kernels"]
    print(f"{'stage':12s} {'avg_us':>8s} {'alg MB':>9s} {'PMC MB':>9s} {'alg/PMC':>8s}")
    for stage, k in line["kernels"].items():
        if "alg_bytes" not in k:
            continue
        names = [n for n in STAGE_KERNELS.get(stage, []) if n in pmc]
        hbm = sum(pmc[n]["hbm_bytes_per_launch"] for n in names)
        ratio = k["alg_bytes"] / hbm if hbm else float("nan")
        print(f"{stage:12s} {1e3 * k['avg_ms']:8.1f} {k['alg_bytes'] / 1e6:9.1f} {hbm / 1e6:9.1f} {ratio:8.2f}"
              f"  ({', '.join(names)})")


if __name__ == "__main__":
    main()
