#!/bin/bash
# Round 6 closing check of the committed tree: GPU suite, smoke, the
# driver-shaped default bench line, 1- and 8-band config 4 emulation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6check
mkdir -p $O
set -e
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -n 30 $O/pytest_gpu.txt; exit 1; }
tail -n 1 $O/pytest_gpu.txt
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 && tail -n 1 $O/smoke.txt
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
python3 - $O/bench_default.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("default", d["value"], d["ms_per_step"], r.get("kernel"), r.get("frac"), r.get("traffic"), d["cpu_baseline"]["value"])
PY
timeout -k 10 300 python3 tools/band_emulate.py --balanced --inflight 3 > $O/bands_c4.jsonl 2> $O/bands_c4.err
tail -n 1 $O/bands_c4.jsonl | cut -c1-300
