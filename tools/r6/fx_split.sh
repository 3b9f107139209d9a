#!/bin/bash
# Round 6: the direct-binning GPU tests, then the emulated group lines at 2 and
# 4 bands on one GPU (bench.py --split).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6fx
mkdir -p $O
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k direct > $O/pytest.txt 2>&1 || { tail -n 30 $O/pytest.txt; exit 1; }
tail -n 1 $O/pytest.txt
for n in 2 4 8; do
  timeout -k 10 200 python3 bench.py --split $n --steps 300 --warmup 60 --no-cpu-baseline > $O/split$n.json 2> $O/split$n.err
  python3 - $O/split$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], json.dumps(d.get("group"))[:300])
PY
done
