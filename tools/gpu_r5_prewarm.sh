#!/bin/bash
# The driver-shaped line (--steps 20 --warmup 5) with untimed pre-warm frames
# of several lengths.  Outputs under gpurun_out/r5pw.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r5pw
mkdir -p $O
for pw in 0 10 25 50 100 0 25 50; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --prewarm-ms $pw --no-cpu-baseline > $O/bench_pw$pw.json 2> $O/bench_pw$pw.err || exit $?
  python3 - $O/bench_pw$pw.json "$pw" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("prewarm_ms", sys.argv[2], d["prewarm"], d["value"], d["ms_per_step"])
PY
done
