#!/bin/bash
# One round-end measurement: kernel stats + PMC passes (one frame in flight),
# the pipelined kernel trace (tools/overlap.py) and the bench line with the
# fresh PMC traffic.  Outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
set -e
export TMPDIR=/tmp
BENCH_ARGS="--inflight 1" PASSES="stats fetch write sq1" STEPS=20 bash tools/profile.sh > gpurun_out/profile.log 2>&1
python3 tools/pmc_summary.py gpurun_out/prof --json gpurun_out/pmc.json > gpurun_out/pmc_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ov -o ov --output-format csv -- python3 bench.py --steps 400 --no-cpu-baseline > gpurun_out/ov.log 2>&1
python3 tools/overlap.py $(find gpurun_out/ov -name "*kernel_trace.csv") > gpurun_out/overlap.txt
timeout -k 10 400 python3 bench.py --pmc-json gpurun_out/pmc.json > gpurun_out/bench.json.log 2>&1
grep '"metric"' gpurun_out/bench.json.log | cut -c1-400
cat gpurun_out/overlap.txt
