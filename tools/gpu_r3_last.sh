#!/bin/bash
# Round-3 last measurement of the final tree: smoke(), config-5 rocprofv3
# kernel stats + FETCH/WRITE PMC passes (tools/round_profile.sh, c5 only), the
# config-5 line that reads them, and the default headline line.  Outputs under
# gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.txt 2>&1 || { tail -5 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
echo "== c5 profile $(date +%T)"
WORKLOADS=c5 PASSES="stats fetch write sq1" bash tools/round_profile.sh || exit $?
echo "== default bench $(date +%T)"
timeout -k 10 600 python bench.py > gpurun_out/bench_default_last.json 2> gpurun_out/bench_default_last.err || exit $?
cut -c1-250 gpurun_out/bench_default_last.json
echo "== driver-shaped $(date +%T)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_s20w5_last.json 2>> gpurun_out/bench_default_last.err || exit $?
cut -c1-250 gpurun_out/bench_s20w5_last.json
echo "== done $(date +%T)"
