#!/bin/bash
# Round-3 end measurement set of the current tree: GPU tests, rocprofv3 kernel
# stats + PMC passes per workload (tools/round_profile.sh), and the default
# bench line (with the CPU baseline) that reads the fresh counters.  Outputs
# under gpurun_out/ (copied to profiles/r03_end/ by hand).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_end.txt 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_gpu_end.txt; [ $rc -eq 0 ] || exit $rc
echo "== profiles $(date +%T)"
PASSES="${PASSES:-stats fetch write sq1 lds}" bash tools/round_profile.sh || exit $?
echo "== default bench $(date +%T)"
timeout -k 10 600 python bench.py --pmc-json gpurun_out/pmc_c3.json > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
cut -c1-300 gpurun_out/bench_default.json
echo "== done $(date +%T)"
