#!/bin/bash
# Round-5 start (one call): GPU tests, smoke, rocprofv3 stats + PMC of config
# 3 (tools/round_profile.sh) with its bench line, then the driver-shaped line
# reading the fresh PMC summary.  Outputs under gpurun_out/r5s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
cat $O/smoke.txt
echo "== profiles c3 $(date +%T)"
WORKLOADS=c3 bash tools/round_profile.sh || exit $?
echo "== driver-shaped bench $(date +%T)"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc-json gpurun_out/pmc_c3.json > $O/bench_driver_shaped.json 2> $O/bench_driver_shaped.err || exit $?
cut -c1-300 $O/bench_driver_shaped.json
echo "== done $(date +%T)"
