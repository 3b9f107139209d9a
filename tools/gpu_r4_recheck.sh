#!/bin/bash
# Re-entry check of the tree as committed: GPU tests, smoke, config-3 kernel
# stats + PMC (tools/round_profile.sh) and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4re
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
cat $O/smoke.txt
echo "== profiles $(date +%T)"
WORKLOADS="${WORKLOADS:-c3}" PASSES="stats fetch write sq1" bash tools/round_profile.sh || exit $?
echo "== default bench $(date +%T)"
timeout -k 10 600 python bench.py --pmc-json gpurun_out/pmc_c3.json > $O/bench_default.json 2> $O/bench_default.err || exit $?
cut -c1-400 $O/bench_default.json
echo "== driver-shaped bench $(date +%T)"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc-json gpurun_out/pmc_c3.json > $O/bench_driver_shaped.json 2> $O/bench_driver_shaped.err || exit $?
cut -c1-200 $O/bench_driver_shaped.json
echo "== done $(date +%T)"
