#!/bin/bash
# GPU tests + smoke + quick default / config-5 / group bench lines.
# Outputs under gpurun_out/${TAG:-r5c}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5c}
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
cat $O/smoke.txt
echo "== bench default $(date +%T)"
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit $?
cut -c1-200 $O/bench_default.json
echo "== bench c5 $(date +%T)"
timeout -k 10 600 python bench.py --config5 --steps 240 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c1-200 $O/bench_c5.json
echo "== bench gather $(date +%T)"
timeout -k 10 600 python bench.py --gather --no-cpu-baseline > $O/bench_gather.json 2> $O/bench_gather.err || exit $?
cut -c1-200 $O/bench_gather.json
echo "== done $(date +%T)"
