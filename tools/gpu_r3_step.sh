#!/bin/bash
# Round-3 measurement step: full GPU tests, config-5 kernel stats (rocprofv3,
# one frame in flight), headline and config-5 bench lines.  Outputs under
# gpurun_out/r3/.  Each GPU step has its own time limit; the first failure ends
# the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
grep -h "fast exp" $O/pytest_gpu.txt || true
if [ -n "$C5PROF" ]; then
  step c5prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python3 bench.py --config5 --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c5.log 2>&1 || exit $?
fi
step bench
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
cut -c1-400 $O/bench_c3.json
if [ -n "$C5BENCH" ]; then
  step bench_c5
  timeout -k 10 600 python bench.py --config5 --steps 240 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
  cut -c1-300 $O/bench_c5.json
fi
step done
