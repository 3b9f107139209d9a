#!/bin/bash
# GPU session for the row-band group: its parity tests, then the bench through
# the group paths (world-1 RCCL, 8 emulated bands) and the default headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step group_tests 400 python -u -m pytest ${TESTS:-tests/test_gpu_group.py} -m gpu -x -v --timeout 200 --timeout-method thread
step bench_gather 300 python bench.py --gather --steps 200 --warmup 10 --no-cpu-baseline
step bench_split8 300 python bench.py --split 8 --steps 200 --warmup 10 --no-cpu-baseline
step bench 400 python bench.py --steps 300 --warmup 10 ${BENCH_ARGS:-}
