#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, short bench.  Every GPU step
# has its own time limit; a crash/timeout (rc >= 124 or signal) stops the run.
#   TESTS="tests/test_gpu_fullsize.py" (default: every -m gpu test)  BENCH_ARGS=...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread
step bench 600 python bench.py --steps ${STEPS:-200} --warmup 10 ${BENCH_ARGS:-}
