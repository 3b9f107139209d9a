#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, short bench.  Every GPU step
# has its own time limit; a crash/timeout (rc >= 124 or signal) stops the run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step build 600 python -c "import __graft_entry__ as g; g.build()"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q --timeout 300
step bench 600 python bench.py --steps 50 --warmup 5
