#!/bin/bash
# A/B of one build under environment switches.
#   VAR=GSPLAT_COUNT_ROWDIFF VALS="0 1" TESTS="parity or fullsize" REPS=2 C5=1 bash tools/ab_env.sh
# 1. GPU tests (-k $TESTS) with the LAST value of VALS forced;
# 2. REPS interleaved rounds of the headline bench (and config 5 with C5=1)
#    for every value.  Each GPU step has its own time limit; a failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
last=${VALS##* }
if [ -n "$TESTS" ]; then
  env $VAR=$last timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "$TESTS" > gpurun_out/abenv_tests.log 2>&1
  rc=$?; echo "tests $VAR=$last rc=$rc $(tail -n 1 gpurun_out/abenv_tests.log)"
  [ $rc -eq 0 ] || exit $rc
fi
summ() {
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
" "$1" "$2"
}
for rep in $(seq ${REPS:-2}); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps ${STEPS:-600} --warmup 200 --no-cpu-baseline \
      > gpurun_out/abenv_c3_$v.log 2>&1 || exit $?
    summ gpurun_out/abenv_c3_$v.log "c3 $VAR=$v"
    if [ -n "$C5" ]; then
      env $VAR=$v timeout -k 10 300 python bench.py --config5 --steps ${C5STEPS:-240} --warmup 60 --no-cpu-baseline \
        > gpurun_out/abenv_c5_$v.log 2>&1 || exit $?
      summ gpurun_out/abenv_c5_$v.log "c5 $VAR=$v"
    fi
  done
done
