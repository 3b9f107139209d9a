#!/bin/bash
# A/B matrix: CASES="name:lib:ENV=VAL,ENV2=VAL2 ..." (lib = a tmp_ab/<lib> build),
# TESTS="-k expr" run once per TESTCASES name, then REPS interleaved rounds of
# the headline bench (and config 5 with C5=1) for every case.
#   CASES="base:base: new:new: pairs:new:GSPLAT_BLEND_PAIRS=1" TESTCASES="pairs" TESTS="lazy or fullsize" C5=1 bash tools/ab_matrix.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
envof() { echo "$1" | tr ',' ' '; }
for c in $CASES; do
  IFS=: read -r name lib ev <<< "$c"
  case " $TESTCASES " in *" $name "*) ;; *) continue ;; esac
  env GSPLAT_LIB=$PWD/tmp_ab/$lib/libgsplat.so $(envof "$ev") timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "${TESTS:-not global_binning}" > gpurun_out/abm_t_$name.log 2>&1
  rc=$?; echo "$name tests rc=$rc $(tail -n 1 gpurun_out/abm_t_$name.log)"
  [ $rc -eq 0 ] || exit $rc
done
summ() {
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
" "$1" "$2"
}
for rep in $(seq ${REPS:-2}); do
  for c in $CASES; do
    IFS=: read -r name lib ev <<< "$c"
    if [ -z "$NO_C3" ]; then
      env GSPLAT_LIB=$PWD/tmp_ab/$lib/libgsplat.so $(envof "$ev") timeout -k 10 300 python bench.py --steps ${STEPS:-600} \
        --warmup 200 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abm_c3_$name.log 2>&1 || exit $?
      summ gpurun_out/abm_c3_$name.log "$rep c3 $name"
    fi
    if [ -n "$C5" ]; then
      env GSPLAT_LIB=$PWD/tmp_ab/$lib/libgsplat.so $(envof "$ev") timeout -k 10 300 python bench.py --config5 \
        --steps ${C5STEPS:-240} --warmup 60 --no-cpu-baseline > gpurun_out/abm_c5_$name.log 2>&1 || exit $?
      summ gpurun_out/abm_c5_$name.log "$rep c5 $name"
    fi
  done
done
