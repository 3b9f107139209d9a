#!/bin/bash
# Round-3 A/B: GPU parity tests (TESTS) of the builds named in $TESTED, then
# interleaved headline benches of every tmp_ab/<name> build (tools/ab_repeat.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for n in $TESTED; do
  GSPLAT_LIB=$PWD/tmp_ab/$n/libgsplat.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTS:-not global_binning}" > gpurun_out/abt_$n.log 2>&1
  rc=$?; echo "$n tests rc=$rc $(tail -n 1 gpurun_out/abt_$n.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
REPS=${REPS:-2} bash tools/ab_repeat.sh
