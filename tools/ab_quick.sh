#!/bin/bash
# GPU parity tests (TESTS, a pytest -k expression) for each tmp_ab/<name>
# build, then interleaved headline benches (tools/ab_repeat.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for d in tmp_ab/*/; do
  n=$(basename "$d")
  GSPLAT_LIB=$PWD/$d/libgsplat.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTS:-not global_binning}" > gpurun_out/abt_$n.log 2>&1
  rc=$?; echo "$n tests rc=$rc $(tail -n 1 gpurun_out/abt_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
REPS=${REPS:-2} bash tools/ab_repeat.sh
