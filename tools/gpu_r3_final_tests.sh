#!/bin/bash
# Round-3: full GPU tests of the tree, then the 8-band A/B of tmp_ab/ builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_final.txt 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_gpu_final.txt; [ $rc -eq 0 ] || exit $rc
if [ -n "$BANDS_AB" ]; then
  echo "== band A/B $(date +%T)"
  GSPLAT_LIB=$PWD/tmp_ab/bandproj4/libgsplat.so timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "band or group" > gpurun_out/pytest_bandproj4.txt 2>&1
  rc=$?; tail -n 1 gpurun_out/pytest_bandproj4.txt; [ $rc -eq 0 ] || exit $rc
  REPS=2 bash tools/ab_bands8.sh || exit $?
fi
echo "== done $(date +%T)"
