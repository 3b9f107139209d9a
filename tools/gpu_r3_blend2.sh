#!/bin/bash
# Round-3: parity of tmp_ab/blend2 (two tiles per blend workgroup), then the
# interleaved headline A/B of every tmp_ab/ build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
GSPLAT_LIB=$PWD/tmp_ab/blend2/libgsplat.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fast_exp.py -x -q --timeout 300 --timeout-method thread -k "not global and not poison" > gpurun_out/pytest_blend2.txt 2>&1
rc=$?; echo "blend2 tests rc=$rc $(tail -n 1 gpurun_out/pytest_blend2.txt)"; [ $rc -eq 0 ] || exit $rc
REPS=3 bash tools/ab_repeat.sh || exit $?
