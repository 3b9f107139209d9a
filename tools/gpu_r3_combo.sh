#!/bin/bash
# Round-3 combined call: slice parity tests, the config-5 slice A/B
# (tools/gpu_r3_slices.sh without its tests), the tmp_ab/ blend variants
# (tools/ab_repeat.sh) and the warm-up A/B (tools/gpu_r3_warm.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -k "slices or config5" > gpurun_out/r3s/pytest.txt 2>&1
rc=$?; tail -n 3 gpurun_out/r3s/pytest.txt; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash tools/gpu_r3_slices.sh || exit $?
echo "== blend variants $(date +%T)"
REPS=2 bash tools/ab_repeat.sh || exit $?
echo "== warm-up $(date +%T)"
bash tools/gpu_r3_warm.sh || exit $?
echo "== done $(date +%T)"
