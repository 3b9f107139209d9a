#!/bin/bash
# Round-4 end set, part A: GPU tests, smoke, rocprofv3 kernel stats + PMC
# passes of configs 3 and 5 (tools/round_profile.sh, which also prints the
# bench lines that read the fresh counters), the FETCH_SIZE calibration.
# Outputs under gpurun_out/ (copied to profiles/r04_end/ by hand).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_end.txt 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_gpu_end.txt; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit $?
cat gpurun_out/smoke.txt
echo "== profiles $(date +%T)"
PASSES="${PASSES:-stats fetch write sq1 lds}" bash tools/round_profile.sh || exit $?
echo "== FETCH_SIZE calibration $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o calib --output-format csv -- tools/hip/fetch_calib > gpurun_out/calib.log 2>&1 || exit $?
python3 tools/fetch_calib.py gpurun_out/calib --json gpurun_out/fetch_calib.json
echo "== done $(date +%T)"
