#!/bin/bash
# The GPU suite on the in-tree library, then config 5 A/B (tools/gpu_r5_c5.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T=${TAG:-r6c5t}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=$T bash tools/gpu_r5_c5.sh
