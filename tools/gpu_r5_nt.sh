#!/bin/bash
# Streaming (non-temporal) accesses: the GPU suite on the in-tree library,
# then interleaved A/Bs against tmp_nt/ variants on config 3, the 8-band
# emulation and config 5.  Outputs under gpurun_out/${TAG:-r6nt3}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T=${TAG:-r6nt3}
mkdir -p gpurun_out/$T
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
  rc=$?; tail -n 2 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
TAG=${T}b ABDIR=tmp_nt NO_TESTS=1 REPEATS=${REPEATS_B:-2} bash tools/ab_r5_bands.sh || exit $?
TAG=$T ABDIR=tmp_nt NO_TESTS=1 REPEATS=${REPEATS_C3:-3} bash tools/ab_r5.sh || exit $?
