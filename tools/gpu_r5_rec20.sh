#!/bin/bash
# The 20-B record experiment (tools/ab_edits/rec20.py): its valid parity
# cases (16x16 whole frames, chunked binning), then config 3 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r6r20
GSPLAT_LIB=$PWD/tmp_nt/rec20/libgsplat.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread \
  -k "test_synthetic_1080p_16x16 or 16-16-False-False or 16-16-False-True or reference_geometry" > gpurun_out/r6r20/tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r6r20/tests.log; echo "tests rc=$rc"
[ $rc -ge 124 ] && exit $rc
TAG=r6r20 ABDIR=tmp_nt NO_TESTS=1 REPEATS=3 bash tools/ab_r5.sh
