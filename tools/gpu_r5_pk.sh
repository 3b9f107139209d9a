#!/bin/bash
# VALU per-instruction rates, the whole GPU test suite with the in-tree
# library, then an interleaved config-3 A/B against tmp_ab/ variants.
# gpurun_out/${TAG:-r5k}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5k}
O=gpurun_out/$T
mkdir -p $O
if [ -n "$VALU" ]; then
  timeout -k 10 120 tools/hip/valu_rate > $O/valu_rate.json || exit $?
  tail -n 14 $O/valu_rate.json
fi
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== ab $(date +%T)"
ABDIR=tmp_ab REPEATS=${REPEATS:-3} TAG=$T/ab bash tools/ab_r5.sh || exit $?
echo "== done $(date +%T)"
