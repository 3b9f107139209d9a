#!/bin/bash
# VALU issue-rate microbenchmark, the band / group / poison parity tests of
# the in-tree library, then interleaved A/Bs: the band emulation against
# tmp_ab_b/ variants and config 3 against tmp_ab/ variants.
# gpurun_out/${TAG:-r5j}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5j}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 60 tools/hip/valu_rate > $O/valu_rate.json || exit $?
cat $O/valu_rate.json
if [ -f tmp_ab_l/lanes/libgsplat.so ]; then
  GSPLAT_LIB=$PWD/tmp_ab_l/lanes/libgsplat.so timeout -k 10 300 python tools/blend_lanes.py --valu 50324476 > $O/blend_lanes.json 2> $O/blend_lanes.err || exit $?
  cat $O/blend_lanes.json
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "band or group or poison or dist or orbit or fullsize" > $O/pytest_band.txt 2>&1
rc=$?; tail -n 3 $O/pytest_band.txt; [ $rc -eq 0 ] || exit $rc
ABDIR=tmp_ab_b NO_TESTS=1 REPEATS=2 TAG=$T/abb bash tools/ab_r5_bands.sh || exit $?
ABDIR=tmp_ab NO_TESTS=1 REPEATS=3 TAG=$T/ab bash tools/ab_r5.sh || exit $?
echo "== done $(date +%T)"
