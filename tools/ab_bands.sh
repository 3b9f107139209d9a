#!/bin/bash
# For every tmp_ab/<name>/libgsplat.so: the 8-band critical path on one GPU
# (tools/band_emulate.py), after tools/ab_libs.sh has run its tests/bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for d in tmp_ab/*/; do
  n=$(basename "$d")
  GSPLAT_LIB=$PWD/$d/libgsplat.so timeout -k 10 300 python tools/band_emulate.py --bands ${BANDS:-8} --steps 60 > gpurun_out/abb_$n.log 2>&1 || { tail -3 gpurun_out/abb_$n.log; exit 1; }
  echo "$n $(grep bands gpurun_out/abb_$n.log)"
done
