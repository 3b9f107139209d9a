#!/bin/bash
# Round 4 (re-entry): the two-pixel record loop as a wave-uniform loop
# (GS_PX2_UNIFORM, tmp_ab/px2uni) -- its GPU parity suite, then config 3
# interleaved against the default library, three repeats.  Outputs under
# gpurun_out/r4uni.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4uni
mkdir -p $O
U=$PWD/tmp_ab/px2uni/libgsplat.so
echo "== tests on px2uni $(date +%T)"
GSPLAT_LIB=$U timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "px2 or fullsize or blend" > $O/pytest_gpu_uni.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu_uni.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"; }
for rep in 1 2 3; do
  for v in base uni; do
    case $v in
      base) E="" ;;
      uni) E="GSPLAT_LIB=$U" ;;
    esac
    echo "== c3 $v rep $rep $(date +%T)"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
echo "== done $(date +%T)"
