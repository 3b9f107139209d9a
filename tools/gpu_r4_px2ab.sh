#!/bin/bash
# Round 4 (re-entry): A/Bs of the two-pixel blend that the tree carries as
# hooks -- whole frames in LPT order (GSPLAT_BLEND_LPT=1), whole frames with
# the sort inside a two-pixel blend (GSPLAT_BLEND_SORT=1 GSPLAT_BAND_PX2=1),
# and 8 row bands of config 4 with two-pixel lanes (GSPLAT_BAND_PX2=1);
# the two-pixel step without the interleaved decisions (tmp_ab/px2il0) and
# with branch-free colour updates (tmp_ab/px2bf);
# interleaved repeats.  Outputs under gpurun_out/r4px2ab.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4px2ab
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
cat $O/smoke.txt
IL0=$PWD/tmp_ab/px2il0/libgsplat.so
BF=$PWD/tmp_ab/px2bf/libgsplat.so
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"; }
for rep in 1 2 3; do
  for v in base il0 bf lpt bsort; do
    case $v in
      base) E="" ;;
      il0) E="GSPLAT_LIB=$IL0" ;;
      bf) E="GSPLAT_LIB=$BF" ;;
      lpt) E="GSPLAT_BLEND_LPT=1" ;;
      bsort) E="GSPLAT_BLEND_SORT=1 GSPLAT_BAND_PX2=1" ;;
    esac
    echo "== c3 $v rep $rep $(date +%T)"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
  for v in base bpx2; do
    case $v in
      base) E="" ;;
      bpx2) E="GSPLAT_BAND_PX2=1" ;;
    esac
    echo "== bands c4 $v rep $rep $(date +%T)"
    env $E timeout -k 10 300 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/b8_${v}_$rep.jsonl 2> $O/b8_${v}_$rep.err || exit $?
    cut -c1-260 $O/b8_${v}_$rep.jsonl
  done
done
echo "== done $(date +%T)"
