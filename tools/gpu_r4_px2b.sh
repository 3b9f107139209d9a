#!/bin/bash
# Round 4: two pixels per lane, all tiles (GSPLAT_BLEND_PX2=1) or only the
# short lists (=2; tmp_ab/px2h73 without the 7-waves cap) -- GPU tests, then
# config 3 interleaved, three repeats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4px2b
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
H73=$PWD/tmp_ab/px2h73/libgsplat.so
for rep in 1 2 3; do
  for v in base px2 px2h px2h73; do
    echo "== c3 $v rep $rep $(date +%T)"
    case $v in
      base) E="" ;;
      px2) E="GSPLAT_BLEND_PX2=1" ;;
      px2h) E="GSPLAT_BLEND_PX2=2" ;;
      px2h73) E="GSPLAT_BLEND_PX2=2 GSPLAT_LIB=$H73" ;;
    esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
for rep in 1 2; do
  for v in base px2h; do
    echo "== c5 $v rep $rep $(date +%T)"
    case $v in
      base) E="" ;;
      px2h) E="GSPLAT_BLEND_PX2=2" ;;
    esac
    env $E timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit $?
    line $O/c5_${v}_$rep.json
  done
done
echo "== done $(date +%T)"
