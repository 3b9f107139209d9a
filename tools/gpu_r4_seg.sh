#!/bin/bash
# Round 4 (re-entry): the two-pixel blend reading each slot's (tile, start,
# length) from the sort launch's table (FrameParams::blend_seg, default)
# against the queue + tile-start reads (GSPLAT_BLEND_SEG=0): GPU tests, then
# config 3 interleaved, three repeats.  Outputs under gpurun_out/r4seg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4seg
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"; }
for rep in 1 2 3; do
  for v in base noseg; do
    case $v in
      base) E="" ;;
      noseg) E="GSPLAT_BLEND_SEG=0" ;;
    esac
    echo "== c3 $v rep $rep $(date +%T)"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
echo "== done $(date +%T)"
