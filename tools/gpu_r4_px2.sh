#!/bin/bash
# Round 4: two pixels per blend lane (GSPLAT_BLEND_PX2=1; tmp_ab/px2w8: the
# same capped at 64 VGPRs) -- GPU tests, then config 3 interleaved, and 8
# bands of config 4 with the sort launch (px2) against the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4px2
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, d['kernels']['blend'].get('records_staged'))"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['bands'], d['slowest_us'], d['us_per_frame_by_band'], d['slowest_band_stage_us'])"; }
W8=$PWD/tmp_ab/px2w8/libgsplat.so
for rep in 1 2 3; do
  for v in base px2 px2w8; do
    echo "== c3 $v rep $rep $(date +%T)"
    case $v in
      base) E="" ;;
      px2) E="GSPLAT_BLEND_PX2=1" ;;
      px2w8) E="GSPLAT_BLEND_PX2=1 GSPLAT_LIB=$W8" ;;
    esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
for v in base px2; do
  echo "== bands c4 $v $(date +%T)"
  case $v in
    base) E="" ;;
    px2) E="GSPLAT_BLEND_PX2=1 GSPLAT_BLEND_SORT=0" ;;
  esac
  env $E timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_$v.jsonl 2> $O/bands_$v.err || exit $?
  bands $O/bands_$v.jsonl
done
echo "== done $(date +%T)"
