#!/bin/bash
# Round 4: after the per-block projection instantiations -- GPU tests, then
# configs 3 / 5 and 8-band configs 4 / 5 against the round-start library
# (tmp_ab/r4start) and the walking projection (GSPLAT_PROJECT_GRID=2048),
# interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4rg2
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['roofline'].get('peak_measured'), {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['bands'], d['slowest_us'], d['us_per_frame_by_band'], d['slowest_band_stage_us'])"; }
ST=$PWD/tmp_ab/r4start/libgsplat.so
for rep in 1 2 3; do
  for v in now start walk; do
    echo "== c3 $v rep $rep $(date +%T)"
    case $v in
      now) E="" ;;
      start) E="GSPLAT_LIB=$ST" ;;
      walk) E="GSPLAT_PROJECT_GRID=2048" ;;
    esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
for v in now start walk; do
  case $v in
    now) E="" ;;
    start) E="GSPLAT_LIB=$ST" ;;
    walk) E="GSPLAT_PROJECT_GRID=2048" ;;
  esac
  echo "== c5 $v $(date +%T)"
  env $E timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_$v.json 2> $O/c5_$v.err || exit $?
  line $O/c5_$v.json
  echo "== bands c4 $v $(date +%T)"
  env $E timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_c4_$v.jsonl 2> $O/bands_c4_$v.err || exit $?
  bands $O/bands_c4_$v.jsonl
done
for v in now start; do
  case $v in
    now) E="" ;;
    start) E="GSPLAT_LIB=$ST" ;;
  esac
  echo "== bands c5 $v $(date +%T)"
  env $E timeout -k 10 500 python tools/band_emulate.py --config5 --balanced --rebalance --inflight 3 --bands 8 > $O/bands_c5_$v.jsonl 2> $O/bands_c5_$v.err || exit $?
  bands $O/bands_c5_$v.jsonl
done
echo "== done $(date +%T)"
