#!/bin/bash
# Round 4: config 3 against the round-start library (tmp_ab/r4start, commit
# 73cb6ff), interleaved on one box, and the default build with the walking
# grids off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4rg
mkdir -p $O
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], d['roofline'].get('peak_measured'), {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
for rep in 1 2 3; do
  for v in now start nogrid; do
    echo "== c3 $v rep $rep $(date +%T)"
    case $v in
      now) E="" ;;
      start) E="GSPLAT_LIB=$PWD/tmp_ab/r4start/libgsplat.so" ;;
      nogrid) E="GSPLAT_PROJECT_GRID=0 GSPLAT_EMIT_GRID=0" ;;
    esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
for v in now start; do
  echo "== c5 $v $(date +%T)"
  case $v in
    now) E="" ;;
    start) E="GSPLAT_LIB=$PWD/tmp_ab/r4start/libgsplat.so" ;;
  esac
  env $E timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_$v.json 2> $O/c5_$v.err || exit $?
  line $O/c5_$v.json
done
echo "== done $(date +%T)"
