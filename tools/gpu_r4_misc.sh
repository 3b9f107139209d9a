#!/bin/bash
# Round 4 (re-entry): zero-code A/Bs of the two-pixel default -- the 48-B
# record with the colour co-located (GSPLAT_REC48=1) and 2 / 4 frames in
# flight against the default 3; config 3, interleaved, three repeats.
# Outputs under gpurun_out/r4misc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4misc
mkdir -p $O
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['avg_launch_ms'], r.get('traffic'), {k:round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"; }
for rep in 1 2 3; do
  for v in base rec48 f2 f4; do
    A=""; E=""
    case $v in
      rec48) E="GSPLAT_REC48=1" ;;
      f2) A="--inflight 2" ;;
      f4) A="--inflight 4" ;;
    esac
    echo "== c3 $v rep $rep $(date +%T)"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline $A > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
echo "== done $(date +%T)"
