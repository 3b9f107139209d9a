#!/bin/bash
# Round 4 (re-entry): config 5 (lazy frames, one pixel per lane) with the
# blend's tiles longest list first (GSPLAT_BLEND_LPT=1) against the tile
# order; interleaved, three repeats.  Outputs under gpurun_out/r4c5lpt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4c5lpt
mkdir -p $O
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"; }
for rep in 1 2 3; do
  for v in base lpt; do
    E=""
    case $v in
      lpt) E="GSPLAT_BLEND_LPT=1" ;;
    esac
    echo "== c5 $v rep $rep $(date +%T)"
    env $E timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit $?
    line $O/c5_${v}_$rep.json
  done
done
echo "== done $(date +%T)"
