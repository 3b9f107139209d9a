#!/bin/bash
# Round 4: config 5's lazy-continuation pass-2 grids (GSPLAT_PASS2_GRID)
# 256 / 1024 / 4096, interleaved, two repeats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4p2
mkdir -p $O
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
for rep in 1 2; do
  for g in 256 1024 4096; do
    echo "== c5 pass-2 grid $g rep $rep $(date +%T)"
    GSPLAT_PASS2_GRID=$g timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_g${g}_$rep.json 2> $O/c5_g${g}_$rep.err || exit $?
    line $O/c5_g${g}_$rep.json
  done
done
echo "== done $(date +%T)"
