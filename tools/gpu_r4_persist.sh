#!/bin/bash
# Round 4: the LDS-scheduled persistent blend (GSPLAT_BLEND_PERSIST=G) against
# the one-workgroup-per-tile blend: parity of the variant, then interleaved
# bench lines at configs 3 and 5.  Outputs under gpurun_out/r4p/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
echo "== parity with the persistent blend $(date +%T)"
GSPLAT_BLEND_PERSIST=512 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_persist.txt 2>&1
rc=$?; tail -n 2 $O/pytest_persist.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
for rep in 1 2; do
  for g in 0 512 768; do
    echo "== c3 persist=$g rep $rep $(date +%T)"
    GSPLAT_BLEND_PERSIST=$g timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_p${g}_$rep.json 2> $O/c3_p${g}_$rep.err || exit $?
    line $O/c3_p${g}_$rep.json
  done
done
for g in 0 512; do
  echo "== c5 persist=$g $(date +%T)"
  GSPLAT_BLEND_PERSIST=$g timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_p$g.json 2> $O/c5_p$g.err || exit $?
  line $O/c5_p$g.json
done
echo "== done $(date +%T)"
