#!/bin/bash
# Round 4: the 48-B record with the colour in it (GSPLAT_REC48=1) against
# the 32-B record + colour gather: GPU tests, interleaved config 3 / config 5
# / 8-band A/B, and FETCH / WRITE passes of config 3 for both (the blend's
# HBM bytes per launch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4r48
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['bands'], d['slowest_us'], d['slowest_band_stage_us'])"; }
for rep in 1 2 3; do
  for v in 0 1; do
    echo "== c3 rec48=$v rep $rep $(date +%T)"
    GSPLAT_REC48=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_r${v}_$rep.json 2> $O/c3_r${v}_$rep.err || exit $?
    line $O/c3_r${v}_$rep.json
  done
done
for v in 0 1; do
  echo "== c5 rec48=$v $(date +%T)"
  GSPLAT_REC48=$v timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_r$v.json 2> $O/c5_r$v.err || exit $?
  line $O/c5_r$v.json
  echo "== bands c4 rec48=$v $(date +%T)"
  GSPLAT_REC48=$v timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_r$v.jsonl 2> $O/bands_r$v.err || exit $?
  bands $O/bands_r$v.jsonl
done
for g in 0 2048; do
  echo "== c5 project grid $g $(date +%T)"
  GSPLAT_PROJECT_GRID=$g timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_pg$g.json 2> $O/c5_pg$g.err || exit $?
  line $O/c5_pg$g.json
done
for v in 0 1; do
  echo "== PMC c3 rec48=$v $(date +%T)"
  GSPLAT_REC48=$v NAME=c3_r48_$v BENCH_ARGS="--inflight 1" PASSES="fetch write" bash tools/profile.sh || exit $?
  python3 tools/pmc_summary.py gpurun_out/prof_c3_r48_$v --json $O/pmc_c3_r48_$v.json > $O/pmc_summary_c3_r48_$v.txt || exit $?
  grep -E "gs_blend|gs_project" $O/pmc_summary_c3_r48_$v.txt | cut -c1-200
done
echo "== done $(date +%T)"
