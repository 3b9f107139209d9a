#!/bin/bash
# Round 4, second A/B: aggregated binning (coalesced scan, run-aggregated emit
# slots) and the compacting band projection, against their A/B switches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4agg2
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
for rep in 1 2; do
  for agg in 1 0; do
    echo "== c3 agg=$agg rep $rep $(date +%T)"
    GSPLAT_BIN_AGG=$agg timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_agg${agg}_$rep.json 2> $O/c3_agg${agg}_$rep.err || exit $?
    line $O/c3_agg${agg}_$rep.json
  done
done
for v in "1 1" "1 0" "0 1" "0 0"; do
  set -- $v
  echo "== bands agg=$1 compact=$2 $(date +%T)"
  GSPLAT_BIN_AGG=$1 GSPLAT_BAND_COMPACT=$2 timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_agg$1_cmp$2.jsonl 2> $O/bands_agg$1_cmp$2.err || exit $?
  python3 -c "
import json
for l in open('$O/bands_agg$1_cmp$2.jsonl'):
    d=json.loads(l); print(d['bands'], d['slowest_us'], d['us_per_frame_by_band'], d['slowest_band_stage_us'])"
done
for agg in 1 0; do
  echo "== c5 agg=$agg $(date +%T)"
  GSPLAT_BIN_AGG=$agg timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_agg$agg.json 2> $O/c5_agg$agg.err || exit $?
  line $O/c5_agg$agg.json
done
echo "== done $(date +%T)"
