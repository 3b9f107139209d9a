#!/bin/bash
# Round 4: GPU tests; the band projection's instantiation (A/B against
# tmp_ab/noband) on 8 bands of configs 4 and 5; the aggregated binning on
# config 3 again (after the scan and grid changes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4l2
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['bands'], d['slowest_us'], d['us_per_frame_by_band'], d['slowest_band_stage_us'])"; }
NB=$PWD/tmp_ab/noband/libgsplat.so
for rep in 1 2; do
  echo "== bands c4 band-projection rep $rep $(date +%T)"
  timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_b_$rep.jsonl 2> $O/bands_b_$rep.err || exit $?
  bands $O/bands_b_$rep.jsonl
  echo "== bands c4 generic projection rep $rep $(date +%T)"
  GSPLAT_LIB=$NB timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_g_$rep.jsonl 2> $O/bands_g_$rep.err || exit $?
  bands $O/bands_g_$rep.jsonl
done
echo "== bands c5 band-projection $(date +%T)"
timeout -k 10 500 python tools/band_emulate.py --config5 --balanced --rebalance --inflight 3 --bands 8 > $O/bands_c5_b.jsonl 2> $O/bands_c5_b.err || exit $?
bands $O/bands_c5_b.jsonl
echo "== bands c5 generic projection $(date +%T)"
GSPLAT_LIB=$NB timeout -k 10 500 python tools/band_emulate.py --config5 --balanced --rebalance --inflight 3 --bands 8 > $O/bands_c5_g.jsonl 2> $O/bands_c5_g.err || exit $?
bands $O/bands_c5_g.jsonl
for rep in 1 2; do
  for agg in 0 1; do
    echo "== c3 agg=$agg rep $rep $(date +%T)"
    GSPLAT_BIN_AGG=$agg timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_agg${agg}_$rep.json 2> $O/c3_agg${agg}_$rep.err || exit $?
    line $O/c3_agg${agg}_$rep.json
  done
done
echo "== done $(date +%T)"
