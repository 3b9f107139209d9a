#!/bin/bash
# Round 4, third A/B: the aggregated binning with the histogram kept on the
# device, auto-selected by tile count; configs 3 / 5, 8-band emulations of
# configs 4 / 5 (agg vs chunked), and a kernel trace of one pipelined band.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4agg3
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['bands'], d['slowest_us'], d['us_per_frame_by_band'], d['slowest_band_stage_us'])"; }
for rep in 1 2; do
  for agg in 1 0; do
    echo "== c3 agg=$agg rep $rep $(date +%T)"
    GSPLAT_BIN_AGG=$agg timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_agg${agg}_$rep.json 2> $O/c3_agg${agg}_$rep.err || exit $?
    line $O/c3_agg${agg}_$rep.json
  done
done
for agg in 1 0; do
  echo "== bands c4 agg=$agg $(date +%T)"
  GSPLAT_BIN_AGG=$agg timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_c4_agg$agg.jsonl 2> $O/bands_c4_agg$agg.err || exit $?
  bands $O/bands_c4_agg$agg.jsonl
done
echo "== c5 auto $(date +%T)"
timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit $?
line $O/c5.json
for agg in 1 0; do
  echo "== bands c5 agg=$agg $(date +%T)"
  GSPLAT_BIN_AGG=$agg timeout -k 10 500 python tools/band_emulate.py --config5 --balanced --rebalance --inflight 3 --bands 8 > $O/bands_c5_agg$agg.jsonl 2> $O/bands_c5_agg$agg.err || exit $?
  bands $O/bands_c5_agg$agg.jsonl
done
echo "== trace band 3 of 8 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_band3 -o band3 --output-format csv -- python3 tools/band_emulate.py --balanced --inflight 3 --bands 8 --only-band 3 --steps 200 > $O/trace_band3.log 2>&1 || exit $?
echo "== FETCH_SIZE calibration $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/calib -o calib --output-format csv -- tools/hip/fetch_calib > $O/calib.log 2>&1 || exit $?
python3 tools/fetch_calib.py $O/calib --json $O/fetch_calib.json
echo "== done $(date +%T)"
