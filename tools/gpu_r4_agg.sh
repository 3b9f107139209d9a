#!/bin/bash
# Round 4: the aggregated binning (default) against the chunked binning
# (GSPLAT_BIN_AGG=0): GPU tests, then interleaved bench lines of configs 3 and
# 5 and the 8-band emulation of config 4.  Outputs under gpurun_out/r4agg/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4agg
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for agg in 1 0; do
    echo "== c3 agg=$agg rep $rep $(date +%T)"
    GSPLAT_BIN_AGG=$agg timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_agg${agg}_$rep.json 2> $O/c3_agg${agg}_$rep.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$O/c3_agg${agg}_$rep.json').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
  done
done
for agg in 1 0; do
  echo "== bands agg=$agg $(date +%T)"
  GSPLAT_BIN_AGG=$agg timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 1,8 > $O/bands_agg$agg.jsonl 2> $O/bands_agg$agg.err || exit $?
  cut -c1-300 $O/bands_agg$agg.jsonl
done
for agg in 1 0; do
  echo "== c5 agg=$agg $(date +%T)"
  GSPLAT_BIN_AGG=$agg timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_agg$agg.json 2> $O/c5_agg$agg.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/c5_agg$agg.json').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
echo "== done $(date +%T)"
