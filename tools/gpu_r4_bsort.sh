#!/bin/bash
# Round 4: the tile sort inside the blend's workgroups (GSPLAT_BLEND_SORT,
# default on) and the packed-fp32 blend step (tmp_ab/nopk: the scalar step):
# GPU tests, interleaved config 3 / config 5 / 8-band A/B, then the band
# period against frames in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4bs
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['bands'], d['slowest_us'], d['slowest_band_stage_us'])"; }
NOPK=$PWD/tmp_ab/nopk/libgsplat.so
for rep in 1 2 3; do
  echo "== c3 sort-in-blend rep $rep $(date +%T)"
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_bs_$rep.json 2> $O/c3_bs_$rep.err || exit $?
  line $O/c3_bs_$rep.json
  echo "== c3 sort launch rep $rep $(date +%T)"
  GSPLAT_BLEND_SORT=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_sl_$rep.json 2> $O/c3_sl_$rep.err || exit $?
  line $O/c3_sl_$rep.json
  echo "== c3 sort-in-blend, scalar step rep $rep $(date +%T)"
  GSPLAT_LIB=$NOPK timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_np_$rep.json 2> $O/c3_np_$rep.err || exit $?
  line $O/c3_np_$rep.json
done
echo "== c5 sort-in-blend $(date +%T)"
timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_bs.json 2> $O/c5_bs.err || exit $?
line $O/c5_bs.json
echo "== c5 sort launch $(date +%T)"
GSPLAT_BLEND_SORT=0 timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_sl.json 2> $O/c5_sl.err || exit $?
line $O/c5_sl.json
for v in bs sl; do
  echo "== bands c4 $v $(date +%T)"
  if [ $v = sl ]; then export GSPLAT_BLEND_SORT=0; fi
  timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_$v.jsonl 2> $O/bands_$v.err || exit $?
  unset GSPLAT_BLEND_SORT
  bands $O/bands_$v.jsonl
done
for f in 1 2 4 5 6; do
  echo "== band 3 of 8, inflight $f $(date +%T)"
  timeout -k 10 300 python tools/band_emulate.py --balanced --inflight $f --bands 8 --only-band 3 --steps 400 > $O/f$f.jsonl 2> $O/f$f.err || exit $?
  bands $O/f$f.jsonl
done
echo "== done $(date +%T)"
