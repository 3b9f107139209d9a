#!/bin/bash
# Round 4: the blend's packed-fp32 power and colour update (GS_BLEND_PACKED,
# the default build) against the scalar build (tmp_ab/nopk): GPU tests with
# the default build, then interleaved config 3 / config 5 / 8-band A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4pk
mkdir -p $O
echo "== tests (packed) $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['bands'], d['slowest_us'], d['slowest_band_stage_us'])"; }
NOPK=$PWD/tmp_ab/nopk/libgsplat.so
for rep in 1 2 3; do
  echo "== c3 packed rep $rep $(date +%T)"
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_pk_$rep.json 2> $O/c3_pk_$rep.err || exit $?
  line $O/c3_pk_$rep.json
  echo "== c3 scalar rep $rep $(date +%T)"
  GSPLAT_LIB=$NOPK timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_sc_$rep.json 2> $O/c3_sc_$rep.err || exit $?
  line $O/c3_sc_$rep.json
done
echo "== c5 packed $(date +%T)"
timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_pk.json 2> $O/c5_pk.err || exit $?
line $O/c5_pk.json
echo "== c5 scalar $(date +%T)"
GSPLAT_LIB=$NOPK timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_sc.json 2> $O/c5_sc.err || exit $?
line $O/c5_sc.json
echo "== bands c4 packed $(date +%T)"
timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_pk.jsonl 2> $O/bands_pk.err || exit $?
bands $O/bands_pk.jsonl
echo "== bands c4 scalar $(date +%T)"
GSPLAT_LIB=$NOPK timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_sc.jsonl 2> $O/bands_sc.err || exit $?
bands $O/bands_sc.jsonl
echo "== done $(date +%T)"
