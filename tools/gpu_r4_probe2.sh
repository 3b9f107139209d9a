#!/bin/bash
# Round 4: the timeline probe with spread atomics, and the walking grids
# (GSPLAT_PROJECT_GRID / GSPLAT_EMIT_GRID) on bands and whole frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4pr2
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['bands'], d['slowest_us'], d['us_per_frame_by_band'], d['slowest_band_stage_us'])"; }
PL=$PWD/tmp_ab/probe/libgsplat.so
for f in 1 3; do
  echo "== probe: band 3 of 8, inflight $f $(date +%T)"
  rm -f $O/probe_b3_f$f.bin
  GSPLAT_LIB=$PL GSPLAT_PROBE_FILE=$O/probe_b3_f$f.bin timeout -k 10 300 python tools/band_emulate.py --balanced --inflight $f --bands 8 --only-band 3 --steps 400 > $O/probe_b3_f$f.jsonl 2> $O/probe_b3_f$f.err || exit $?
  bands $O/probe_b3_f$f.jsonl
  python3 tools/probe_timeline.py $O/probe_b3_f$f.bin --json $O/probe_b3_f$f.json
done
echo "== probe: band 3 of 8, grids 2048, inflight 3 $(date +%T)"
rm -f $O/probe_b3_g2048_f3.bin
GSPLAT_PROJECT_GRID=2048 GSPLAT_EMIT_GRID=2048 GSPLAT_LIB=$PL GSPLAT_PROBE_FILE=$O/probe_b3_g2048_f3.bin timeout -k 10 300 python tools/band_emulate.py --balanced --inflight 3 --bands 8 --only-band 3 --steps 400 > $O/probe_b3_g2048_f3.jsonl 2> $O/probe_b3_g2048_f3.err || exit $?
python3 tools/probe_timeline.py $O/probe_b3_g2048_f3.bin --json $O/probe_b3_g2048_f3.json
echo "== probe: whole frame, inflight 3 $(date +%T)"
rm -f $O/probe_full_f3.bin
GSPLAT_LIB=$PL GSPLAT_PROBE_FILE=$O/probe_full_f3.bin timeout -k 10 300 python tools/band_emulate.py --inflight 3 --bands 1 --steps 400 > $O/probe_full_f3.jsonl 2> $O/probe_full_f3.err || exit $?
bands $O/probe_full_f3.jsonl
python3 tools/probe_timeline.py $O/probe_full_f3.bin --json $O/probe_full_f3.json
for g in 0 1536 2048; do
  echo "== all 8 bands of config 4, grids $g $(date +%T)"
  GSPLAT_PROJECT_GRID=$g GSPLAT_EMIT_GRID=$g timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_g$g.jsonl 2> $O/bands_g$g.err || exit $?
  bands $O/bands_g$g.jsonl
done
for rep in 1 2; do
  for g in 0 2048; do
    echo "== c3, project grid $g, rep $rep $(date +%T)"
    GSPLAT_PROJECT_GRID=$g timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_g${g}_$rep.json 2> $O/c3_g${g}_$rep.err || exit $?
    line $O/c3_g${g}_$rep.json
  done
done
for g in 0 2048; do
  echo "== bands c5, grids $g $(date +%T)"
  GSPLAT_PROJECT_GRID=$g GSPLAT_EMIT_GRID=$g timeout -k 10 500 python tools/band_emulate.py --config5 --balanced --rebalance --inflight 3 --bands 8 > $O/bands_c5_g$g.jsonl 2> $O/bands_c5_g$g.err || exit $?
  bands $O/bands_c5_g$g.jsonl
done
echo "== done $(date +%T)"
