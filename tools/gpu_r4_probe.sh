#!/bin/bash
# Round 4: GPU tests; config 3 and 8-band config 4 with the default build;
# then kernel timelines of the probe build (tools/edit_probe.py): band 3 of 8
# with 1 / 3 / 6 frames in flight and the whole frame with 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4pr
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['bands'], d['slowest_us'], d['slowest_band_stage_us'])"; }
echo "== c3 $(date +%T)"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit $?
line $O/c3.json
echo "== bands c4 $(date +%T)"
timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands.jsonl 2> $O/bands.err || exit $?
bands $O/bands.jsonl
PL=$PWD/tmp_ab/probe/libgsplat.so
for f in 1 3 6; do
  echo "== probe: band 3 of 8, inflight $f $(date +%T)"
  rm -f $O/probe_b3_f$f.bin
  GSPLAT_LIB=$PL GSPLAT_PROBE_FILE=$O/probe_b3_f$f.bin timeout -k 10 300 python tools/band_emulate.py --balanced --inflight $f --bands 8 --only-band 3 --steps 400 > $O/probe_b3_f$f.jsonl 2> $O/probe_b3_f$f.err || exit $?
  bands $O/probe_b3_f$f.jsonl
  python3 tools/probe_timeline.py $O/probe_b3_f$f.bin --json $O/probe_b3_f$f.json
done
echo "== probe: whole frame, inflight 3 $(date +%T)"
rm -f $O/probe_full_f3.bin
GSPLAT_LIB=$PL GSPLAT_PROBE_FILE=$O/probe_full_f3.bin timeout -k 10 300 python tools/band_emulate.py --inflight 3 --bands 1 --steps 400 > $O/probe_full_f3.jsonl 2> $O/probe_full_f3.err || exit $?
bands $O/probe_full_f3.jsonl
python3 tools/probe_timeline.py $O/probe_full_f3.bin --json $O/probe_full_f3.json
for g in 256 1024; do
  echo "== band 3 of 8, emit grid $g, inflight 3 / 6 $(date +%T)"
  for f in 3 6; do
    GSPLAT_EMIT_GRID=$g timeout -k 10 300 python tools/band_emulate.py --balanced --inflight $f --bands 8 --only-band 3 --steps 400 > $O/eg${g}_f$f.jsonl 2> $O/eg${g}_f$f.err || exit $?
    bands $O/eg${g}_f$f.jsonl
  done
done
for g in 1024 2048; do
  echo "== band 3 of 8, project + emit grid $g, inflight 3 / 6 $(date +%T)"
  for f in 3 6; do
    GSPLAT_PROJECT_GRID=$g GSPLAT_EMIT_GRID=$g timeout -k 10 300 python tools/band_emulate.py --balanced --inflight $f --bands 8 --only-band 3 --steps 400 > $O/pg${g}_f$f.jsonl 2> $O/pg${g}_f$f.err || exit $?
    bands $O/pg${g}_f$f.jsonl
  done
done
echo "== probe: band 3 of 8, emit grid 256, inflight 6 $(date +%T)"
rm -f $O/probe_eg256_f6.bin
GSPLAT_EMIT_GRID=256 GSPLAT_LIB=$PL GSPLAT_PROBE_FILE=$O/probe_eg256_f6.bin timeout -k 10 300 python tools/band_emulate.py --balanced --inflight 6 --bands 8 --only-band 3 --steps 400 > $O/probe_eg256_f6.jsonl 2> $O/probe_eg256_f6.err || exit $?
python3 tools/probe_timeline.py $O/probe_eg256_f6.bin --json $O/probe_eg256_f6.json
echo "== done $(date +%T)"
