#!/bin/bash
# Interleaved A/B of tmp_ab/<name>/libgsplat.so builds on the 8-band critical
# path (tools/band_emulate.py --balanced --inflight 3, config 4), REPS rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for d in tmp_ab/*/; do
    n=$(basename "$d")
    GSPLAT_LIB=$PWD/$d/libgsplat.so timeout -k 10 300 python tools/band_emulate.py --balanced --inflight 3 --bands 8 --steps 400 > gpurun_out/ab8_$n.jsonl 2> gpurun_out/ab8_$n.err || { tail -3 gpurun_out/ab8_$n.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ab8_$n.jsonl'):
  d=json.loads(l); print('$rep $n slowest', d['slowest_us'], 'stages', d.get('slowest_band_stage_us'))
"
  done
done
