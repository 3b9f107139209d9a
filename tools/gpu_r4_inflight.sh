#!/bin/bash
# Round 4: the band period against frames in flight (8-band split of config
# 4, band 3): is the band period its frame latency / F?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['slowest_us'], d['host_enqueue_us_by_band'], d['slowest_band_stage_us'])"; }
for f in 1 2 3 4 5 6; do
  echo "== band 3 of 8, inflight $f $(date +%T)"
  timeout -k 10 300 python tools/band_emulate.py --balanced --inflight $f --bands 8 --only-band 3 --steps 400 > $O/f$f.jsonl 2> $O/f$f.err || exit $?
  bands $O/f$f.jsonl
done
for f in 3 4 6; do
  echo "== band 3 of 8, inflight $f, GPU_MAX_HW_QUEUES=8 $(date +%T)"
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/band_emulate.py --balanced --inflight $f --bands 8 --only-band 3 --steps 400 > $O/q8f$f.jsonl 2> $O/q8f$f.err || exit $?
  bands $O/q8f$f.jsonl
done
echo "== done $(date +%T)"
bash tools/gpu_r4_packed.sh
