#!/bin/bash
# 8-band emulation (config 4) at several frames in flight and HIP hardware
# queue counts: does a band's small, latency-bound frame gain from more
# frames in flight?  One line per (queues, in-flight).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for q in ${QUEUES:-4 8}; do
  for f in ${INFLIGHT:-3 4 6}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 tools/band_emulate.py --balanced --inflight $f --bands 8 --only-band 3 \
      --steps 400 > gpurun_out/bif_${q}_$f.jsonl 2> gpurun_out/bif_${q}_$f.err || exit $?
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
  d=json.loads(l); print('queues $q inflight $f', d['bands'], d['slowest_us'], d['us_per_frame_by_band'])
" gpurun_out/bif_${q}_$f.jsonl
  done
done
