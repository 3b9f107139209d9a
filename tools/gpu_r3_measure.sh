#!/bin/bash
# Round-3 measurement set of the current tree: rocprofv3 kernel stats + PMC
# passes + the bench lines that read them (tools/round_profile.sh, c3 and c5),
# then the row-band emulation at 1/2/4/8 bands for config 4 (1M/1080p) and
# config 5 (8M/4K orbit, re-balanced), three frames in flight.  Every GPU step
# has its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_PROF" ]; then
  WORKLOADS="${WORKLOADS:-c3 c5}" bash tools/round_profile.sh || exit $?
fi
if [ -z "$SKIP_BANDS" ]; then
  echo "== bands c4 $(date +%T)"
  timeout -k 10 400 python3 tools/band_emulate.py --balanced --inflight 3 --bands 1,2,4,8 --steps 300 \
    > gpurun_out/bands_c4.jsonl 2> gpurun_out/bands_c4.err || exit $?
  echo "== bands c5 $(date +%T)"
  timeout -k 10 600 python3 tools/band_emulate.py --balanced --rebalance --config5 --inflight 3 --bands 1,2,4,8 \
    --steps 120 > gpurun_out/bands_c5.jsonl 2> gpurun_out/bands_c5.err || exit $?
fi
echo "== done $(date +%T)"
