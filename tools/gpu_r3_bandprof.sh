#!/bin/bash
# Round-3: rocprofv3 kernel stats of one middle band of the 8-band balanced
# split (config 4), one frame in flight.  Outputs under gpurun_out/r3bp/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3bp; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o b3 --output-format csv -- python3 tools/band_emulate.py --balanced --inflight 1 --bands 8 --only-band 3 --steps 200 > $O/b3.log 2>&1 || exit $?
tail -2 $O/b3.log
timeout -k 10 300 python3 tools/band_emulate.py --balanced --inflight 3 --bands 8 --steps 400 > $O/b8_if3.jsonl 2> $O/b8_if3.err || exit $?
cut -c1-400 $O/b8_if3.jsonl
