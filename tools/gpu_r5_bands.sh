#!/bin/bash
# Row-band emulation on one GPU (tools/band_emulate.py): configs 4 and 5,
# three frames in flight, the slowest band's period.  gpurun_out/${TAG:-r5b}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${TAG:-r5b}
mkdir -p $O
timeout -k 10 600 python tools/band_emulate.py --balanced --inflight 3 --bands ${BANDS:-1,8} > $O/bands_c4.jsonl 2> $O/bands_c4.err || exit $?
cut -c1-400 $O/bands_c4.jsonl
if [ -z "$NO_C5" ]; then
timeout -k 10 600 python tools/band_emulate.py --config5 --balanced --rebalance --inflight 3 --bands 1,8 > $O/bands_c5.jsonl 2> $O/bands_c5.err || exit $?
cut -c1-400 $O/bands_c5.jsonl
fi
