#!/bin/bash
# Round-3 end: 1/2/4/8-band emulations (balanced, three frames in flight) of
# configs 4 and 5 on the final tree.  Outputs under gpurun_out/r3e/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3e; mkdir -p $O
timeout -k 10 600 python tools/band_emulate.py --balanced --rebalance --inflight 3 --config5 --steps 120 > $O/bands_c5.jsonl 2> $O/bands_c5.err || exit $?
true
python3 -c "
import json
for f in ('bands_c5',):
  for l in open('$O/'+f+'.jsonl'):
    d=json.loads(l); print(f, d['bands'], d['slowest_us'], d.get('speedup'), d.get('skew_slowest_over_mean'))"
