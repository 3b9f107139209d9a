#!/bin/bash
# Five driver-shaped lines (20 steps after 5 warm-up frames, the default
# 50-ms pre-warm) back to back: the spread of the short line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${TAG:-r6s5}
mkdir -p $O
for r in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/short_$r.json 2> $O/short_$r.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/short_$r.json').read().strip().splitlines()[-1]); print('short', d['value'], d['ms_per_step'])"
done
