#!/bin/bash
# Config 3 at 3 frames in flight with the default 4 hardware queues and with
# GPU_MAX_HW_QUEUES=8, interleaved.  gpurun_out/${TAG:-r6hq}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${TAG:-r6hq}
mkdir -p $O
for r in 1 2 3; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 600 --no-cpu-baseline > $O/q${q}_$r.json 2> $O/q${q}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$O/q${q}_$r.json').read().strip().splitlines()[-1]); print('q$q', d['value'])"
  done
done
