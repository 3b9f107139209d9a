#!/bin/bash
# The 20-step line against an untimed pre-warm (--prewarm-ms), interleaved,
# three rounds.  gpurun_out/${TAG:-r6p}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6p}
mkdir -p $O
for r in 1 2 3; do
  for pw in 0 50 100 200; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --prewarm-ms $pw --no-cpu-baseline --e2e-frames 0 > $O/b_${pw}_$r.json 2> $O/b_${pw}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('prewarm', sys.argv[2], d['value'], d['ms_per_step'], d['config'].get('prewarm', d.get('prewarm')))" $O/b_${pw}_$r.json $pw
  done
done
