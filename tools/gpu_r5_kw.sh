#!/bin/bash
# Short-run sensitivity of the headline line: steps / warm-up combinations,
# interleaved, three rounds.  gpurun_out/${TAG:-r6k}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6k}
mkdir -p $O
for r in 1 2 3; do
  for kw in "20 5" "20 50" "100 5" "600 200"; do
    set -- $kw
    timeout -k 10 300 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --e2e-frames 0 > $O/b_${1}_${2}_$r.json 2> $O/b_${1}_${2}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b_${1}_${2}_$r.json "K=$1 W=$2"
  done
done
