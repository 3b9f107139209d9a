#!/bin/bash
# Round-3: how the driver-shaped run (20 steps after 5 warm-up frames) reads
# with the copy-peak measurement of --copy-peak-s seconds before the timed
# region, against 200 warm-up frames.  Outputs under gpurun_out/r3w/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3w; mkdir -p $O
for k in 1 2; do
  for cfg in "0:5" "0.06:5" "0.3:5" "0:200"; do
    cs=${cfg%%:*}; w=${cfg##*:}
    timeout -k 10 300 python bench.py --steps 20 --warmup $w --copy-peak-s $cs --no-cpu-baseline --profile-frames 2 > $O/w_${cs}_${w}_$k.json 2>> $O/err.txt || exit $?
    python3 -c "
import json; d=json.loads(open('$O/w_${cs}_${w}_$k.json').read().strip().splitlines()[-1]); print('copy_s=$cs warmup=$w rep $k', d['value'], d['roofline']['peak_measured'])"
  done
done
