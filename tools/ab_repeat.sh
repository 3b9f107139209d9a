#!/bin/bash
# Interleaved repeats of the headline bench over tmp_ab/<name>/libgsplat.so
# builds (REPS rounds, STEPS frames each): box-to-box noise is larger than
# most single changes, so A/B only within one call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for d in tmp_ab/*/; do
    n=$(basename "$d")
    GSPLAT_LIB=$PWD/$d/libgsplat.so timeout -k 10 200 python bench.py --steps ${STEPS:-400} --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abr_$n.log 2>&1 || exit $?
    python3 -c "
import json
for l in open('gpurun_out/abr_$n.log'):
  if l.startswith('{'):
    d=json.loads(l); print('$rep $n', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
"
  done
done
