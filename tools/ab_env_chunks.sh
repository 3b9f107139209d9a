#!/bin/bash
# Interleaved A/B of the binning chunk size (GSPLAT_BIN_CHUNK_SIZE, read at
# gs_create) at config 5 and config 3, REPS rounds.  Outputs under gpurun_out/abc/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/abc; mkdir -p $O
run() {  # run <tag> <chunk or -> <bench args...>
  local tag=$1 cs=$2; shift 2
  if [ "$cs" = "-" ]; then unset GSPLAT_BIN_CHUNK_SIZE; else export GSPLAT_BIN_CHUNK_SIZE=$cs; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --warmup 10 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -3 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$tag', d['value'], {n: round(k[n]['avg_ms']*1e3,1) for n in k})"
}
for rep in $(seq ${REPS:-2}); do
  for cs in - 16384 20480 47000 65535; do run c5_${cs}_$rep $cs --config5 --steps 240 || exit 1; done
  for cs in - 8192; do run c3_${cs}_$rep $cs --steps 400 || exit 1; done
done
unset GSPLAT_BIN_CHUNK_SIZE
