#!/bin/bash
# XCD-aware blend mapping A/B: interleaved config-3 lines (tools/ab_r5.sh over
# tmp_ab/), then a FETCH_SIZE pass per library (one frame in flight) for the
# blend's HBM read bytes.  gpurun_out/${TAG:-r5x}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
T=${TAG:-r5x}
[ -z "$NO_AB" ] && { ABDIR=tmp_ab REPEATS=${REPEATS:-3} TAG=$T/ab bash tools/ab_r5.sh || exit $?; }
mkdir -p gpurun_out/$T
for n in ${LIBS:-base}; do
  if [ $n = base ]; then unset GSPLAT_LIB; else export GSPLAT_LIB=$PWD/tmp_ab/$n/libgsplat.so; fi
  NAME=${T}_$n BENCH_ARGS="--inflight 1" PASSES="fetch" STEPS=20 bash tools/profile.sh > gpurun_out/${T}_$n.log 2>&1 || exit $?
  python3 tools/pmc_summary.py gpurun_out/prof_${T}_$n --json gpurun_out/$T/pmc_$n.json > gpurun_out/$T/pmc_$n.txt 2>&1 || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['kernels']; k=[x for x in d if 'blend' in x]; print(sys.argv[2], {x: round(d[x].get("fetch_bytes_raw",0)/1e6,1) for x in k})" gpurun_out/$T/pmc_$n.json $n
done
unset GSPLAT_LIB
echo "== done $(date +%T)"
