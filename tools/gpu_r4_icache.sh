#!/bin/bash
# Round 4: does the blend kernel's code size (the in-blend sort compiled in,
# ~41 KB) slow whole frames whose kernels share the CUs' instruction cache?
# config 3 with the default build against tmp_ab/nosortcode (same behaviour,
# sort code compiled out), interleaved; then config 3 at 2 / 4 frames in
# flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4ic
mkdir -p $O
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
NS=$PWD/tmp_ab/nosortcode/libgsplat.so
for rep in 1 2 3; do
  echo "== c3 default rep $rep $(date +%T)"
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_d_$rep.json 2> $O/c3_d_$rep.err || exit $?
  line $O/c3_d_$rep.json
  echo "== c3 no sort code rep $rep $(date +%T)"
  GSPLAT_LIB=$NS timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_ns_$rep.json 2> $O/c3_ns_$rep.err || exit $?
  line $O/c3_ns_$rep.json
done
for f in 2 4; do
  echo "== c3 inflight $f $(date +%T)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --inflight $f > $O/c3_f$f.json 2> $O/c3_f$f.err || exit $?
  line $O/c3_f$f.json
done
echo "== done $(date +%T)"
