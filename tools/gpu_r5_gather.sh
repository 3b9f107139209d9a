#!/bin/bash
# The one-GPU group's own cost: interleaved rounds of the plain line and the
# group line (--gather) for the in-tree library and tmp_ab_g/ variants.
# gpurun_out/${TAG:-r5g}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5g}
mkdir -p $O
shopt -s nullglob
libs="base"
for d in tmp_ab_g/*/; do libs="$libs $(basename $d)"; done
path() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab_g/$1/libgsplat.so"; }
for r in $(seq 1 ${REPEATS:-3}); do
  timeout -k 10 300 python bench.py --steps 600 --no-cpu-baseline --e2e-frames 0 > $O/plain_$r.json 2> $O/plain_$r.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('plain', d['value'])" $O/plain_$r.json
  for n in $libs; do
    GSPLAT_LIB=$(path $n) timeout -k 10 300 python bench.py --gather --steps 600 --no-cpu-baseline > $O/g_${n}_$r.json 2> $O/g_${n}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d.get('group', {}).get('gather_ms'))" $n $O/g_${n}_$r.json
  done
done
