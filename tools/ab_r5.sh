#!/bin/bash
# Interleaved A/B of the in-tree library against tmp_ab/<name>/libgsplat.so
# variants (tools/build_x.sh <name> "-D..."): the GPU parity tests once per variant
# (first failure stops it), then REPEATS rounds of a bench line per library,
# libraries interleaved within a round.  BENCH_ARGS adds bench.py flags.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${TAG:-ab}
mkdir -p $O
shopt -s nullglob
libs="base"
for d in ${ABDIR:-tmp_ab}/*/; do libs="$libs $(basename $d)"; done
path() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/${ABDIR:-tmp_ab}/$1/libgsplat.so"; }
if [ -z "$NO_TESTS" ]; then
for n in $libs; do
  [ "$n" = base ] && continue
  [[ $n == t_* ]] && continue
  GSPLAT_LIB=$(path $n) timeout -k 10 400 python -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread ${TEST_ARGS:-} > $O/test_$n.log 2>&1
  rc=$?
  echo "$n tests rc=$rc $(tail -n 1 $O/test_$n.log)"
  [ $rc -ge 124 ] && exit $rc
done
fi
for r in $(seq 1 ${REPEATS:-3}); do
  for n in $libs; do
    GSPLAT_LIB=$(path $n) timeout -k 10 300 python bench.py --steps ${STEPS:-600} --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit $?
    python3 - "$n" "$O/bench_${n}_$r.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], {k: round(1e3 * v["avg_ms"], 1) for k, v in d["kernels"].items()})
PY
  done
done
