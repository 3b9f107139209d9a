#!/bin/bash
# Interleaved A/B of tmp_ab/<name>/libgsplat.so variants against the in-tree
# library on the row-band emulation (8 balanced bands of config 4, slowest
# band) and config 5's whole frame (its lazy continuation): parity tests of
# the band / lazy paths first, then REPEATS rounds.  gpurun_out/${TAG:-abb}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${TAG:-abb}
mkdir -p $O
shopt -s nullglob
libs="base"
for d in ${ABDIR:-tmp_ab}/*/; do libs="$libs $(basename $d)"; done
path() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/${ABDIR:-tmp_ab}/$1/libgsplat.so"; }
[ -z "$NO_TESTS" ] && for n in $libs; do
  [ "$n" = base ] && continue
  GSPLAT_LIB=$(path $n) timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "band or lazy or group or orbit or config5 or large_tile or equal_depths" > $O/test_$n.log 2>&1
  rc=$?
  echo "$n tests rc=$rc $(tail -n 1 $O/test_$n.log)"
  [ $rc -ge 124 ] && exit $rc
done
for r in $(seq 1 ${REPEATS:-2}); do
  for n in $libs; do
    GSPLAT_LIB=$(path $n) timeout -k 10 300 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/b_${n}_$r.jsonl 2>/dev/null || exit $?
    GSPLAT_LIB=$(path $n) timeout -k 10 300 python bench.py --config5 --steps 240 --no-cpu-baseline > $O/c5_${n}_$r.json 2>/dev/null || exit $?
    python3 - "$n" $O/b_${n}_$r.jsonl $O/c5_${n}_$r.json <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1], "bands8 slowest", b["slowest_us"], b["slowest_band_stage_us"].get("blend"),
      "| c5", c["value"], {k: round(1e3 * v["avg_ms"], 1) for k, v in c["kernels"].items()})
PY
  done
done
