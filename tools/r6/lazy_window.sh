#!/bin/bash
# Round 6: the lazy big lists' continuation window (GS_X_LAZY_WINDOW keys past
# the prefix; 1536 the product): config-5 parity tests on each variant, then
# interleaved config-5 bench lines, and the kernel stats of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6lw
mkdir -p $O
set -e
export TMPDIR=/tmp
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
for v in lw2048 lw3072; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "config5 or big or lazy or cont" > $O/pytest_$v.txt 2>&1 || { tail -n 30 $O/pytest_$v.txt; exit 1; }
  echo "$v $(tail -n 1 $O/pytest_$v.txt)"
done
for rep in 1 2; do
  for v in base lw2048 lw3072; do
    GSPLAT_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config5 --steps 240 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    python3 - $O/bench_${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], {k: round(1e3 * v["avg_ms"], 1) for k, v in d["kernels"].items()}, d["frame"]["n_big_tiles"])
PY
  done
done
