#!/bin/bash
# Config 5 only: the in-tree library against tmp_nt/ variants, interleaved,
# REPEATS rounds.  gpurun_out/${TAG:-r6c5}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${TAG:-r6c5}
mkdir -p $O
for r in $(seq 1 ${REPEATS:-2}); do
  for lib in base tmp_nt/*/; do
    n=$(basename $lib); L=$PWD/$lib/libgsplat.so; [ $n = base ] && L=$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so
    GSPLAT_LIB=$L timeout -k 10 300 python bench.py --config5 --steps 240 --no-cpu-baseline > $O/c5_${n}_$r.json 2> $O/c5_${n}_$r.err || exit $?
    python3 - "$n" $O/c5_${n}_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], {k: round(1e3 * v["avg_ms"], 1) for k, v in d["kernels"].items()})
PY
  done
done
