#!/bin/bash
# Config 3: the in-tree library at 2 / 3 / 4 frames in flight and the
# tmp_nt/ variants at 3, interleaved, REPEATS rounds.  gpurun_out/${TAG:-r6if}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${TAG:-r6if}
mkdir -p $O
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  GSPLAT_LIB=$lib timeout -k 10 300 python bench.py --steps 600 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || return $?
  python3 - "$n" $O/$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], {k: round(1e3 * v["avg_ms"], 1) for k, v in d["kernels"].items()})
PY
}
base=$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so
for r in $(seq 1 ${REPEATS:-2}); do
  run base_f3_$r $base --inflight 3 || exit $?
  run base_f2_$r $base --inflight 2 || exit $?
  run base_f4_$r $base --inflight 4 || exit $?
  for d in tmp_nt/*/; do run $(basename $d)_f3_$r $PWD/$d/libgsplat.so --inflight 3 || exit $?; done
done
