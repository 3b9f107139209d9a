#!/bin/bash
# Round-3 A/B of the count / emit row slices at config 5 (GSPLAT_BIN_SLICES=1
# turns them off at run time), after the slice parity tests.  Outputs under
# gpurun_out/r3s/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -k "slices or config5" > $O/pytest.txt 2>&1
rc=$?; tail -n 3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
fi
for k in 1 2; do
  for v in 1 0; do
    echo "== c5 slices_off=$v rep $k $(date +%T)"
    if [ $v = 1 ]; then export GSPLAT_BIN_SLICES=1; else unset GSPLAT_BIN_SLICES; fi
    timeout -k 10 400 python bench.py --config5 --steps 240 --no-cpu-baseline > $O/c5_off${v}_$k.json 2> $O/c5_off${v}_$k.err || exit $?
    python3 -c "
import json,sys; d=json.loads(open('$O/c5_off${v}_$k.json').read().strip().splitlines()[-1]); k=d['kernels']
print(d['value'], {n: round(k[n]['avg_ms']*1e3,1) for n in k})"
  done
done
unset GSPLAT_BIN_SLICES
echo "== done $(date +%T)"
