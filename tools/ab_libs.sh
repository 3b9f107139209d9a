#!/bin/bash
# A/B timing of alternative builds: for every tmp_ab/<name>/libgsplat.so run
# the GPU parity tests (first failure stops) and a short bench.  Names
# starting with t_ are timing-only probes (deliberately wrong output): no tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for d in tmp_ab/*/; do
  n=$(basename "$d")
  if [[ $n == t_* ]]; then rc=0; echo "$n timing only"; else
  GSPLAT_LIB=$PWD/$d/libgsplat.so timeout -k 10 300 python -m pytest tests -m gpu -q --timeout 200 -x > gpurun_out/ab_$n.test.log 2>&1
  rc=$?
  echo "$n tests rc=$rc $(tail -n 1 gpurun_out/ab_$n.test.log)"
  [ $rc -ge 124 ] && exit $rc
  fi
  GSPLAT_LIB=$PWD/$d/libgsplat.so timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$n.bench.log 2>&1 || exit $?
  python3 -c "
import json
for l in open('gpurun_out/ab_$n.bench.log'):
  if l.startswith('{'):
    d=json.loads(l); print('$n', d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
"
done
