#!/bin/bash
# GPU parity tests + short bench, printing per-kernel averages.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q --timeout 200 -x > gpurun_out/t1.log 2>&1
rc=$?
tail -n 3 gpurun_out/t1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/b1.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/b1.log'):
  if l.startswith('{'):
    d=json.loads(l); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
"
