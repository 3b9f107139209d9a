#!/bin/bash
# headline A/B (tools/ab_r3.sh) then config-5 benches of the builds in $C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/ab_r3.sh || exit $?
for n in $C5; do
  GSPLAT_LIB=$PWD/tmp_ab/$n/libgsplat.so timeout -k 10 300 python bench.py --config5 --steps ${C5STEPS:-120} --warmup 10 --no-cpu-baseline > gpurun_out/abc5_$n.log 2>&1 || exit $?
  python3 -c "
import json
for l in open('gpurun_out/abc5_$n.log'):
  if l.startswith('{'):
    d=json.loads(l); print('c5 $n', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
"
done
