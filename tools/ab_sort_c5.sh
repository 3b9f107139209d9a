#!/bin/bash
# Big-list parity tests, then config 5 kernel stats (rocprofv3) and bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS_K:-} > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
WORKLOADS=c5 bash tools/prof_stats.sh || exit 1
GSPLAT_LAZY=0 timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 10 --no-cpu-baseline --profile-frames 12 > gpurun_out/c5_full.log 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/c5_full.log'):
    if l.startswith('{'):
        d=json.loads(l); print('c5 (no lazy) fps', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 10 --no-cpu-baseline > gpurun_out/c5_bench.log 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/c5_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('c5 fps', d['value'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
