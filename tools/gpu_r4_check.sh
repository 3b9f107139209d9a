#!/bin/bash
# Round-4 check of the current tree on one MI355X: GPU tests, the default
# bench line, the in-process group path (--gather), and the 1/8-band
# emulation of config 4.  Outputs under gpurun_out/r4/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== bench default $(date +%T)"
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cut -c1-400 $O/bench_default.json
echo "== bench gather $(date +%T)"
timeout -k 10 300 python bench.py --gather --no-cpu-baseline > $O/bench_gather.json 2> $O/bench_gather.err || exit $?
cut -c1-300 $O/bench_gather.json
echo "== bands c4 $(date +%T)"
timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 1,8 > $O/bands_c4.jsonl 2> $O/bands_c4.err || exit $?
cut -c1-400 $O/bands_c4.jsonl
echo "== done $(date +%T)"
