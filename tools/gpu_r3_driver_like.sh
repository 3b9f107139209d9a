#!/bin/bash
# What the driver runs at round end, on the final tree: GPU tests, smoke(),
# bench.py with the driver's arguments.  Outputs under gpurun_out/r3d/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 1 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -n 1 $O/smoke.txt
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-200 $O/bench.json
