#!/bin/bash
# Round 6: the config-5 orbit tests alone (they faulted with the first direct
# binning build), then the direct-binning A/B (tools/r6/ab3.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6c5b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 --timeout-method thread -k "config5" > $O/pytest_c5.txt 2>&1 || { tail -n 30 $O/pytest_c5.txt; exit 1; }
tail -n 2 $O/pytest_c5.txt
bash tools/r6/ab3.sh
