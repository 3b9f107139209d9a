#!/bin/bash
# Band / group parity tests, then the per-band critical path (band emulation,
# balanced bands, three frames in flight).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bands_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bands_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/band_emulate.py --balanced --inflight 3 --steps 200 > gpurun_out/band_emulate.log 2>&1 || exit 1
cat gpurun_out/band_emulate.log | tail -12
