#!/bin/bash
# Round-3: parity of the tmp_ab/xcd* blend orders (full-frame tests), the
# headline A/B and a config-5 A/B of every tmp_ab/ build, then the
# round-end bench lines of the tree with the current byte model.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for n in xcd64 xcd128; do
  GSPLAT_LIB=$PWD/tmp_ab/$n/libgsplat.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "not global and not poison" > gpurun_out/pytest_$n.txt 2>&1
  rc=$?; echo "$n tests rc=$rc $(tail -n 1 gpurun_out/pytest_$n.txt)"; [ $rc -eq 0 ] || exit $rc
done
REPS=3 bash tools/ab_repeat.sh || exit $?
REPS=2 STEPS=240 BENCH_ARGS=--config5 bash tools/ab_repeat.sh || exit $?
mkdir -p gpurun_out/r3f
timeout -k 10 600 python bench.py --steps 600 --no-cpu-baseline --pmc-json profiles/r03_end/pmc_c3.json > gpurun_out/r3f/bench_c3.json 2> gpurun_out/r3f/err.txt || exit $?
timeout -k 10 600 python bench.py --config5 --steps 240 --no-cpu-baseline --pmc-json profiles/r03_end/pmc_c5.json > gpurun_out/r3f/bench_c5.json 2>> gpurun_out/r3f/err.txt || exit $?
echo done
