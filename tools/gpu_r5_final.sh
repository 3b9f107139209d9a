#!/bin/bash
# Round-5 end set (one call): GPU tests, smoke, rocprofv3 stats + PMC passes
# of configs 3 and 5 with their bench lines (tools/round_profile.sh), then the
# default line (reading the fresh config-3 PMC summary), the driver-shaped,
# SH-3 and in-process group lines, and the band emulations of configs 4
# (1/2/4/8) and 5 (1/8).  Outputs under gpurun_out/r5fin.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5fin}
mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
  rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
fi
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
cat $O/smoke.txt
echo "== profiles $(date +%T)"
PASSES="stats fetch write sq1 lds" bash tools/round_profile.sh || exit $?
PMC=gpurun_out/pmc_c3.json
echo "== default bench $(date +%T)"
timeout -k 10 600 python bench.py --pmc-json $PMC > $O/bench_default.json 2> $O/bench_default.err || exit $?
cut -c1-300 $O/bench_default.json
echo "== driver-shaped bench $(date +%T)"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc-json $PMC > $O/bench_driver_shaped.json 2> $O/bench_driver_shaped.err || exit $?
cut -c1-200 $O/bench_driver_shaped.json
echo "== SH-3 bench $(date +%T)"
timeout -k 10 600 python bench.py --sh --no-cpu-baseline > $O/bench_sh.json 2> $O/bench_sh.err || exit $?
cut -c1-300 $O/bench_sh.json
echo "== group bench $(date +%T)"
timeout -k 10 600 python bench.py --gather --no-cpu-baseline > $O/bench_gather.json 2> $O/bench_gather.err || exit $?
cut -c1-200 $O/bench_gather.json
echo "== bands c4 $(date +%T)"
timeout -k 10 600 python tools/band_emulate.py --balanced --inflight 3 --bands 1,2,4,8 > $O/bands_c4.jsonl 2> $O/bands_c4.err || exit $?
cut -c1-300 $O/bands_c4.jsonl
echo "== bands c5 $(date +%T)"
timeout -k 10 600 python tools/band_emulate.py --config5 --balanced --rebalance --inflight 3 --bands 1,8 > $O/bands_c5.jsonl 2> $O/bands_c5.err || exit $?
cut -c1-300 $O/bands_c5.jsonl
echo "== done $(date +%T)"
