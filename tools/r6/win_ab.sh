#!/bin/bash
# Round 6: the window-2 two-pixel blend.  GPU tests on the product, then an
# interleaved A/B of the bench (600 frames) against tmp_ab/ variants, then
# rocprof kernel stats of the product and the one-batch walk (one frame in
# flight), then the band probe (tools/r6/probe2.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6win
mkdir -p $O
set -e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -n 1 $O/pytest_gpu.txt
NO_TESTS=1 REPEATS=${REPEATS:-2} TAG=r6win bash tools/ab_r5.sh
for v in base xnowin; do
  L=$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so; [ $v != base ] && L=$PWD/tmp_ab/$v/libgsplat.so
  GSPLAT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$v -o stats --output-format csv -- python3 bench.py --steps 50 --warmup 3 --no-cpu-baseline --inflight 1 > $O/stats_$v.log 2>&1
  python3 tools/pmc_summary.py $O/stats_$v --config x > $O/stats_$v.txt 2>&1 || true
  grep -E "gs_blend|gs_project|gs_sort" $O/stats_$v.txt
done
bash tools/r6/probe2.sh
