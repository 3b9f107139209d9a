#!/bin/bash
# Round-3: config-5 bench line (kernel table) of the current tree, the opt-in
# hardware-exp mode's error (tests -s) and its headline bench line.  Outputs
# under gpurun_out/r3c5/.  Each GPU step has its own time limit; the first
# failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3c5; mkdir -p $O
echo "== c5 $(date +%T)"
timeout -k 10 600 python bench.py --config5 --steps 240 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c1-300 $O/bench_c5.json
echo "== fastexp tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast_exp.py -x -v -s --timeout 200 --timeout-method thread > $O/fast_exp_tests.txt 2>&1 || exit $?
grep -h "fast exp" $O/fast_exp_tests.txt
echo "== fastexp bench $(date +%T)"
timeout -k 10 400 python bench.py --fast-exp --no-cpu-baseline > $O/bench_c3_fastexp.json 2> $O/bench_c3_fastexp.err || exit $?
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
echo "== driver-shaped runs $(date +%T)"
for k in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3_s20w5_$k.json 2>> $O/bench_c3.err || exit $?
  cut -c1-260 $O/bench_c3_s20w5_$k.json
done
echo "== done $(date +%T)"
