cd "${GRAFT_REPO_ROOT}" || exit 1
TESTED=pipe TESTS="lazy or fullsize or parity" REPS=2 C5="base pipe" C5STEPS=200 bash tools/ab_r3_c5.sh > gpurun_out/ab8.txt 2>&1 || exit $?
WORKLOADS=c5 bash tools/prof_stats.sh > gpurun_out/prof8.txt 2>&1
