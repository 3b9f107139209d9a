cd "${GRAFT_REPO_ROOT}" || exit 1
TESTED="ls64" TESTS="lazy or fullsize or parity or bin" REPS=2 C5="base ls64 base ls64" C5STEPS=200 bash tools/ab_r3_c5.sh > gpurun_out/ab12.txt 2>&1
