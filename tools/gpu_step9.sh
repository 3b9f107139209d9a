cd "${GRAFT_REPO_ROOT}" || exit 1
TESTED="cur s32" TESTS="lazy or fullsize or parity" REPS=0 C5="base cur s32 s64 cur s32 s64" C5STEPS=200 bash tools/ab_r3_c5.sh > gpurun_out/ab9.txt 2>&1
