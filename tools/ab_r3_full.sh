cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
GSPLAT_LIB=$PWD/tmp_ab/a_onerec/libgsplat.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/abt_full_a_onerec.log 2>&1
rc=$?; echo "a_onerec full tests rc=$rc $(tail -n 1 gpurun_out/abt_full_a_onerec.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TESTED="f1_early f2_nobranch f3_prescale" TESTS="parity or fullsize" REPS=3 STEPS=400 bash tools/ab_r3.sh
