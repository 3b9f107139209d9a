#!/bin/bash
# rocprofv3 passes on the headline bench: kernel trace + stats, then PMC
# counters in separate passes (never combined with other trace domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $BENCH > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run stats 600 --kernel-trace --stats
run pmc_fetch 600 --pmc FETCH_SIZE
run pmc_write 600 --pmc WRITE_SIZE
run pmc_sq1 600 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
run pmc_sq2 600 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE
find $OUT -name "*.csv" | head -50
