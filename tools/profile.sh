#!/bin/bash
# rocprofv3 passes on the bench: kernel trace + stats, then PMC counters in
# separate passes (never combined with other trace domains).
#   NAME=c3 BENCH_ARGS="--inflight 1" PASSES="stats fetch write sq1 sq2" STEPS=20
# Outputs: gpurun_out/prof_$NAME/<pass>/..., gpurun_out/prof_$NAME/<pass>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_${NAME:-c3}
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-}"
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $BENCH > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '"metric"' $OUT/$name.log | cut -c1-160
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
for p in ${PASSES:-stats fetch write sq1 sq2}; do
  case $p in
    stats) run stats 600 --kernel-trace --stats ;;
    fetch) run pmc_fetch 600 --pmc FETCH_SIZE ;;
    write) run pmc_write 600 --pmc WRITE_SIZE ;;
    sq1) run pmc_sq1 600 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU ;;
    sq2) run pmc_sq2 600 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE ;;
    lds) run pmc_lds 600 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU ;;
  esac
done
