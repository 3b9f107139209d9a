#!/bin/bash
# Round 6: where a row band's projection spends its time.  Band 3 of 8
# balanced bands of config 4, one frame in flight: plain timings, rocprof
# kernel stats and PMC passes for the product (base) and the GS_X_BAND
# variants in tmp_ab/ (tools/build_x.sh).  Outputs under gpurun_out/r6band/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6band
mkdir -p $O
set -e
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps ${STEPS:-100}"
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
  tail -n 1 $O/pytest_gpu.txt
fi
for v in ${VARIANTS:-base xb1 xb2}; do
  for f in 1 3; do
    GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f$f.jsonl 2> $O/emu_${v}_f$f.err
    echo "$v f$f $(tail -n 1 $O/emu_${v}_f$f.jsonl | cut -c1-400)"
  done
  GSPLAT_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$v -o stats --output-format csv -- python3 $EMU --inflight 1 > $O/stats_$v.log 2>&1
  python3 tools/pmc_summary.py $O/stats_$v --config c4:band3of8 > $O/stats_$v.txt 2>&1 || true
  head -n 20 $O/stats_$v.txt
done
if [ -z "$NO_PMC" ]; then
  for p in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
    n=$(echo $p | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $p -d $O/pmc_$n -o pmc --output-format csv -- python3 $EMU --inflight 1 --steps 20 > $O/pmc_$n.log 2>&1
  done
  python3 tools/pmc_summary.py $O --config c4:band3of8 --json $O/pmc_band3.json > $O/pmc_band3.txt 2>&1 || true
  head -n 40 $O/pmc_band3.txt
fi
