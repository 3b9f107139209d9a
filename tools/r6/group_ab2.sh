#!/bin/bash
# Round 6, second group-cull A/B (the float-tail group_culled): band 3 of 8,
# base / g1 / g2 interleaved, kernel stats of base; then the VALU operand-kind
# rates (tools/hip/valu_rate).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6group2
mkdir -p $O
set -e
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps ${STEPS:-200}"
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "band or group or split or cull" > $O/pytest_band.txt 2>&1
tail -n 1 $O/pytest_band.txt
for rep in 1 2; do
  for v in ${VARIANTS:-base g1 g2}; do
    for f in 1 3; do
      GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f${f}_$rep.jsonl 2> $O/emu_${v}_f${f}_$rep.err
      echo "$v f$f rep$rep $(tail -n 1 $O/emu_${v}_f${f}_$rep.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"])')"
    done
  done
done
for v in base; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$v -o stats --output-format csv -- python3 $EMU --inflight 1 > $O/stats_$v.log 2>&1
  python3 tools/pmc_summary.py $O/stats_$v --config c4:band3of8 > $O/stats_$v.txt 2>&1 || true
  grep -i 'project\|agg\|blend' $O/stats_$v.txt | head -n 8
done
timeout -k 10 120 tools/hip/valu_rate > $O/valu_rate.json
grep bv_ $O/valu_rate.json
