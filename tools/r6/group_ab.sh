#!/bin/bash
# Round 6: the band projection's per-group cull (group_culled) A/B.  Band 3 of
# 8 balanced bands of config 4, one and three frames in flight, interleaved
# repeats of: base (the in-tree library), g1 (no group cull), g2 (no group
# cull, the rounds 2-5 factor 2), xb1 (every block returns after the cull
# pass); then rocprof kernel stats of base and g2, and all 8 bands of base.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6group
mkdir -p $O
set -e
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps ${STEPS:-200}"
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
  tail -n 1 $O/pytest_gpu.txt
fi
for rep in 1 2; do
  for v in ${VARIANTS:-base g1 g2 xb1}; do
    for f in 1 3; do
      GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f${f}_$rep.jsonl 2> $O/emu_${v}_f${f}_$rep.err
      echo "$v f$f rep$rep $(tail -n 1 $O/emu_${v}_f${f}_$rep.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"])')"
    done
  done
done
for v in base g2; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$v -o stats --output-format csv -- python3 $EMU --inflight 1 > $O/stats_$v.log 2>&1
  python3 tools/pmc_summary.py $O/stats_$v --config c4:band3of8 > $O/stats_$v.txt 2>&1 || true
  grep -i 'project\|agg\|blend' $O/stats_$v.txt | head -n 8
done
timeout -k 10 300 python3 tools/band_emulate.py --balanced --bands 1,8 --inflight 3 > $O/bands_c4.jsonl 2> $O/bands_c4.err
tail -n 1 $O/bands_c4.jsonl | cut -c1-700
