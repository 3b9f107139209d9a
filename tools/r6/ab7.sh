#!/bin/bash
# Round 6 (ab7): direct band binning into the layout of the view's last scan
# against classic (tmp_ab/classic: GS_X_DIRECT_OFF, the scan and emit):
# GPU suite + smoke, band 3 of 8 (config 4) one and three frames in flight,
# 1- and 8-band splits, a kernel trace of band 3, PMC summaries of the band
# shapes (pmc_bands.sh), and the bench's default and --gather lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6ab7
mkdir -p $O
set -e
export TMPDIR=/tmp
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -n 30 $O/pytest_gpu.txt; exit 1; }
tail -n 1 $O/pytest_gpu.txt
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && tail -n 1 $O/smoke.txt
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for rep in 1 2; do
  for v in base classic; do
    for f in 1 3; do
      GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f${f}_$rep.jsonl 2> $O/emu_${v}_f${f}_$rep.err
      echo "$v f$f rep$rep $(tail -n 1 $O/emu_${v}_f${f}_$rep.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"])')"
    done
  done
done
for v in base classic; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 400 python3 tools/band_emulate.py --balanced --bands 1,8 --inflight 3 > $O/bands_${v}.jsonl 2> $O/bands_${v}.err
  echo "$v $(tail -n 1 $O/bands_${v}.jsonl | cut -c1-400)"
done
for v in base classic; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o band3 -- python3 $EMU --inflight 3 > $O/prof_$v.log 2>&1
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -n 1)
  echo "== $v"; python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.2f} us')
PY
done
