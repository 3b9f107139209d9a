#!/bin/bash
# Round 6: the direct band binning.  GPU suite with it on (the in-tree
# library), then band 3 of 8 (config 4) one and three frames in flight:
# base (direct), classic (GS_X_DIRECT_OFF: the scan and emit), xb5 (classic
# without the scan and emit launches after the first frames: wrong frames, the
# bound); all 8 bands for base and classic.  (ab4: the totals in a kernel of
# their own instead of the last blend workgroup's ticket.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6ab4
mkdir -p $O
set -e
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -n 30 $O/pytest_gpu.txt; exit 1; }
tail -n 1 $O/pytest_gpu.txt
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for rep in 1 2; do
  for v in base classic xb5; do
    for f in 1 3; do
      GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f${f}_$rep.jsonl 2> $O/emu_${v}_f${f}_$rep.err
      echo "$v f$f rep$rep $(tail -n 1 $O/emu_${v}_f${f}_$rep.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"])')"
    done
  done
done
for v in base classic; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 400 python3 tools/band_emulate.py --balanced --bands 1,8 --inflight 3 > $O/bands_${v}.jsonl 2> $O/bands_${v}.err
  echo "$v $(tail -n 1 $O/bands_${v}.jsonl | cut -c1-330)"
done
