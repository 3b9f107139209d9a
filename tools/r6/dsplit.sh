#!/bin/bash
# Round 6: the direct blend's sort against its walk: band 3 of 8 (config 4),
# base, ds1 (GS_X_DSPLIT=1: no sort), ds2 (no blend walk); one and three
# frames in flight, and kernel traces at one in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6dsplit
mkdir -p $O
set -e
export TMPDIR=/tmp
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for v in base ds1 ds2; do
  for f in 1 3; do
    GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f$f.jsonl 2> $O/emu_${v}_f$f.err
    echo "$v f$f $(tail -n 1 $O/emu_${v}_f$f.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"])')"
  done
  GSPLAT_LIB=$(lib $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o p -- python3 $EMU --inflight 1 --steps 100 > $O/prof_$v.log 2>&1
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -n 1)
  python3 - "$f" $v <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:3]:
    print(sys.argv[2], f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.2f} us')
PY
done
