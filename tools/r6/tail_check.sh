#!/bin/bash
# Round 6: the direct totals' block counts in one load round -- direct GPU
# tests, band 3 of 8 one / three frames in flight, 8 bands, kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6tail
mkdir -p $O
set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -n 30 $O/pytest.txt; exit 1; }
tail -n 1 $O/pytest.txt
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for f in 1 3 1 3; do
  timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_f$f.jsonl 2> $O/emu_f$f.err
  echo "f$f $(tail -n 1 $O/emu_f$f.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"]["blend"])')"
done
timeout -k 10 300 python3 tools/band_emulate.py --balanced --bands 1,8 --inflight 3 > $O/bands_c4.jsonl 2> $O/bands_c4.err
tail -n 1 $O/bands_c4.jsonl | cut -c1-260
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $EMU --inflight 1 --steps 100 > $O/prof.log 2>&1
f=$(find $O/prof -name '*kernel_stats.csv' | head -n 1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:2]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.2f} us')
PY
