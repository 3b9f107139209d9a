#!/bin/bash
# Round 6: frames in flight with direct band binning (2-kernel band chains):
# 8 balanced bands of config 4 (128 pairs per tile) at F = 2, 3, 4, band 3 of
# 8 alone at F = 2, 3, 4; config 5's 8 re-balanced bands at F = 3; the
# emulated 8-band bench line (bench.py --split 8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6infl
mkdir -p $O
set -e
for f in 2 3 4; do
  timeout -k 10 300 python3 tools/band_emulate.py --balanced --bands 1,8 --inflight $f > $O/bands_c4_f$f.jsonl 2> $O/bands_c4_f$f.err
  echo "c4 8 bands F=$f $(tail -n 1 $O/bands_c4_f$f.jsonl | cut -c1-300)"
  timeout -k 10 200 python3 tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300 --inflight $f > $O/band3_f$f.jsonl 2> $O/band3_f$f.err
  echo "band3 F=$f $(tail -n 1 $O/band3_f$f.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"])')"
done
timeout -k 10 500 python3 tools/band_emulate.py --config5 --balanced --rebalance --bands 1,8 --inflight 3 --steps 60 > $O/bands_c5.jsonl 2> $O/bands_c5.err
echo "c5 $(tail -n 1 $O/bands_c5.jsonl | cut -c1-300)"
timeout -k 10 300 python3 bench.py --split 8 --steps 600 --no-cpu-baseline > $O/bench_split8.json 2> $O/bench_split8.err
python3 - $O/bench_split8.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("split8", d["value"], d["ms_per_step"], d["config"].get("binning"), d["config"].get("parallelism"))
PY
