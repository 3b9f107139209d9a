#!/bin/bash
# Round 6: frames in flight 2..8 (band 3 of 8, config 4; whole frame, config 3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6inflight2
mkdir -p $O
set -e
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for f in 2 3 4 5 6 7 8; do
  timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_f${f}.jsonl 2> $O/emu_f${f}.err
  echo "band3 f$f $(tail -n 1 $O/emu_f${f}.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"])')"
done
for f in 2 3 4 5 6 8; do
  timeout -k 10 300 python3 bench.py --steps 600 --no-cpu-baseline --inflight $f > $O/bench_f$f.json 2> $O/bench_f$f.err
  echo "c3 f$f $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"])' $O/bench_f$f.json)"
done
