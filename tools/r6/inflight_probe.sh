#!/bin/bash
# Round 6: frames in flight x hardware queues (GPU_MAX_HW_QUEUES, HIP's
# default 4 on the box), band 3 of 8 (config 4) and the whole frame (config 3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6inflight
mkdir -p $O
set -e
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for rep in 1 2; do
  for q in 4 8; do
    for f in 3 4 6; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_q${q}_f${f}_$rep.jsonl 2> $O/emu_q${q}_f${f}_$rep.err
      echo "band3 q$q f$f rep$rep $(tail -n 1 $O/emu_q${q}_f${f}_$rep.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["host_enqueue_us_by_band"])')"
    done
  done
done
for q in 4 8; do
  for f in 3 4; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --steps 600 --no-cpu-baseline --inflight $f > $O/bench_q${q}_f$f.json 2> $O/bench_q${q}_f$f.err
    echo "c3 q$q f$f $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"])' $O/bench_q${q}_f$f.json)"
  done
done
