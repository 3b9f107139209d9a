#!/bin/bash
# Round-4 end set, part B: the default bench line (CPU baseline included,
# reading the committed config-3 PMC summary), the driver-shaped line, the
# SH-3 line, the in-process group line, and the band emulations of configs 4
# (1/2/4/8) and 5 (8).  Outputs under gpurun_out/r4end/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4end
mkdir -p $O
PMC=profiles/r04_end/pmc_c3.json
echo "== default bench $(date +%T)"
timeout -k 10 600 python bench.py --pmc-json $PMC > $O/bench_default.json 2> $O/bench_default.err || exit $?
cut -c1-300 $O/bench_default.json
echo "== driver-shaped bench $(date +%T)"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc-json $PMC > $O/bench_driver_shaped.json 2> $O/bench_driver_shaped.err || exit $?
cut -c1-200 $O/bench_driver_shaped.json
echo "== SH-3 bench $(date +%T)"
timeout -k 10 600 python bench.py --sh --no-cpu-baseline > $O/bench_sh.json 2> $O/bench_sh.err || exit $?
cut -c1-300 $O/bench_sh.json
echo "== group bench $(date +%T)"
timeout -k 10 600 python bench.py --gather --no-cpu-baseline > $O/bench_gather.json 2> $O/bench_gather.err || exit $?
cut -c1-200 $O/bench_gather.json
echo "== bands c4 $(date +%T)"
timeout -k 10 600 python tools/band_emulate.py --balanced --inflight 3 --bands 1,2,4,8 > $O/bands_c4.jsonl 2> $O/bands_c4.err || exit $?
cut -c1-300 $O/bands_c4.jsonl
echo "== bands c5 $(date +%T)"
timeout -k 10 600 python tools/band_emulate.py --config5 --balanced --rebalance --inflight 3 --bands 1,8 > $O/bands_c5.jsonl 2> $O/bands_c5.err || exit $?
cut -c1-300 $O/bands_c5.jsonl
echo "== done $(date +%T)"
