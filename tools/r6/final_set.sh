#!/bin/bash
# Round 6 end set: GPU suite, smoke, config 5 PMC (appended to the bench's
# default PMC file), bench lines (driver-shaped default, 600 frames, the
# one-GPU group, SH-3, config 5), 1/2/4/8-band emulations of configs 4 and 5.
# Outputs under gpurun_out/r6final/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6final
mkdir -p $O
set -e
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
  tail -n 1 $O/pytest_gpu.txt
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
  cat $O/smoke.txt
fi
if [ -z "$NO_C5PMC" ]; then
  # config 5 whole frame: kernel stats + PMC, appended under its key
  cp profiles/pmc_latest.json $O/pmc_all.json
  NAME=c5 BENCH_ARGS="--inflight 1 --config5" PASSES="stats fetch write sq1" STEPS=20 bash tools/profile.sh > $O/profile_c5.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/prof_c5 --json $O/pmc_all.json --append > $O/pmc_summary_c5.txt
  tail -n 25 $O/pmc_summary_c5.txt | cut -c1-160
  PJ="--pmc-json $O/pmc_all.json"
fi
timeout -k 10 300 python3 bench.py $PJ > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 300 python3 bench.py --steps 600 $PJ --no-cpu-baseline > $O/bench_600.json 2> $O/bench_600.err
timeout -k 10 300 python3 bench.py --steps 600 --gather $PJ --no-cpu-baseline > $O/bench_gather.json 2> $O/bench_gather.err
timeout -k 10 300 python3 bench.py --steps 600 --sh $PJ --no-cpu-baseline > $O/bench_sh.json 2> $O/bench_sh.err
timeout -k 10 300 python3 bench.py --config5 --steps 240 $PJ > $O/bench_c5.json 2> $O/bench_c5.err
for f in bench_default bench_600 bench_gather bench_sh bench_c5; do
  python3 - $O/$f.json $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(sys.argv[2], d["value"], d.get("ms_per_step"), "blend", r.get("kernel"), r.get("frac"), "traffic", r.get("traffic"),
      "valu", r.get("valu_issue_frac"), r.get("valu_issue_frac_2cyc"))
PY
done
timeout -k 10 400 python3 tools/band_emulate.py --balanced --inflight 3 > $O/bands_c4.jsonl 2> $O/bands_c4.err
tail -n 1 $O/bands_c4.jsonl | cut -c1-400
timeout -k 10 500 python3 tools/band_emulate.py --config5 --balanced --rebalance --bands 1,8 --inflight 3 --steps 60 > $O/bands_c5.jsonl 2> $O/bands_c5.err
tail -n 1 $O/bands_c5.jsonl | cut -c1-400
