#!/bin/bash
# One round-end measurement set, per workload (c3: the headline 1M/1080p; c5:
# config 5, 8M/4K orbit): kernel stats + PMC passes with one frame in flight,
# their summary (tools/pmc_summary.py, keyed on the bench's pmc_key), then the
# bench line that reads the fresh counters.  Outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
set -e
export TMPDIR=/tmp
for w in ${WORKLOADS:-c3 c5}; do
  case $w in
    c3) EXTRA=""; BSTEPS=600 ;;
    c5) EXTRA="--config5"; BSTEPS=240 ;;
  esac
  NAME=$w BENCH_ARGS="--inflight 1 $EXTRA" PASSES="${PASSES:-stats fetch write sq1}" STEPS=20 bash tools/profile.sh > gpurun_out/profile_$w.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/prof_$w --json gpurun_out/pmc_$w.json > gpurun_out/pmc_summary_$w.txt
  timeout -k 10 600 python3 bench.py $EXTRA --steps $BSTEPS --pmc-json gpurun_out/pmc_$w.json > gpurun_out/bench_$w.json.log 2>&1
  grep '"metric"' gpurun_out/bench_$w.json.log | cut -c1-300
done
