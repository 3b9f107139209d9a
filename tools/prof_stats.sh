#!/bin/bash
# rocprofv3 kernel stats of the bench, one frame in flight, for the headline
# workload and config 5.  Outputs under gpurun_out/prof_<name>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <name> <timeout> <bench args...>
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o $name --output-format csv -- python3 bench.py "$@" > gpurun_out/prof_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$name.log; exit $rc; fi
  python3 - "$name" <<'PY'
import csv, glob, sys
name = sys.argv[1]
for f in glob.glob(f"gpurun_out/prof_{name}/**/*kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:16]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.2f} pct {float(r["Percentage"]):6.2f}')
PY
}
for w in ${WORKLOADS:-c3 c5}; do
  case $w in
    c3) run c3 300 --steps 40 --warmup 5 --inflight 1 --no-cpu-baseline ;;
    c5) run c5 600 --config5 --steps 40 --warmup 5 --inflight 1 --no-cpu-baseline --profile-frames 8 ;;
  esac
done
