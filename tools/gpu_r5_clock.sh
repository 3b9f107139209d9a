#!/bin/bash
# GPU clock and power while the headline workload runs (rocm-smi samples
# beside a long bench run), then idle.  gpurun_out/${TAG:-r6c}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6clk}
mkdir -p $O
timeout -k 10 120 rocm-smi --showclocks --showpower --showuse > $O/smi_idle.txt 2>&1
( timeout -k 10 300 python bench.py --steps 200000 --warmup 200 --no-cpu-baseline --e2e-frames 0 > $O/bench_long.json 2> $O/bench_long.err ) &
BP=$!
k=0
while kill -0 $BP 2>/dev/null && [ $k -lt 200 ]; do
  k=$((k + 1))
  timeout -k 5 20 rocm-smi --showclocks --showpower --showuse > $O/smi_$k.txt 2>&1
  sleep 0.3
done
wait $BP
rc=$?
grep -h "sclk\|Power\|GPU use" $O/smi_*.txt | sort | uniq -c | head -40
cut -c1-200 $O/bench_long.json
exit $rc
