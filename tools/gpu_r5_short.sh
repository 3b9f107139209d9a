#!/bin/bash
# Short-run behaviour of the headline line (the driver runs --steps 20
# --warmup 5) and the group path: group tests, the in-process group line,
# then bench lines at several step / warmup counts.  Outputs under
# gpurun_out/${TAG:-r5short}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${TAG:-r5short}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_bench.py tests/test_gpu_poison.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_group.txt 2>&1
rc=$?; tail -n 2 $O/pytest_group.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gather --no-cpu-baseline > $O/bench_gather.json 2> $O/bench_gather.err || exit $?
python3 - $O/bench_gather.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("gather", d["value"], {k: round(1e3 * v["avg_ms"], 1) for k, v in d["kernels"].items()}, d["group"]["gather_ms"])
PY
for sw in "20 5" "20 5" "20 200" "100 5" "600 200" "20 5"; do
  set -- $sw
  timeout -k 10 300 python bench.py --steps $1 --warmup $2 --no-cpu-baseline > $O/bench_s$1_w$2.json 2> $O/bench_s$1_w$2.err || exit $?
  python3 - $O/bench_s$1_w$2.json "$1 $2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("steps/warmup", sys.argv[2], d["value"], d["ms_per_step"], d["frame_latency_ms"])
PY
done
