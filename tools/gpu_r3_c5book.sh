#!/bin/bash
# Round-3: bench lines of configs 3 and 5 with the fresh PMC summaries of the
# round-end profile (gpurun_out/pmc_c3.json, pmc_c5.json must exist on the box:
# they are copied in from profiles/r03_end), so the algorithmic bytes of every
# stage can be set against the PMC bytes.  Outputs under gpurun_out/r3b/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 600 python bench.py --config5 --steps 240 --no-cpu-baseline --pmc-json profiles/r03_end/pmc_c5.json > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
timeout -k 10 600 python bench.py --steps 600 --no-cpu-baseline --pmc-json profiles/r03_end/pmc_c3.json > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
cut -c1-200 $O/bench_c5.json $O/bench_c3.json
