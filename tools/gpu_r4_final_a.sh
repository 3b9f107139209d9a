#!/bin/bash
# Round-4 end, part A: GPU tests, smoke, the lean-projection A/B (config 3,
# interleaved against tmp_ab/nolean), rocprofv3 stats + PMC passes of configs
# 3 and 5 (tools/round_profile.sh), the FETCH_SIZE calibration, and the
# kernel stats of one pipelined band (band 3 of 8, three frames in flight).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4fa
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
cat $O/smoke.txt
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
NL=$PWD/tmp_ab/nolean/libgsplat.so
for rep in 1 2 3; do
  echo "== c3 lean rep $rep $(date +%T)"
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_lean_$rep.json 2> $O/c3_lean_$rep.err || exit $?
  line $O/c3_lean_$rep.json
  echo "== c3 not lean rep $rep $(date +%T)"
  GSPLAT_LIB=$NL timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_fat_$rep.json 2> $O/c3_fat_$rep.err || exit $?
  line $O/c3_fat_$rep.json
done
echo "== profiles $(date +%T)"
PASSES="stats fetch write sq1 lds" bash tools/round_profile.sh || exit $?
echo "== FETCH_SIZE calibration $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o calib --output-format csv -- tools/hip/fetch_calib > gpurun_out/calib.log 2>&1 || exit $?
python3 tools/fetch_calib.py gpurun_out/calib --json $O/fetch_calib.json
echo "== band 3 of 8 kernel stats $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_band3 -o band3 --output-format csv -- python3 tools/band_emulate.py --balanced --inflight 3 --bands 8 --only-band 3 --steps 200 > $O/trace_band3.log 2>&1 || exit $?
echo "== done $(date +%T)"
