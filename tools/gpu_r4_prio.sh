#!/bin/bash
# Round 4 (re-entry): the two-pixel blend's long-list waves at raised priority (GS_PX2_PRIO:
# the waves of lists longer than 256 / 1024 keys at raised issue priority, tmp_ab/prio256 / prio1024)
# -- the two-pixel parity tests on each, then config 3 interleaved, three
# repeats.  Outputs under gpurun_out/r4prio.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4prio
mkdir -p $O
for v in prio256 prio1024; do
  echo "== px2 tests on $v $(date +%T)"
  GSPLAT_LIB=$PWD/tmp_ab/$v/libgsplat.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "px2 or fullsize" > $O/pytest_$v.txt 2>&1
  rc=$?; tail -n 1 $O/pytest_$v.txt; [ $rc -eq 0 ] || exit $rc
done
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"; }
for rep in 1 2 3; do
  for v in base prio256 prio1024; do
    E=""
    [ $v != base ] && E="GSPLAT_LIB=$PWD/tmp_ab/$v/libgsplat.so"
    echo "== c3 $v rep $rep $(date +%T)"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
echo "== done $(date +%T)"
