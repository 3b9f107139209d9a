#!/bin/bash
# Round 4: workgroup shapes that the dispatcher can place beside the other
# frames' waves -- the aggregated scan at 256 threads (default build) against
# 1024 (tmp_ab/scan1024) on 8 bands; the aggregated binning (lean projection,
# 256-thread scan) against the chunked one on config 3; the tile sort's code
# size (tmp_ab/kpl1: its rare radix path at one key per lane; tmp_ab/sortlean:
# also the E = 4 network rolled) on config 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4sc
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; }
bands() { python3 -c "
import json
for l in open('$1'):
    d=json.loads(l); print(d['inflight'], d['bands'], d['slowest_us'], d['us_per_frame_by_band'], d['slowest_band_stage_us'])"; }
for rep in 1 2; do
  echo "== bands c4 scan 256 rep $rep $(date +%T)"
  timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_256_$rep.jsonl 2> $O/bands_256_$rep.err || exit $?
  bands $O/bands_256_$rep.jsonl
  echo "== bands c4 scan 1024 rep $rep $(date +%T)"
  GSPLAT_LIB=$PWD/tmp_ab/scan1024/libgsplat.so timeout -k 10 400 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/bands_1024_$rep.jsonl 2> $O/bands_1024_$rep.err || exit $?
  bands $O/bands_1024_$rep.jsonl
done
for rep in 1 2; do
  for v in chunked agg kpl1 sortlean; do
    echo "== c3 $v rep $rep $(date +%T)"
    case $v in
      chunked) E="" ;;
      agg) E="GSPLAT_BIN_AGG=1" ;;
      *) E="GSPLAT_LIB=$PWD/tmp_ab/$v/libgsplat.so" ;;
    esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
echo "== done $(date +%T)"
