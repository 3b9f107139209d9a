#!/bin/bash
# Round 4 (re-entry): the one-pixel blend with its record walk software-
# pipelined (GS_BLEND_PIPE: tmp_ab/pipe7 at >= 7 waves per SIMD, tmp_ab/pipe8
# at 8) -- the GPU parity suite on pipe7, then config 5 (lazy frames), 8 row
# bands of config 4 (in-blend sort) and config 3 with one pixel per lane,
# interleaved against the default library; first config 3's two-pixel
# blend (LPT order) against its branch-free (px2bf) and non-interleaved
# (px2il0) steps.  Outputs under gpurun_out/r4pipe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4pipe
mkdir -p $O
P7=$PWD/tmp_ab/pipe7/libgsplat.so
P8=$PWD/tmp_ab/pipe8/libgsplat.so
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
echo "== tests on pipe7 $(date +%T)"
GSPLAT_LIB=$P7 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_pipe7.txt 2>&1
rc=$?; tail -n 2 $O/pytest_gpu_pipe7.txt; [ $rc -eq 0 ] || exit $rc
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['value'], {k:round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"; }
BF=$PWD/tmp_ab/px2bf/libgsplat.so
IL0=$PWD/tmp_ab/px2il0/libgsplat.so
for rep in 1 2 3; do
  for v in base bf il0; do
    case $v in
      base) E="" ;;
      bf) E="GSPLAT_LIB=$BF" ;;
      il0) E="GSPLAT_LIB=$IL0" ;;
    esac
    echo "== c3 $v rep $rep $(date +%T)"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit $?
    line $O/c3_${v}_$rep.json
  done
done
for rep in 1 2; do
  for v in base pipe7 pipe8; do
    case $v in
      base) E="" ;;
      pipe7) E="GSPLAT_LIB=$P7" ;;
      pipe8) E="GSPLAT_LIB=$P8" ;;
    esac
    echo "== c5 $v rep $rep $(date +%T)"
    env $E timeout -k 10 400 python bench.py --config5 --steps 240 --warmup 120 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit $?
    line $O/c5_${v}_$rep.json
    echo "== bands c4 $v rep $rep $(date +%T)"
    env $E timeout -k 10 300 python tools/band_emulate.py --balanced --inflight 3 --bands 8 > $O/b8_${v}_$rep.jsonl 2> $O/b8_${v}_$rep.err || exit $?
    cut -c1-260 $O/b8_${v}_$rep.jsonl
    echo "== c3 px1 $v rep $rep $(date +%T)"
    env $E GSPLAT_BLEND_PX2=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3px1_${v}_$rep.json 2> $O/c3px1_${v}_$rep.err || exit $?
    line $O/c3px1_${v}_$rep.json
  done
done
echo "== done $(date +%T)"
