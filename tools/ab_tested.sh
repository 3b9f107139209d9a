#!/bin/bash
# For each tmp_ab/<name>/libgsplat.so: the GPU parity tests (stop at the first
# failing build), then interleaved headline benches (REPS rounds) and one
# 8-band gather-path bench per build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for d in tmp_ab/*/; do
  n=$(basename "$d")
  GSPLAT_LIB=$PWD/$d/libgsplat.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_$n.log 2>&1
  rc=$?; echo "$n tests rc=$rc $(tail -n 1 gpurun_out/abt_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
REPS=${REPS:-2} bash tools/ab_repeat.sh || exit $?
for d in tmp_ab/*/; do
  n=$(basename "$d")
  GSPLAT_LIB=$PWD/$d/libgsplat.so timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --gather --split 8 --steps 600 --no-cpu-baseline > gpurun_out/abg_$n.log 2>&1 || exit $?
  echo "split8 $n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abg_$n.log)"
done
