cd "${GRAFT_REPO_ROOT}" || exit 1
o=gpurun_out/s16.txt; : > $o
for q in 4 16; do
  for f in 3 6 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tools/band_emulate.py --balanced --inflight $f --bands 8 --steps 200 > gpurun_out/be8_q${q}_f$f.txt 2>&1 || exit $?
    echo "q=$q f=$f $(grep bands gpurun_out/be8_q${q}_f$f.txt | cut -c1-260)" >> $o
  done
  for f in 3 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --inflight $f > gpurun_out/bq${q}_f$f.log 2>&1 || exit $?
    echo "bench q=$q f=$f $(grep -o '"value": [0-9.]*' gpurun_out/bq${q}_f$f.log)" >> $o
  done
done
