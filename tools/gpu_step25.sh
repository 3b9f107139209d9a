cd "${GRAFT_REPO_ROOT}" || exit 1
o=gpurun_out/s25.txt; : > $o
GSPLAT_LIB=$PWD/tmp_ab/cr/libgsplat.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "band or group or poison" > gpurun_out/t25.txt 2>&1
echo "tests rc=$? $(tail -n 1 gpurun_out/t25.txt)" >> $o
for rep in 1 2; do
for v in base cr; do
  GSPLAT_LIB=$PWD/tmp_ab/$v/libgsplat.so timeout -k 10 300 python tools/band_emulate.py --balanced --inflight 3 --bands 8 --only-band 3 --steps 400 > gpurun_out/be25_$v.txt 2>&1 || exit $?
  grep bands gpurun_out/be25_$v.txt | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print('c4 $v', d['bands'], d['slowest_us'], d['slowest_band_stage_us'])" >> $o
done
done
for v in base cr; do
  GSPLAT_LIB=$PWD/tmp_ab/$v/libgsplat.so timeout -k 10 400 python tools/band_emulate.py --balanced --rebalance --config5 --inflight 3 --bands 8 --only-band 4 --steps 120 > gpurun_out/be25c5_$v.txt 2>&1 || exit $?
  grep bands gpurun_out/be25c5_$v.txt | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print('c5 $v', d['bands'], d['slowest_us'], d['slowest_band_stage_us'])" >> $o
done
