cd "${GRAFT_REPO_ROOT}" || exit 1
o=gpurun_out/s22.txt; : > $o
for rep in 1 2; do
for v in nobc bc; do
  GSPLAT_LIB=$PWD/tmp_ab/$v/libgsplat.so timeout -k 10 200 python tools/band_emulate.py --balanced --inflight 3 --bands 8 --only-band 3 --steps 400 > gpurun_out/be22_$v.txt 2>&1 || exit $?
  echo "c4 $v $(grep bands gpurun_out/be22_$v.txt | cut -c1-120) $(grep -o '"slowest_band_stage_us.*' gpurun_out/be22_$v.txt)" >> $o
done
done
for v in nobc bc; do
  GSPLAT_LIB=$PWD/tmp_ab/$v/libgsplat.so timeout -k 10 400 python tools/band_emulate.py --balanced --rebalance --config5 --inflight 3 --bands 8 --only-band 4 --steps 120 > gpurun_out/be22c5_$v.txt 2>&1 || exit $?
  echo "c5 $v $(grep -o '"us_per_frame_by_band.*' gpurun_out/be22c5_$v.txt)" >> $o
done
