cd "${GRAFT_REPO_ROOT}" || exit 1
for f in 3 4 6 2; do
  timeout -k 10 300 python bench.py --config5 --steps 200 --warmup 10 --no-cpu-baseline --inflight $f > gpurun_out/inf_$f.log 2>&1 || exit $?
  python3 -c "
import json
for l in open('gpurun_out/inf_$f.log'):
  if l.startswith('{'): d=json.loads(l); print('inflight $f', d['value'], d['ms_per_step'])"
done
GSPLAT_LIB=$PWD/tmp_ab/nocont/libgsplat.so timeout -k 10 300 python bench.py --config5 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/inf_nocont.log 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/inf_nocont.log'):
  if l.startswith('{'): d=json.loads(l); print('nocont', d['value'], d['ms_per_step'])"
