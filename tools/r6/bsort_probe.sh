#!/bin/bash
# Round 6: what a row band's blend-with-sort spends on the sort and on the
# walk (GS_X_BSORT variants in tmp_x/), band 3 of 8 of config 4, 1 and 3
# frames in flight, plus rocprof kernel times of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6bsort
mkdir -p $O
set -e
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 200"
for v in base xs1 xs2 xb3; do
  L=$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so; [ $v != base ] && L=$PWD/tmp_x/$v/libgsplat.so
  for f in 1 3; do
    GSPLAT_LIB=$L timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f$f.jsonl 2> $O/emu_${v}_f$f.err
    echo "$v f$f $(tail -n 1 $O/emu_${v}_f$f.jsonl | grep -o '"slowest_us[^,]*') $(tail -n 1 $O/emu_${v}_f$f.jsonl | grep -o '"slowest_band_stage.*')"
  done
  GSPLAT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$v -o stats --output-format csv -- python3 $EMU --inflight 1 --steps 100 > $O/stats_$v.log 2>&1
  python3 - $O/stats_$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gsk::(anonymous namespace)::", "")
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, x in sorted(d.items()):
    x.sort()
    print(f"  {k}: n={len(x)} median={x[len(x)//2]:.2f} us")
PY
done
