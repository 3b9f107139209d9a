#!/bin/bash
# Round 6 (ab8): where the direct blend's extra time goes.  GPU suite (the
# in-tree library: direct binning into the view's last scan layout, raster
# tile order), band 3 of 8 (config 4) one and three frames in flight for base,
# fin1 (GS_X_DIRECT_FIN=1: no ticket / totals), fin2 (nor the end barrier),
# classic (the scan and emit); SQ and TCC counters of band 3 for base and classic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6ab8
mkdir -p $O
set -e
export TMPDIR=/tmp
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -n 30 $O/pytest_gpu.txt; exit 1; }
tail -n 1 $O/pytest_gpu.txt
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for v in base fin1 fin2 classic base classic; do
  for f in 1 3; do
    GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f${f}.jsonl 2> $O/emu_${v}_f${f}.err
    echo "$v f$f $(tail -n 1 $O/emu_${v}_f${f}.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"])')"
  done
done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
for v in base classic; do
  GSPLAT_LIB=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_sq_$v -o p -- python3 $EMU --inflight 1 --steps 60 > $O/pmc_sq_$v.log 2>&1
  GSPLAT_LIB=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/pmc_tcc_$v -o p -- python3 $EMU --inflight 1 --steps 60 > $O/pmc_tcc_$v.log 2>&1
  GSPLAT_LIB=$(lib $v) timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o p -- python3 $EMU --inflight 1 --steps 60 > $O/kt_$v.log 2>&1
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for v in ("base", "classic"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for kind in ("sq", "tcc"):
        for f in glob.glob(f"{O}/pmc_{kind}_{v}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                n[(k, r["Counter_Name"])] += 1
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{O}/kt_{v}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, d in sorted(agg.items()):
        if not any(s in k for s in ("blend", "project", "agg_")):
            continue
        out = {c: round(x / max(1, n[(k, c)]), 1) for c, x in sorted(d.items())}
        ds = sorted(dur.get(k, [0]))
        print(v, k, "median_us", ds[len(ds) // 2], out)
PY
