#!/bin/bash
# Round 6: direct binning's totals -- a kernel of their own (base) against the
# blend's last workgroup behind a write-through hand-off (ticket,
# GS_X_DIRECT_TICKET) -- and classic (the scan and emit).  Direct and band
# tests on the ticket build, band 3 of 8 (config 4) at three frames in
# flight, all 8 bands, kernel traces, and FETCH/WRITE + SQ counters of band 3
# for base and classic (blend_direct against blend_sort).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6ab6
mkdir -p $O
set -e
export TMPDIR=/tmp
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
GSPLAT_LIB=$(lib ticket) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "direct or band or async" > $O/pytest_ticket.txt 2>&1 || { tail -n 30 $O/pytest_ticket.txt; exit 1; }
tail -n 1 $O/pytest_ticket.txt
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for rep in 1 2; do
  for v in base ticket classic; do
    GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight 3 > $O/emu_${v}_$rep.jsonl 2> $O/emu_${v}_$rep.err
    echo "$v rep$rep $(tail -n 1 $O/emu_${v}_$rep.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"])')"
  done
done
for v in base ticket; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 400 python3 tools/band_emulate.py --balanced --bands 8 --inflight 3 > $O/bands_${v}.jsonl 2> $O/bands_${v}.err
  echo "$v $(tail -n 1 $O/bands_${v}.jsonl | cut -c1-330)"
done
top() { python3 - "$1" <<'PY'
import sqlite3, sys, glob
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
for r in sqlite3.connect(db).execute("select name, total_calls, average from top_kernels limit 8"):
    print(f"{r[0][:70]:70s} {r[1]:6d} {r[2]/1e3 if r[2] > 1000 else r[2]:8.2f}")
PY
}
for v in base ticket classic; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o band3 -- python3 $EMU --inflight 3 > $O/prof_$v.log 2>&1
  echo "== $v"; top $O/prof_$v
done
for v in base classic; do
  GSPLAT_LIB=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d $O/pmc_bytes_$v -o band3 -- python3 $EMU --inflight 3 --steps 60 > $O/pmc_bytes_$v.log 2>&1
  GSPLAT_LIB=$(lib $v) timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d $O/pmc_sq_$v -o band3 -- python3 $EMU --inflight 3 --steps 60 > $O/pmc_sq_$v.log 2>&1
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for v in ("base", "classic"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for kind in ("bytes", "sq"):
        for f in glob.glob(f"{O}/pmc_{kind}_{v}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].split("::")[-1]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                if r["Counter_Name"] in ("FETCH_SIZE", "SQ_WAVES"):
                    n[(k, r["Counter_Name"])] += 1
    for k, d in agg.items():
        if not any(s in k for s in ("blend", "project", "agg_", "totals")):
            continue
        L = n[(k, "FETCH_SIZE")] or 1; S = n[(k, "SQ_WAVES")] or 1
        print(v, k, {c: round(x / (L if c in ("FETCH_SIZE", "WRITE_SIZE") else S), 1) for c, x in sorted(d.items())})
PY
