#!/bin/bash
# Round 6 A/Bs: (1) xb5 -- a band renderer without the aggregated scan and
# emit launches after its first frames (what the two launches cost the band
# chain); (2) expm -- the blend's in-range exponential with the magic-number
# rint (parity tests first, then interleaved config-3 bench lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6ab2
mkdir -p $O
set -e
lib() { [ "$1" = base ] && echo "$PWD/gaussian_splat_ipu_amd/lib/libgsplat.so" || echo "$PWD/tmp_ab/$1/libgsplat.so"; }
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 300"
for rep in 1 2; do
  for v in base xb5; do
    for f in 1 3; do
      GSPLAT_LIB=$(lib $v) timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_${v}_f${f}_$rep.jsonl 2> $O/emu_${v}_f${f}_$rep.err
      echo "$v f$f rep$rep $(tail -n 1 $O/emu_${v}_f${f}_$rep.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["slowest_us"], d["slowest_band_stage_us"])')"
    done
  done
done
GSPLAT_LIB=$(lib expm) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_expm.txt 2>&1
tail -n 1 $O/pytest_expm.txt
for rep in 1 2 3; do
  for v in base expm; do
    GSPLAT_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 600 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    python3 - $v $O/bench_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], {k: round(1e3 * v["avg_ms"], 1) for k, v in d["kernels"].items()})
PY
  done
done
