#!/bin/bash
# PMC summaries per band shape (bench.pmc_key_of), one --append'ed file:
#   whole   c3 whole frame (bench.py, one frame in flight)
#   bands1  the one-GPU group (bench.py --gather): band 0 of a 1-way split
#   bandsN  band 0 of an N-way balanced split (tools/band_emulate.py
#           --only-band 0): the band a --gpus N line's rank 0 renders
# Passes: kernel trace + stats, FETCH_SIZE, WRITE_SIZE, the SQ set (separate
# runs, never combined with other trace domains).  Output:
# gpurun_out/pmcb/pmc_bands.json (copy to profiles/pmc_latest.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmcb
mkdir -p $O
J=$O/pmc_bands.json
[ -f "${SEED:-profiles/pmc_latest.json}" ] && cp "${SEED:-profiles/pmc_latest.json}" $J
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
shape() {  # shape <name> <key> <python args...>
  local name=$1 key=$2; shift 2
  local d=$O/$name
  mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/stats -o stats --output-format csv -- python3 "$@" > $d/stats.log 2>&1 || return 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $d/fetch -o fetch --output-format csv -- python3 "$@" > $d/fetch.log 2>&1 || return 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $d/write -o write --output-format csv -- python3 "$@" > $d/write.log 2>&1 || return 1
  timeout -s KILL 240 rocprofv3 --pmc $SQ -d $d/sq -o sq --output-format csv -- python3 "$@" > $d/sq.log 2>&1 || return 1
  python3 tools/pmc_summary.py $d --config "$key" --json $J --append > $d/summary.txt 2>&1 || return 1
  echo "== $name $key"; cat $d/summary.txt
}
K=c3:1000000@1920x1080/t16
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --inflight 1"
E="tools/band_emulate.py --balanced --only-band 0 --inflight 1 --steps 20 --warmup 3"
for s in ${SHAPES:-whole bands1 bands2 bands4 bands8}; do
  case $s in
    whole) shape $s $K/whole $B || exit 1 ;;
    bands1) shape $s $K/bands1/band0 $B --gather || exit 1 ;;
    bands*) n=${s#bands}; shape $s $K/bands$n/band0 $E --bands $n || exit 1 ;;
  esac
done
python3 -c "import json; print(sorted(json.load(open('$J'))['summaries']))"
