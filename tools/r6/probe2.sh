#!/bin/bash
# Round 6: the projection's share of the pipelined band frame (GS_X_BAND=3:
# no projection after a renderer's first frame), frames in flight 1-6, and
# the VALU issue-rate table with the compiler-emitted forms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/r6band
mkdir -p $O
set -e
timeout -k 10 120 tools/hip/valu_rate > $O/valu_rate.json
tail -n 8 $O/valu_rate.json
EMU="tools/band_emulate.py --balanced --bands 8 --only-band 3 --steps 200"
for f in 1 3; do
  GSPLAT_LIB=$PWD/tmp_x/xb3/libgsplat.so timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_xb3_f$f.jsonl 2> $O/emu_xb3_f$f.err
  echo "xb3 f$f $(tail -n 1 $O/emu_xb3_f$f.jsonl | cut -c1-100) $(tail -n 1 $O/emu_xb3_f$f.jsonl | grep -o '"slowest_band_stage.*')"
done
for f in 2 3 4 6; do
  timeout -k 10 200 python3 $EMU --inflight $f > $O/emu_base_f${f}b.jsonl 2> $O/emu_base_f${f}b.err
  echo "base f$f $(tail -n 1 $O/emu_base_f${f}b.jsonl | grep -o '"slowest_us[^,]*')"
done
