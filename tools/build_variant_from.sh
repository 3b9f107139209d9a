#!/bin/bash
# build_variant_from.sh <name> <git-rev> [edit.py ...]: the csrc + include of
# <git-rev>, each edit script applied in turn (run inside csrc/), built into
# tmp_ab/<name>/libgsplat.so (A/B experiments; tmp_ab/ is not committed).
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2; shift 2
root=/tmp/v_$name
rm -rf $root && mkdir -p $root
git archive "$rev" include gaussian_splat_ipu_amd/csrc | tar -x -C $root
for e in "$@"; do (cd $root/gaussian_splat_ipu_amd/csrc && python3 "$e"); done  # (absolute paths)
make -s -C $root/gaussian_splat_ipu_amd/csrc ../lib/libgsplat.so
mkdir -p ${ABDIR:-tmp_ab}/$name && cp $root/gaussian_splat_ipu_amd/lib/libgsplat.so ${ABDIR:-tmp_ab}/$name/
