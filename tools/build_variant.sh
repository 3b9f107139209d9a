#!/bin/bash
# build_variant.sh <name> <python-edit-script>: copy the sources, apply the
# edit (run inside the copied csrc/), build tmp_ab/<name>/libgsplat.so
# (A/B experiments; tmp_ab/ is not committed).
set -e
cd "$(dirname "$0")/.."
name=$1; edit=$(realpath "$2")
root=/tmp/v_$name
rm -rf $root && mkdir -p $root/gaussian_splat_ipu_amd
cp -r include $root/ && cp -r gaussian_splat_ipu_amd/csrc $root/gaussian_splat_ipu_amd/ && rm -rf $root/gaussian_splat_ipu_amd/csrc/build
(cd $root/gaussian_splat_ipu_amd/csrc && python3 "$edit")
make -s -C $root/gaussian_splat_ipu_amd/csrc ../lib/libgsplat.so
mkdir -p ${ABDIR:-tmp_ab}/$name && cp $root/gaussian_splat_ipu_amd/lib/libgsplat.so ${ABDIR:-tmp_ab}/$name/
