#!/bin/bash
# build_x.sh <name> "<-D flags>": a compile-time measurement variant of
# libgsplat.so in tmp_ab/<name>/ (the sources as they are, built with the
# flags in a scratch copy; the in-tree build is untouched).  The variant
# switches are the GS_X_* macros in csrc/ (0 = the product).
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
root=/tmp/vx_$name
rm -rf $root && mkdir -p $root/gaussian_splat_ipu_amd
cp -r include $root/ && cp -r gaussian_splat_ipu_amd/csrc $root/gaussian_splat_ipu_amd/ && rm -rf $root/gaussian_splat_ipu_amd/csrc/build
make -s -j8 -C $root/gaussian_splat_ipu_amd/csrc ../lib/libgsplat.so XFLAGS="$flags"
mkdir -p ${ABDIR:-tmp_ab}/$name && cp $root/gaussian_splat_ipu_amd/lib/libgsplat.so ${ABDIR:-tmp_ab}/$name/
echo "built ${ABDIR:-tmp_ab}/$name/libgsplat.so ($flags)"
