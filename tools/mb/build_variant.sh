#!/bin/bash
# Build a lab variant of libwtprune.so from the in-tree sources with a sed edit applied to a temp
# copy: tools/mb/build_variant.sh NAME 'sed-expression' [file]  ->  tools/mb/libwtprune_NAME.so
set -e
N=$1; E=$2; F=${3:-wtp_internal.h}
R=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
mkdir -p $T/w $T/include; cp -r $R/wavelettransforms_amd/csrc $T/w/csrc; cp $R/include/*.h $T/include/
sed -i "$E" $T/w/csrc/$F
cd $T/w/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -I. -I../../include \
  -o $R/tools/mb/libwtprune_$N.so kernels.hip filterbank.hip small.hip api.hip
rm -rf $T
