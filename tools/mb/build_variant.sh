#!/bin/bash
# Build a lab variant of libwtprune.so from the in-tree sources with sed edits applied to a temp
# copy: tools/mb/build_variant.sh NAME 'sed-expression' [file] [ 'sed-expression' file ... ]
#   ->  tools/ab/libwtprune_NAME.so (tools/ab/ travels to the GPU box)   (file defaults to wtp_internal.h)
set -e
N=$1; shift
R=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
mkdir -p $T/w $T/include; cp -r $R/wavelettransforms_amd/csrc $T/w/csrc; cp $R/include/*.h $T/include/
while [ $# -gt 0 ]; do
  E=$1; F=${2:-wtp_internal.h}; shift; [ $# -gt 0 ] && shift
  cp $T/w/csrc/$F $T/w/csrc/$F.orig
  sed -i "$E" $T/w/csrc/$F
  if cmp -s $T/w/csrc/$F $T/w/csrc/$F.orig; then echo "variant $N: '$E' changed nothing in $F" >&2; exit 1; fi
done
cd $T/w/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -I. -I../../include \
  -o $R/tools/ab/libwtprune_$N.so kernels.hip filterbank.hip small.hip api.hip
rm -rf $T
