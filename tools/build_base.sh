#!/bin/bash
# Build libwtprune.so from a git revision (default HEAD) into tools/ab/libwtprune_base.so, for
# same-box A/B runs against the working tree (tools/gpu_ab.sh).  tools/ab/ travels to the GPU
# box (.so files are git-ignored, not gpurun-ignored).
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/w/csrc $T/include $R/tools/ab
for f in $(git -C $R ls-tree --name-only $REV wavelettransforms_amd/csrc/); do git -C $R show $REV:$f > $T/w/csrc/$(basename $f); done
for f in $(git -C $R ls-tree --name-only $REV include/); do git -C $R show $REV:$f > $T/include/$(basename $f); done
cd $T/w/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -I. -I../../include \
  -o $R/tools/ab/libwtprune_base.so kernels.hip filterbank.hip small.hip api.hip
rm -rf $T
echo "built tools/ab/libwtprune_base.so from $REV"
