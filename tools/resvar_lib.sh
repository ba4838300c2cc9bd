#!/bin/bash
# Build tools/ab/libwtprune_<v>.so from the in-tree csrc/ with the sed edits of tools/resvar/<v>.sed
# (one "FILE<TAB>sed-expression" a line).  Usage: bash tools/resvar_lib.sh v1 [v2 ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/tools/ab
build_one() {
  v=$1
  T=$(mktemp -d); mkdir -p $T/w $T/include; cp $R/include/*.h $T/include/; cp -r $R/wavelettransforms_amd/csrc $T/w/csrc
  while IFS=$'\t' read -r f e; do [ -z "$f" ] && continue
    cp $T/w/csrc/$f $T/o; sed -i "$e" $T/w/csrc/$f
    if cmp -s $T/o $T/w/csrc/$f; then echo "variant $v: '$e' changed nothing in $f" >&2; exit 1; fi
  done < $R/tools/resvar/$v.sed
  (cd $T/w/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -I. -I../../include \
    -o $R/tools/ab/libwtprune_$v.so kernels.hip filterbank.hip small.hip api.hip)
  rm -rf $T
  echo "built tools/ab/libwtprune_$v.so"
}
# the variants in parallel (at most 4 at once), each in its own temp tree
n=0
for v in "$@"; do
  build_one $v &
  n=$((n + 1))
  if [ $n -ge 4 ]; then wait -n; n=$((n - 1)); fi
done
wait
