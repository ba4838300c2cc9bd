#!/bin/bash
# tie-heavy timing (tools/tie_time.py) with the working tree's library and tools/ab/libwtprune_base.so
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for v in new base; do
  L=""; [ $v = base ] && L=$(pwd)/tools/ab/libwtprune_base.so
  echo "== $v"; WTP_LIB_PATH=$L timeout -k 10 300 python tools/tie_time.py || exit 1
done
