#!/bin/bash
# Same-box A/B of one stage standalone (tools/microbench.py STAGE:0) between the in-tree library and
# variants, alternating: bash tools/dbg/stage_ab.sh STAGE NAME [NAME ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
st=$1; shift
for r in 1 2 3; do
  for lib in tree "$@"; do
    if [ "$lib" = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=pyorbslam_amd/_lib/variants/$lib/liborbfe.so; fi
    v=$(timeout -k 10 120 python tools/microbench.py --pairs 256 --rounds 3 $st:0 2>/dev/null | tail -1) || exit 1
    echo "round $r lib $lib: $v"
  done
done
