#!/bin/bash
# Same-box microbench A/B of library builds (tree = the in-tree library, NAME = pyorbslam_amd/_lib/variants/NAME),
# alternating, every stage standalone at --pairs P.  usage: bash tools/dbg/mb_ab.sh P NAME [NAME ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
p=$1; shift
for r in 1 2; do
  for lib in tree "$@"; do
    if [ "$lib" = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=pyorbslam_amd/_lib/variants/$lib/liborbfe.so; fi
    v=$(timeout -k 10 120 python tools/microbench.py --pairs "$p" --rounds 2 --reps 10 0:0 1:0 2:0 3:0 4:0 2>/dev/null | tail -1) || exit 1
    echo "round $r lib $lib pairs $p: $v"
  done
done
