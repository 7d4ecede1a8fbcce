#!/bin/bash
# Same-box A/B of library builds: the default 4-handle 512-pair step (tools/dbg/env_sweep.py, one configuration)
# and every stage standalone at 512 pairs (tools/microbench.py), alternating over AB_ROUNDS rounds (default 3).
# LIB "tree" = the in-tree library, NAME = _ab/NAME/liborbfe.so (tools/dbg/ab_prep.sh).
# usage: bash tools/dbg/ab.sh tree NAME [NAME ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=${AB_ROUNDS:-3}
for r in $(seq 1 "$R"); do
  for lib in "$@"; do
    if [ "$lib" = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=_ab/$lib/liborbfe.so; fi
    v=$(timeout -k 10 120 python tools/dbg/env_sweep.py --var ORBFE_AB --rounds 1 --steps 30 =0 2>/dev/null | tail -1) || exit 1
    m=$(timeout -k 10 120 python tools/microbench.py --pairs 512 --rounds 2 --reps 5 2>/dev/null | tail -1) || exit 1
    echo "round $r lib $lib: $v | $m"
  done
done
