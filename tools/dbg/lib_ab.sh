#!/bin/bash
# Same-box A/B of the in-tree library against variant builds (pyorbslam_amd/_lib/variants/NAME/liborbfe.so):
# the 4-handle step (tools/dbg/env_sweep.py, one configuration) and the standalone octree stage, alternating.
# usage: bash tools/dbg/lib_ab.sh NAME [NAME ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for r in 1 2; do
  for lib in tree "$@"; do
    if [ "$lib" = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=pyorbslam_amd/_lib/variants/$lib/liborbfe.so; fi
    v=$(timeout -k 10 120 python tools/dbg/env_sweep.py --var ORBFE_OCT_V --rounds 2 =0 2>/dev/null | tail -1) || exit 1
    st=$(timeout -k 10 120 python bench.py --roofline-only --cpu-sample 0 --allow-dev-env 2>/dev/null | tail -1 | python -c "import sys,json; print(json.loads(sys.stdin.read())['stage_ms_standalone_step'])") || exit 1
    echo "round $r lib $lib: $v | standalone $st"
  done
done
