#!/bin/bash
# Same-box A/B of the frame path (tools/dbg/frame_extract_time.py) for the in-tree library against
# variants/NAME.  usage (GPU box): bash tools/dbg/fx_ab.sh NAME
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for r in 1 2; do
  for lib in tree "$1"; do
    if [ "$lib" = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=pyorbslam_amd/_lib/variants/$lib/liborbfe.so; fi
    echo "round $r lib $lib"
    timeout -k 10 120 python tools/dbg/frame_extract_time.py 200 2>/dev/null | head -4 || exit 1
  done
done
