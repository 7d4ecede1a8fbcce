#!/bin/bash
# k_orb keypoints per wave, standalone (tools/microbench.py, dev build): variant 0 = production choice (8 for big
# batches), 10 = 16 keypoints per wave, 9 = 4.  usage (GPU box): bash tools/dbg/orb_kpw.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export ORBFE_LIB=pyorbslam_amd/_lib/variants/dev/liborbfe.so
for r in 1 2; do
  timeout -k 10 120 python tools/microbench.py --pairs 256 --rounds 2 --reps 10 3:0 3:10 3:9 2>/dev/null | tail -1 || exit 1
done
