#!/bin/bash
# Same-box A/B of k_octree_bins' level-group split (ORBFE_OCT_SPLIT: first level of the second launch,
# -1 = one launch): parity of the extractor tests under a forced split, then per split the octree stage
# standalone (tools/microbench.py) and the default 4-handle step (tools/dbg/env_sweep.py), KITTI and EuRoC.
# The knob lived in the reverted experiment build (launch_octree's level groups with per-group LDS carves,
# profiles/r03/octree_split_ab*_r3f.log); on the current tree every setting runs the one-launch kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/oct_split
ORBFE_OCT_SPLIT=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 250 \
  --timeout-method thread > gpurun_out/oct_split/pytest_split3.log 2>&1 || { tail -20 gpurun_out/oct_split/pytest_split3.log; exit 1; }
tail -1 gpurun_out/oct_split/pytest_split3.log
for r in 1 2; do
  for sp in ${SPLITS:--1 3}; do
    m=$(ORBFE_OCT_SPLIT=$sp timeout -k 10 120 python tools/microbench.py --pairs 256 --rounds 3 2:0 2>/dev/null | tail -1) || exit 1
    st=$(ORBFE_OCT_SPLIT=$sp timeout -k 10 120 python tools/dbg/env_sweep.py --var ORBFE_NONE --rounds 2 =0 2>/dev/null | tail -1) || exit 1
    eu=$(ORBFE_OCT_SPLIT=$sp timeout -k 10 200 python bench.py --width 752 --height 480 --nfeatures 1000 --cpu-sample 0 --no-c3 \
         --no-c4 --no-host-fed --no-parity 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_standalone_step']['octree'])") || exit 1
    echo "round $r split $sp: octree $m | step $st | euroc pairs/s, octree ms: $eu"
  done
done
