#!/bin/bash
# GPU A/B of the in-tree library against variant builds (tools/build_rev.sh): extractor parity tests,
# per-stage microbench of stage $MB_ITEMS, then the default bench alternating libraries.
# usage (gpurun): bash tools/ab_run.sh REV [REV ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
for lib in "" "$@"; do
  if [ -n "$lib" ]; then export ORBFE_LIB=pyorbslam_amd/_lib/variants/$lib/liborbfe.so; else unset ORBFE_LIB; fi
  echo "lib=${lib:-tree}"; timeout -k 10 120 python tools/microbench.py --pairs 256 --rounds 2 ${MB_ITEMS:-1:0} 2>&1 | grep "us per" || exit 1
done
unset ORBFE_LIB
timeout -k 10 400 bash tools/ab_bench.sh "--steps 20 --warmup 5" "$@"
