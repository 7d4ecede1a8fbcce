set -o pipefail
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1_test.log 2>&1 || { tail -20 gpurun_out/ab1_test.log; exit 1; }
tail -2 gpurun_out/ab1_test.log
for lib in "" HEAD; do
  if [ -n "$lib" ]; then export ORBFE_LIB=pyorbslam_amd/_lib/variants/$lib/liborbfe.so; else unset ORBFE_LIB; fi
  echo "lib=${lib:-tree}"; timeout -k 10 120 python tools/microbench.py --pairs 256 --rounds 3 1:0 2>&1 | grep detect || exit 1
done
timeout -k 10 400 bash tools/ab_bench.sh "--steps 20 --warmup 5" HEAD
