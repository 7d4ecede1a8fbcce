# d1 = s2 (next bucket slots prefetched in the stereo search) + k_detect ROI loads unconditional through a
# level-bounded resource: parity of d1 (covers s2), then same-box A/B tree (s1) / s2 / d1
mkdir -p gpurun_out/r6n
export ORBFE_LIB=_ab/d1/liborbfe.so
timeout -k 10 700 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_paths.py tests/test_gpu_stereo.py -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r6n/pytest_d1.log 2>&1 || { tail -30 gpurun_out/r6n/pytest_d1.log; exit 1; }
tail -1 gpurun_out/r6n/pytest_d1.log
unset ORBFE_LIB
AB_ROUNDS=3 bash tools/dbg/ab.sh tree s2 d1 > gpurun_out/r6n/ab.log 2>&1 || { cat gpurun_out/r6n/ab.log; exit 1; }
cat gpurun_out/r6n/ab.log
