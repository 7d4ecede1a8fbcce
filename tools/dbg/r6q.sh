# orb8w = k_orb at 8 waves per workgroup for batches (6 waves per SIMD: the per-workgroup tables amortised
# over 8 waves fit 3 workgroups per CU in LDS): parity, then same-box A/B against the tree (4 waves)
mkdir -p gpurun_out/r6q
export ORBFE_LIB=_ab/orb8w/liborbfe.so
timeout -k 10 700 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_paths.py tests/test_gpu_stereo.py -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r6q/pytest_orb8w.log 2>&1 || { tail -30 gpurun_out/r6q/pytest_orb8w.log; exit 1; }
tail -1 gpurun_out/r6q/pytest_orb8w.log
unset ORBFE_LIB
AB_ROUNDS=3 bash tools/dbg/ab.sh tree orb8w > gpurun_out/r6q/ab.log 2>&1 || { cat gpurun_out/r6q/ab.log; exit 1; }
cat gpurun_out/r6q/ab.log
