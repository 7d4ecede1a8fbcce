# st3 = tree + the sheared windows' padded (row, col) from one float-reciprocal divmod per lane (shared by the
# left and right views) instead of two signed divisions: parity of st3, then same-box A/B
mkdir -p gpurun_out/r6o
export ORBFE_LIB=_ab/st3/liborbfe.so
timeout -k 10 700 python -u -m pytest tests/test_gpu_stereo.py tests/test_gpu_paths.py tests/test_gpu_extract.py -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r6o/pytest_st3.log 2>&1 || { tail -30 gpurun_out/r6o/pytest_st3.log; exit 1; }
tail -1 gpurun_out/r6o/pytest_st3.log
unset ORBFE_LIB
AB_ROUNDS=3 bash tools/dbg/ab.sh tree st3 > gpurun_out/r6o/ab.log 2>&1 || { cat gpurun_out/r6o/ab.log; exit 1; }
cat gpurun_out/r6o/ab.log
