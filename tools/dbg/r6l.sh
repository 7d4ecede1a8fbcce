# resize staging (guarded buffer loads, resource halves as uint32_t) + 2-row unrolled tap reuse, stereo search branch-free + winner x
# carried through the reduction: parity first (the batch path at 4 500 px that faulted the unguarded staging),
# then same-box A/B
mkdir -p gpurun_out/r6l
timeout -k 10 200 python -u -m pytest "tests/test_gpu_extract.py::test_level_sides_above_4095_px_frame_and_batch" -x -q --timeout 150 --timeout-method thread \
  > gpurun_out/r6l/pytest0.log 2>&1 || { tail -30 gpurun_out/r6l/pytest0.log; exit 1; }
tail -1 gpurun_out/r6l/pytest0.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_paths.py tests/test_gpu_stereo.py -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r6l/pytest.log 2>&1 || { tail -30 gpurun_out/r6l/pytest.log; exit 1; }
tail -1 gpurun_out/r6l/pytest.log
AB_ROUNDS=3 bash tools/dbg/ab.sh tree base > gpurun_out/r6l/ab.log 2>&1 || { cat gpurun_out/r6l/ab.log; exit 1; }
cat gpurun_out/r6l/ab.log
