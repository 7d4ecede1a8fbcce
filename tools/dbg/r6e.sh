mkdir -p gpurun_out/r6e
timeout -k 10 300 python -u -m pytest tests/test_gpu_stereo.py tests/test_sequence.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6e/tests.log 2>&1 || exit 1
AB_ROUNDS=2 bash tools/dbg/ab.sh tree base > gpurun_out/r6e/ab.log 2>&1
