# resize-only tree vs base (HEAD) vs s1 (resize + stereo winner x carried through the reduction): stereo parity
# of s1, then same-box A/B
mkdir -p gpurun_out/r6m
ORBFE_LIB=_ab/s1/liborbfe.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stereo.py -x -q --timeout 250 --timeout-method thread \
  > gpurun_out/r6m/pytest_s1.log 2>&1 || { tail -30 gpurun_out/r6m/pytest_s1.log; exit 1; }
tail -1 gpurun_out/r6m/pytest_s1.log
AB_ROUNDS=3 bash tools/dbg/ab.sh tree base s1 > gpurun_out/r6m/ab.log 2>&1 || { cat gpurun_out/r6m/ab.log; exit 1; }
cat gpurun_out/r6m/ab.log
