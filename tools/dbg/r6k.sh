mkdir -p gpurun_out/r6k
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_paths.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r6k/tests.log 2>&1 || exit 1
for r in 1 2; do for lib in tree base; do
  if [ $lib = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=_ab/$lib/liborbfe.so; fi
  a=$(timeout -k 10 120 python tools/microbench.py --pairs 512 --rounds 2 --reps 5 0:0 2>/dev/null | tail -1) || exit 1
  echo "round $r $lib: $a" >> gpurun_out/r6k/resize_ab.log
done; done
