mkdir -p gpurun_out/r6i
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_sequence.py tests/test_gpu_paths.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6i/tests.log 2>&1 || exit 1
for r in 1 2 3; do for lib in tree base; do
  if [ $lib = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=_ab/$lib/liborbfe.so; fi
  a=$(timeout -k 10 120 python tools/microbench.py --pairs 512 --rounds 2 --reps 5 2:0 2>/dev/null | tail -1) || exit 1
  b=$(timeout -k 10 120 python tools/microbench.py --pairs 8 --rounds 3 --reps 50 2:0 2>/dev/null | tail -1) || exit 1
  c=$(timeout -k 10 120 python tools/small_batch.py --handles 3 --graphs 0 --no-frame --steps 400 2>/dev/null | tail -1) || exit 1
  echo "round $r $lib: 512p $a | 8p $b | share $c" >> gpurun_out/r6i/octree_ab.log
done; done
