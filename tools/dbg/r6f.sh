mkdir -p gpurun_out/r6f
for r in 1 2; do for lib in tree preblur; do
  if [ $lib = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=_ab/$lib/liborbfe.so; fi
  v=$(timeout -k 10 120 python tools/microbench.py --pairs 512 --rounds 3 --reps 5 3:0 5:0 0:0 2>/dev/null | tail -1) || exit 1
  echo "round $r $lib: $v" >> gpurun_out/r6f/orb_preblur.log
done; done
