mkdir -p gpurun_out/r6d
for r in 1 2; do for lib in dev nosad nosearch; do
  export ORBFE_LIB=_ab/$lib/liborbfe.so
  v=$(timeout -k 10 120 python tools/microbench.py --pairs 512 --rounds 3 --reps 5 4:0 2>/dev/null | tail -1) || exit 1
  echo "round $r $lib: $v" >> gpurun_out/r6d/stereo_abl.log
done; done
unset ORBFE_LIB
timeout -k 10 120 python tools/octree_profile.py --pairs 8 > gpurun_out/r6d/octree_profile_pairs8.log 2>&1
timeout -k 10 120 python tools/octree_profile.py --seq > gpurun_out/r6d/octree_profile_seq.log 2>&1
