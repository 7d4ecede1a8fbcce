mkdir -p gpurun_out/r6g
timeout -k 10 200 python tools/microbench.py --pairs 512 --rounds 2 --reps 5 0:0 0:104 0:108 0:116 0:132 > gpurun_out/r6g/resize_cascade_512.log 2>&1 || exit 1
