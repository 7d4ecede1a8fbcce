mkdir -p gpurun_out/r6g
timeout -k 10 200 python tools/microbench.py --pairs 512 --rounds 3 --reps 5 0:0 0:6 0:7 0:132 0:164 > gpurun_out/r6g/resize_cascade_512.log 2>&1 || exit 1
timeout -k 10 200 python tools/microbench.py --pairs 128 --rounds 3 --reps 5 0:0 0:6 0:7 > gpurun_out/r6g/resize_cascade_128.log 2>&1
