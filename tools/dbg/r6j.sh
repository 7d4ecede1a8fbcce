mkdir -p gpurun_out/r6j
timeout -k 10 200 python tools/dbg/matcher_profile.py 96 tottime f_f > gpurun_out/r6j/prof_ff.log 2>&1 || exit 1
timeout -k 10 200 python tools/dbg/matcher_profile.py 96 tottime frame > gpurun_out/r6j/prof_frame.log 2>&1 || exit 1
timeout -k 10 200 python tools/dbg/matcher_profile.py 96 tottime f_p > gpurun_out/r6j/prof_fp.log 2>&1
