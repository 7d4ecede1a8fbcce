mkdir -p gpurun_out/r6h
timeout -k 10 170 python tools/rccl_probe.py > gpurun_out/r6h/rccl_probe.log 2>&1
echo "rc=$?" >> gpurun_out/r6h/rccl_probe.log
