cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for gr in 0 1; do
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_pyr$gr -o run -- python3 tools/small_trace.py --frame --pyramid 1 --graphs $gr --steps 30 > gpurun_out/kt_pyr$gr.log 2>&1 || exit 1
done
