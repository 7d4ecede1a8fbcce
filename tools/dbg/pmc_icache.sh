#!/bin/bash
# Instruction-cache counters per kernel: the 4-stream step (all kernels co-resident) and the standalone
# stage pass (one kernel at a time). usage: bash tools/dbg/pmc_icache.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
C="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE"
timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_ic_step -o run -- python bench.py --cpu-sample 0 --no-parity --roofline-steps 0 --no-c4 --no-host-fed --no-c3 --steps 5 --warmup 2 > gpurun_out/pmc_ic_step.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_ic_solo -o run -- python bench.py --roofline-only --roofline-steps 2 > gpurun_out/pmc_ic_solo.log 2>&1 || exit 1
python tools/pmc_agg.py gpurun_out/pmc_ic_step gpurun_out/pmc_ic_solo > gpurun_out/pmc_ic_summary.txt 2>&1
