#!/bin/bash
# SQ stall / issue counters of one stage standalone (tools/microbench.py STAGE:0, 256 pairs), in-tree library
# and optionally a variant: bash tools/dbg/pmc_stage.sh STAGE OUTNAME [VARIANT]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
st=$1; name=$2; var=$3
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
bash tools/pmc_run.sh gpurun_out/pmc_${name}_tree "$C1" "$C2" -- python tools/microbench.py --pairs 256 --rounds 2 $st:0 > gpurun_out/pmc_${name}_tree.log 2>&1 || exit 1
dirs="gpurun_out/pmc_${name}_tree/p0 gpurun_out/pmc_${name}_tree/p1"
if [ -n "$var" ]; then
  ORBFE_LIB=pyorbslam_amd/_lib/variants/$var/liborbfe.so bash tools/pmc_run.sh gpurun_out/pmc_${name}_$var "$C1" "$C2" -- python tools/microbench.py --pairs 256 --rounds 2 $st:0 > gpurun_out/pmc_${name}_$var.log 2>&1 || exit 1
  dirs="$dirs gpurun_out/pmc_${name}_$var/p0 gpurun_out/pmc_${name}_$var/p1"
fi
python tools/pmc_agg.py $dirs > gpurun_out/pmc_${name}_summary.txt 2>&1
