set -o pipefail
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
bash tools/pmc_run.sh gpurun_out/pmc_orb_tree "$C1" "$C2" -- python tools/microbench.py --pairs 256 --rounds 2 3:0 > gpurun_out/pmc_orb_tree.log 2>&1 || exit 1
ORBFE_LIB=pyorbslam_amd/_lib/variants/base/liborbfe.so bash tools/pmc_run.sh gpurun_out/pmc_orb_base "$C1" "$C2" -- python tools/microbench.py --pairs 256 --rounds 2 3:0 > gpurun_out/pmc_orb_base.log 2>&1 || exit 1
python tools/pmc_agg.py gpurun_out/pmc_orb_tree/p0 gpurun_out/pmc_orb_tree/p1 gpurun_out/pmc_orb_base/p0 gpurun_out/pmc_orb_base/p1 > gpurun_out/pmc_orb_summary.txt 2>&1
