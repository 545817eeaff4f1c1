set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r5prof NAMES=cur REPS=1 TRACE_LIB=cur HIPTRACE=1 bash tools/gpu_ab.sh > gpurun_out/r5prof_ab.log 2>&1 || exit 3
IAS_SERIAL=1 TAG=r5prof/pmc PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" bash tools/pmc.sh > gpurun_out/r5prof_pmc.log 2>&1 || exit 4
python3 tools/pmc_kernels.py gpurun_out/r5prof/pmc "k_" > gpurun_out/r5prof/pmc_summary.txt
tail -3 gpurun_out/r5prof/ab_summary.txt
