#!/bin/bash
# PMC counters of the symbolic kernels (K3'): issue / wait / LDS mix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3d}
mkdir -p $OUT
export PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA;SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
TAG=${TAG:-r3d} BENCH_ARGS="--no-host-e2e" bash tools/pmc.sh
rc=$?
cat $OUT/pmc_status.txt
python3 tools/pmc_kernels.py $OUT 'sym3|sym2<(128|256|512)|k_num2$|short_sym<4>' > $OUT/kernels.txt
cat $OUT/kernels.txt
exit $rc
