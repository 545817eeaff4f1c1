#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only, as
# MI355X_MICROARCH.md prescribes) over a short bench run; CSVs -> $OUT/pmc_<i>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
CMD="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-weak-anchor ${BENCH_ARGS:-}"
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-trace --output-format csv -d $OUT/pmc_$i -o p -- $CMD > $OUT/pmc_$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc: $group" >> $OUT/pmc_status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
done < <(if [ -n "$PMC_GROUPS" ]; then printf '%s\n' "$PMC_GROUPS" | tr ';' '\n'; else cat <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GROUPS
fi)
