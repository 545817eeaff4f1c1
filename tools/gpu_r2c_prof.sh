#!/bin/bash
# Serial kernel-stats passes (IAS_SERIAL=1) of the configs in $CFGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2c_prof}
mkdir -p $OUT
for cfg in ${CFGS:-k2 k1}; do
  IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$cfg -o run --output-format csv -- \
     python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e > $OUT/prof_$cfg.log 2>&1 || exit $?
done
