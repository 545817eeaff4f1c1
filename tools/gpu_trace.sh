#!/bin/bash
# Concurrent-schedule kernel traces (rocprofv3 --kernel-trace) of bench configs (CFGS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-trace}
mkdir -p $OUT
for c in ${CFGS:-k3p}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_$c -o run --output-format csv -- \
     python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor > $OUT/tr_$c.json 2> $OUT/tr_$c.err || exit $?
done
