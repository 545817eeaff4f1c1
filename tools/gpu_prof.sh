#!/bin/bash
# Serial kernel stats (IAS_SERIAL=1, rocprofv3 --kernel-trace --stats) of the
# configs in CFGS (default k3p), one directory each under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
for c in ${CFGS:-k3p}; do
  IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$c -o run --output-format csv -- \
     python bench.py --config $c --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-host-e2e --no-anchor \
     --no-one-shot > $OUT/$c.log 2>&1 || exit $?
  python3 tools/kstats.py $OUT/$c/run_kernel_stats.csv $((${STEPS:-5} + 2 + ${EXTRA:-1})) > $OUT/$c.txt
  head -30 $OUT/$c.txt
done
