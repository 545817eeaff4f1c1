#!/bin/bash
# Bench lines (+ serial kernel stats) for the listed configs: CONFIGS="k1 k2".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cfg}
mkdir -p $OUT
for c in ${CONFIGS:-k1 k2}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 3 --no-host-e2e ${BENCH_ARGS:-} \
      > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  if [ -n "$PROFILE" ]; then
    IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- \
        python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-} \
        > $OUT/prof_$c.log 2>&1 || exit $?
  fi
done
