#!/bin/bash
# Shipped library vs variants (VARS), serial kernel stats of each, GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3g}
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-}"
timeout -k 10 300 $B > $OUT/bench.json 2> $OUT/bench.err || exit $?
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-} > $OUT/prof.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('shipped', d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['ms_per_launch'])"
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv 7 | grep -E "${KPAT:-sym|num2}" | sed "s/^/shipped /"
if [ -n "$VARS" ]; then
  TAG=${TAG:-r3g}/var NAMES="$VARS" PROFILE=1 STEPS=20 bash tools/run_variants.sh || exit $?
  for n in $VARS; do python3 tools/kstats.py $OUT/var/prof_$n/run_kernel_stats.csv 7 | grep -E "${KPAT:-sym|num2}" | sed "s/^/$n /"; done
fi
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu.log
  exit $rc
fi
