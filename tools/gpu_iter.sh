#!/bin/bash
# Iteration session: GPU tests, then bench lines for each A/B environment in
# $AB (space-separated NAME=VAL assignments, "base" = none), then one serial
# rocprofv3 kernel-stats pass of the default.  Steps chained with &&; each
# GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-iter}
mkdir -p $OUT
run_tests() {
  if [ -n "$SKIP_TESTS" ]; then return 0; fi
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
}
run_bench() {
  local i=0
  for ab in ${AB:-base}; do
    i=$((i+1))
    if [ "$ab" = "base" ]; then
      timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-} > $OUT/bench_$i.json 2> $OUT/bench_$i.err || return $?
    else
      env $ab timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-} > $OUT/bench_$i.json 2> $OUT/bench_$i.err || return $?
    fi
    echo "$i $ab" >> $OUT/bench_index.txt
  done
}
run_prof() {
  if [ -z "$PROFILE" ]; then return 0; fi
  local i=0
  for ab in ${PROF_AB:-base}; do
    i=$((i+1))
    local e="IAS_SERIAL=1"
    [ "$ab" != "base" ] && e="$e $ab"
    env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial_$i -o run --output-format csv -- \
        python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-} > $OUT/prof_serial_$i.log 2>&1 || return $?
    echo "$i $ab" >> $OUT/prof_index.txt
  done
}
run_tests && run_bench && run_prof
