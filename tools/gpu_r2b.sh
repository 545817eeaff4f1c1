#!/bin/bash
# Iteration: GPU suite, K3' / K3 bench lines, kernel traces of K3', K2, K1
# (one pipeline timeline each via tools/timeline.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2b}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-e2e > $OUT/bench_k3p.json 2> $OUT/bench_k3p.err || exit $?
timeout -k 10 300 python bench.py --config k3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e > $OUT/bench_k3.json 2> $OUT/bench_k3.err || exit $?
for cfg in ${TRACE_CFGS:-k3p k2 k1}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_$cfg -o run --output-format csv -- \
      python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e > $OUT/tr_$cfg.json 2> $OUT/tr_$cfg.err || exit $?
done
