#!/bin/bash
# Row-block pipeline (ias_csr_mul_csr_into, bench --engine pipe) against the
# two-phase engine, then the full-size parity tests, then the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3h}
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-e2e"
for e in pipe twophase; do
  timeout -k 10 300 $B --engine $e > $OUT/bench_$e.json 2> $OUT/bench_$e.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/bench_$e.json')); print('$e', d['value'], d['ms_per_step'], d['phases_ms_rank0'])"
done
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py tests/test_format_fullsize.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_full.log 2>&1; rc=$?
tail -15 $OUT/pytest_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
exit $rc
