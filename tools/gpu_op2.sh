#!/bin/bash
# Single-pass engine: full GPU tests, bench (both engines), kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-op2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_onepass.json 2> $OUT/bench_onepass.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --engine twophase > $OUT/bench_twophase.json 2> $OUT/bench_twophase.err &&
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
cat $OUT/bench_onepass.json $OUT/bench_twophase.json
exit $rc
