#!/bin/bash
# Iteration loop on the box: GPU parity tests, K3' bench, serial kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err &&
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv 7 2>/dev/null | head -30
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['ms_per_launch'])"
exit $rc
