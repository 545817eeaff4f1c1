#!/bin/bash
# sym3 A/B: K3' bench with sym3 (default) and IAS_SYM3=0, serial kernel
# profile, then the GPU parity suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3b}
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-}"
timeout -k 10 300 $B > $OUT/bench.json 2> $OUT/bench.err &&
IAS_SYM3=0 timeout -k 10 300 $B > $OUT/bench_nosym3.json 2> $OUT/bench_nosym3.err &&
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
rc=$?
for f in bench bench_nosym3; do
  python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['ms_per_launch'])"
done
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv 7 2>/dev/null | head -24
[ $rc -eq 0 ] && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -5 $OUT/pytest_gpu.log
exit $rc
