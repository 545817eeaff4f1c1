#!/bin/bash
# Round 3 baseline: K3' bench as shipped, the same with the sym2 gathers
# ablated (IAS_S2_ABLATE=2: column = product index), and a serial kernel
# profile (IAS_SERIAL=1) — where the symbolic time goes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3a}
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-e2e"
timeout -k 10 300 $B > $OUT/bench.json 2> $OUT/bench.err &&
IAS_S2_ABLATE=2 timeout -k 10 300 $B > $OUT/bench_abl2.json 2> $OUT/bench_abl2.err &&
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e > $OUT/prof.log 2>&1
rc=$?
for f in bench bench_abl2; do
  python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['ms_per_launch'])"
done
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv 7 2>/dev/null | head -40
[ $rc -eq 0 ] && timeout -k 10 400 python -u -m pytest tests/test_multi_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_multi.log 2>&1; rc=$?
tail -25 $OUT/pytest_multi.log
exit $rc
