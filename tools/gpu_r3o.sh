#!/bin/bash
# bench + k_num2 FETCH/WRITE PMC + the GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3o}
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"
for c in FETCH_SIZE WRITE_SIZE; do
  IAS_SERIAL=1 timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$c -o p -- \
     python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-e2e --no-anchor --no-one-shot > $OUT/pmc_$c.log 2>&1 || exit $?
done
python3 tools/pmc_kernels.py $OUT "k_num2$|k_sym3|k_sym2" | tee $OUT/pmc.txt | head -40
[ -n "$NOTEST" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
exit $rc
