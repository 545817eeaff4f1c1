#!/bin/bash
# Round-2 closing iteration: GPU suite, then A/B variants on K2 / K1 / K3'.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2c}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
for cfg in ${CFGS:-k2 k1 k3p}; do
  for name in $NAMES; do
    IAS_LIB=$PWD/build_var/libias_$name.so timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-20} --warmup 3 \
       --no-cpu-baseline --no-host-e2e > $OUT/bench_${cfg}_$name.json 2> $OUT/bench_${cfg}_$name.err || exit $?
    echo "$cfg $name $(python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_$name.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'],d['roofline']['ms_per_launch'],d['roofline']['frac'])")" >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
