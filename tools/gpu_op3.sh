#!/bin/bash
# Engine comparison on the BASELINE configs (K1 band, K2 ELL, K3' R-MAT).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-op3}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
for cfg in k1 k2 k3p; do
  for eng in twophase onepass; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --config $cfg --engine $eng > $OUT/bench_${cfg}_${eng}.json 2> $OUT/bench_${cfg}_${eng}.err || exit 1
  done
done
tail -2 $OUT/pytest_gpu.log
for f in $OUT/bench_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['ms_per_launch'])"; done
