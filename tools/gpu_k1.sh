#!/bin/bash
# K1 through CSR and DIA (bench lines) and a kernel + runtime trace of the CSR step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/${TAG:-k1}
mkdir -p $OUT
B="python bench.py --config k1 --steps 50 --warmup 5 --no-cpu-baseline --no-host-e2e --no-anchor --no-one-shot"
timeout -k 10 200 $B > $OUT/k1.json 2> $OUT/k1.err || exit $?
timeout -k 10 200 $B --format dia > $OUT/k1dia.json 2> $OUT/k1dia.err || exit $?
for f in k1 k1dia; do python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('phases_ms_rank0'))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --runtime-trace -d $OUT/tr -o run --output-format csv -- \
  python $R/bench.py --config k1 --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e --no-anchor --no-one-shot > $OUT/tr.log 2>&1
