#!/bin/bash
# Rehearse the heaviest rank of the 8-GPU K4-family run (scale 23, rank 0 holds
# the R-MAT hub rows) on one GPU: parity-free size check of the int64 paths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-k4rank}
mkdir -p $OUT
for r in ${RANKS:-0 7}; do
  timeout -k 10 400 python bench.py --gpus 8 --as-rank $r --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_rank$r.json 2> $OUT/bench_rank$r.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/bench_rank$r.json')); print($r, d['value'], d['ms_per_step'], d['as_rank'], d['phases_ms_rank0'], d['config']['nnz_c'])"
done
