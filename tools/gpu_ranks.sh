#!/bin/bash
# Every rank of the 8-GPU K4-family run (scale 23), one at a time on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ranks}
mkdir -p $OUT
for r in ${RANKS:-0 1 2 3 4 5 6 7}; do
  timeout -k 10 300 python bench.py --gpus ${NG:-8} --as-rank $r --steps 3 --warmup 1 --no-cpu-baseline > $OUT/rank$r.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; d=json.load(open('$OUT/rank$r.json')); print('rank $r', d['as_rank']['rows'], d['as_rank']['flops'], d['value'], d['ms_per_step'], d['phases_ms_rank0'])"
done
