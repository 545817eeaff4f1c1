#!/bin/bash
# One build, environment variants: K3' and the heaviest 8-GPU rank per
# setting of $VAR (VALS, space-separated), interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-envab}
mkdir -p $OUT
for rep in 1 2; do for v in $VALS; do
  export $VAR=$v
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $OUT/k3p_$v.json 2>> $OUT/err.log || exit 1
  timeout -k 10 300 python bench.py --gpus 8 --as-rank 0 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/r0_$v.json 2>> $OUT/err.log || exit 1
  python3 -c "
import json
a=json.load(open('$OUT/k3p_$v.json')); b=json.load(open('$OUT/r0_$v.json'))
print('$VAR=$v', 'k3p', a['value'], a['phases_ms_rank0']['symbolic'], a['phases_ms_rank0']['numeric'], 'rank0', b['value'], b['phases_ms_rank0']['symbolic'], b['phases_ms_rank0']['numeric'])"
done; done
