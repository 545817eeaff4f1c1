#!/bin/bash
# A change on the box: full GPU suite, K3' bench, heaviest 8-GPU rank, and
# (TIM=1) the per-phase timing build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $OUT/k3p.json 2>> $OUT/err.log || exit 1
timeout -k 10 300 python bench.py --gpus 8 --as-rank 0 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/r0.json 2>> $OUT/err.log || exit 1
python3 -c "
import json
a=json.load(open('$OUT/k3p.json')); b=json.load(open('$OUT/r0.json'))
print('k3p', a['value'], a['ms_per_step'], a['phases_ms_rank0']); print('rank0', b['value'], b['ms_per_step'], b['phases_ms_rank0'])"
if [ -n "$TIM" ]; then TAG=${TAG:-ab}_tim bash tools/timing.sh && cat gpurun_out/${TAG:-ab}_tim/timing.txt; fi
