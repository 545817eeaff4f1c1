#!/bin/bash
# Kernel profile of the heaviest rank (rank 0 of 8, scale 23) and K3' bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-k4prof}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "long or tiers or collisions or wide or edges" > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/bench.json 2>> $OUT/bench.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('k3p', d['value'], d['ms_per_step'], d['phases_ms_rank0'])"
IAS_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof0 -o run --output-format csv -- \
      python bench.py --gpus 8 --as-rank 0 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof0.log 2>&1 || exit 1
python3 tools/kstats.py $OUT/prof0/run_kernel_stats.csv 4 | head -22
