#!/bin/bash
# Partition buckets on/off: GPU parity tests, K3' bench both ways, serial
# kernel profile, and the heaviest / lightest rank of the 8-GPU K4-family run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pb}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for pb in 1 0 1; do export IAS_PART_BUCKET=$pb;
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/bench_pb$pb.json 2>> $OUT/bench.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench_pb$pb.json')); print('pb$pb', d['value'], d['ms_per_step'], d['phases_ms_rank0'])"
done
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv 7 | head -14
for r in 0 7; do
  timeout -k 10 400 python bench.py --gpus 8 --as-rank $r --steps 3 --warmup 1 --no-cpu-baseline > $OUT/k4_rank$r.json 2>> $OUT/bench.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/k4_rank$r.json')); print('k4 rank $r', d['value'], d['ms_per_step'], d['phases_ms_rank0'])"
done
