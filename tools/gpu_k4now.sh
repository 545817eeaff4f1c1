#!/bin/bash
# K4 now: whole K4 on one GPU (serial per-kernel stats + the bench line) and
# the 8-shard rehearsal (each rank's shard one at a time on this GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-k4now}
mkdir -p $OUT
B="python bench.py"
timeout -k 10 600 $B --gpus 8 --as-rank all --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e > $OUT/k4_as_rank_all.jsonl 2> $OUT/k4_as_rank_all.err || exit $?
timeout -k 10 600 $B --config k4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor > $OUT/bench_k4_1gpu.json 2> $OUT/bench_k4_1gpu.err || exit $?
IAS_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/serial -o run --output-format csv -- \
  python bench.py --config k4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor \
  > $OUT/serial.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial/run_kernel_stats.csv 3 > $OUT/serial_kstats.txt
