#!/bin/bash
# One K4 shard (rank R of 8, default 4): serial per-kernel stats and a
# concurrent timeline of its step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${R:-4}
OUT=gpurun_out/${TAG:-k4rank$R}
mkdir -p $OUT
IAS_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/serial -o run --output-format csv -- \
  python bench.py --gpus 8 --as-rank $R --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e \
  > $OUT/serial.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial/run_kernel_stats.csv 4 > $OUT/serial_kstats.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python bench.py --gpus 8 --as-rank $R --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e \
  > $OUT/trace.log 2>&1 || exit $?
python3 tools/timeline.py $OUT/trace/run_kernel_trace.csv k_an_entries -2 > $OUT/timeline.txt
