#!/bin/bash
# K3: serial per-kernel stats and a concurrent timeline of one step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-k3prof}
mkdir -p $OUT
IAS_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/serial -o run --output-format csv -- \
  python bench.py --config k3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor \
  > $OUT/serial.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial/run_kernel_stats.csv 4 > $OUT/serial_kstats.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python bench.py --config k3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor \
  > $OUT/trace.log 2>&1 || exit $?
python3 tools/timeline.py $OUT/trace/run_kernel_trace.csv k_an_entries -2 > $OUT/timeline.txt
