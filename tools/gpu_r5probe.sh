#!/bin/bash
# Round-5 probes: per-phase timing of the row kernels on K3' (timing build),
# a K1 kernel timeline, and the K3 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5probe}
mkdir -p $OUT
IAS_SERIAL=1 IAS_LIB=$PWD/build_tim/libias.so timeout -k 10 300 python tools/timing_run.py > $OUT/timing_k3p.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k1 -o run --output-format csv -- python bench.py --config k1 --steps 20 --warmup 5 \
   --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor > $OUT/k1.json 2> $OUT/k1.err || exit $?
python3 tools/timeline.py $OUT/k1/run_kernel_trace.csv k_an_entries -2 > $OUT/k1_timeline.txt || exit $?
timeout -k 10 300 python bench.py --config k3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor > $OUT/k3.json 2> $OUT/k3.err || exit $?
