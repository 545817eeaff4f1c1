#!/bin/bash
# GPU suite on the in-tree library, K3' A/B (NAMES), then profiles: sorted
# (serial kernel stats), K3 (line + serial kernel stats), K1 CSR timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
TAG=${TAG:-r4f} bash tools/gpu_ab.sh || exit $?
B="python bench.py --no-cpu-baseline --no-host-e2e --no-one-shot"
timeout -k 10 300 $B --order sorted --steps 5 --warmup 2 > $OUT/sorted.json 2> $OUT/sorted.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/sorted.json'));print('sorted',d['value'],d['ms_per_step'],d['phases_ms_rank0'])"
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial_sorted -o run --output-format csv -- \
   $B --order sorted --steps 3 --warmup 1 > $OUT/serial_sorted.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial_sorted/run_kernel_stats.csv 4 > $OUT/serial_sorted_kstats.txt
head -14 $OUT/serial_sorted_kstats.txt
timeout -k 10 300 $B --config k3 --steps 5 --warmup 2 > $OUT/k3.json 2> $OUT/k3.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/k3.json'));print('k3',d['value'],d['ms_per_step'],d['phases_ms_rank0'])"
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial_k3 -o run --output-format csv -- \
   $B --config k3 --steps 3 --warmup 1 > $OUT/serial_k3.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial_k3/run_kernel_stats.csv 4 > $OUT/serial_k3_kstats.txt
head -25 $OUT/serial_k3_kstats.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace_k1 -o run --output-format csv -- \
   $B --config k1 --steps 5 --warmup 2 > $OUT/trace_k1.log 2>&1 || exit $?
python3 tools/timeline.py $OUT/trace_k1/run_kernel_trace.csv k_an_entries -2 > $OUT/timeline_k1.txt
cat $OUT/timeline_k1.txt | tail -40
