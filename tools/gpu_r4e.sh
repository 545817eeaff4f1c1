#!/bin/bash
# nnz consistency of variants, GPU suite on the in-tree library, K3' A/B,
# sorted and K3 lines, a serial K3 kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4e}
mkdir -p $OUT
for name in $CHECK_NAMES; do
  IAS_LIB=$PWD/build_var/libias_$name.so timeout -k 10 120 python tools/nnz_check.py k3p >> $OUT/nnz_check.txt 2>&1
  rc=$?; [ $rc -gt 1 ] && { cat $OUT/nnz_check.txt; exit $rc; }
done
cat $OUT/nnz_check.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
[ $rc -ne 0 ] && exit $rc
TAG=${TAG:-r4e} bash tools/gpu_ab.sh || exit $?
timeout -k 10 300 python bench.py --order sorted --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e --no-one-shot > $OUT/sorted.json 2> $OUT/sorted.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/sorted.json'));print('sorted',d['value'],d['ms_per_step'],d['phases_ms_rank0'])"
timeout -k 10 300 python bench.py --config k3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e --no-one-shot > $OUT/k3.json 2> $OUT/k3.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/k3.json'));print('k3',d['value'],d['ms_per_step'],d['phases_ms_rank0'])"
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial_k3 -o run --output-format csv -- \
   python bench.py --config k3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot > $OUT/serial_k3.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial_k3/run_kernel_stats.csv 4 > $OUT/serial_k3_kstats.txt
head -25 $OUT/serial_k3_kstats.txt
