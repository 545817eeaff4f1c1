#!/bin/bash
# GPU suite on the in-tree library, sorted-order A/B (SORT_NAMES), K1 DIA,
# then the K3' A/B + profiles (gpu_ab.sh) and a K3 A/B (K3_NAMES).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
for name in $SORT_NAMES; do
  IAS_LIB=$PWD/build_var/libias_$name.so timeout -k 10 300 python bench.py --order sorted --steps 5 --warmup 2 --no-cpu-baseline \
     --no-host-e2e --no-one-shot > $OUT/sorted_$name.json 2> $OUT/sorted_$name.err || exit $?
  echo "sorted $name $(python3 -c "import json;d=json.load(open('$OUT/sorted_$name.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'])")"
done
timeout -k 10 200 python bench.py --config k1 --format dia --steps 20 --warmup 5 --no-cpu-baseline > $OUT/k1dia.json 2> $OUT/k1dia.err || exit $?
python3 -c "import json;d=json.load(open('$OUT/k1dia.json'));print('k1 dia', d['ms_per_step'], d['roofline']['ms_per_launch'], d['alloc_call'])"
TAG=${TAG:-r4d} bash tools/gpu_ab.sh || exit $?
for name in $K3_NAMES; do
  IAS_LIB=$PWD/build_var/libias_$name.so timeout -k 10 300 python bench.py --config k3 --steps 5 --warmup 2 --no-cpu-baseline \
     --no-host-e2e --no-one-shot > $OUT/k3_$name.json 2> $OUT/k3_$name.err || exit $?
  echo "k3 $name $(python3 -c "import json;d=json.load(open('$OUT/k3_$name.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'])")"
done
