#!/bin/bash
# GPU suite on the in-tree library, then the sorted-order K3' line of each
# variant (SORT_NAMES, alternating twice) and a serial kernel profile of the last.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sort}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --no-cpu-baseline --no-host-e2e --no-one-shot --order sorted --steps 5 --warmup 2"
for rep in 1 2; do
  for name in $SORT_NAMES; do
    IAS_LIB=$PWD/build_var/libias_$name.so timeout -k 10 300 $B > $OUT/sorted_${name}_$rep.json 2> $OUT/sorted_${name}_$rep.err || exit $?
    echo "sorted $name $rep $(python3 -c "import json;d=json.load(open('$OUT/sorted_${name}_$rep.json'));print(d['value'],d['ms_per_step'])")"
  done
done
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial_sorted -o run --output-format csv -- \
   $B > $OUT/serial_sorted.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial_sorted/run_kernel_stats.csv 7 | grep -E "sort|num2" > $OUT/serial_sorted_kstats.txt
cat $OUT/serial_sorted_kstats.txt
