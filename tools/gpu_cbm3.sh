#!/bin/bash
# k_sym_cbm over the expansion: long-row parity cases, nnz(C) of K3' / K3, then
# K3' and K3 with the hash partitions (IAS_SYM_CBM=0), the column bitmap for
# rows beyond 16,384 products, and for rows from IAS_SYM_CBM_MIN = MINS;
# build_var variants LIBS; serial K3 kernel stats of the default.  SUITE=1:
# the whole GPU suite after the nnz checks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cbm3}
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -m gpu -k "duplicate_tiers or long_row or wide_row or heavy" \
   > $OUT/pytest_long.log 2>&1
rc=$?; tail -2 $OUT/pytest_long.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/nnz_check.py k3p k3 || exit $?
for m in ${MINS-8193 4097}; do
  IAS_SYM_CBM_MIN=$m timeout -k 10 300 python tools/nnz_check.py k3p k3 || exit $?
done
if [ -n "$SUITE" ]; then
  timeout -k 10 600 $T tests -m gpu > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
B="python bench.py --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor --steps 10 --warmup 3"
for rep in 1 2; do
  for cfg in k3p k3; do
    for v in off on ${MINS-8193 4097} $LIBS; do
      case $v in off) E="IAS_SYM_CBM=0";; on) E="IAS_SYM_CBM=1";; [0-9]*) E="IAS_SYM_CBM_MIN=$v";;
        *) E="IAS_LIB=$PWD/build_var/libias_$v.so";; esac
      env $E timeout -k 10 300 $B --config $cfg > $OUT/${cfg}_${v}_$rep.json 2> $OUT/${cfg}_${v}_$rep.err || exit $?
      echo "$cfg $v $rep $(python3 -c "import json;d=json.load(open('$OUT/${cfg}_${v}_$rep.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'])")"
    done
  done
done
IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial_k3 -o run --output-format csv -- \
   $B --config k3 --steps 3 --warmup 1 > $OUT/serial_k3.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial_k3/run_kernel_stats.csv 4 > $OUT/serial_k3_kstats.txt
head -16 $OUT/serial_k3_kstats.txt
