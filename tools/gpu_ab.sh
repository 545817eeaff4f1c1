#!/bin/bash
# Same-box A/B of build_var/libias_<name>.so variants (NAMES), alternating
# REPS times, K3' unless BENCH_ARGS says otherwise; optional extras:
#   PMC_LIB=name     LDS / traffic counter passes of that variant
#   SERIAL_LIB=name  IAS_SERIAL=1 rocprofv3 kernel stats of that variant
#   TRACE_LIB=name   concurrent rocprofv3 kernel trace (timeline) of that variant
#   HIPTRACE=1       HIP API trace of the driver's bench command (one-shot leg)
# A name may be lib+VAR=value[+VAR2=value2...]: that library with those environment variables.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
S=$OUT/ab_summary.txt
for rep in $(seq 1 ${REPS:-2}); do
  for name in $NAMES; do
    # name = lib or lib+VAR=value (an environment variant of a library)
    lib=${name%%+*}; envv=; [ "$lib" != "$name" ] && envv=${name#*+}
    env ${envv//+/ } IAS_LIB=$PWD/build_var/libias_$lib.so timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
       --no-host-e2e --no-one-shot --no-anchor --no-weak-anchor $BENCH_ARGS > $OUT/ab_${name}_$rep.json 2> $OUT/ab_${name}_$rep.err || exit $?
    echo "$name $rep $(python3 -c "import json;d=json.load(open('$OUT/ab_${name}_$rep.json'));print(d['value'],d['ms_per_step'],d.get('phases_ms_rank0'),d.get('roofline',{}).get('ms_per_launch'))")" >> $S
  done
done
cat $S
if [ -n "$SERIAL_LIB" ]; then
  IAS_SERIAL=1 IAS_LIB=$PWD/build_var/libias_$SERIAL_LIB.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
     -d $OUT/serial -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
     --no-host-e2e --no-one-shot --no-anchor --no-weak-anchor $BENCH_ARGS > $OUT/serial.log 2>&1 || exit $?
  python3 tools/kstats.py $OUT/serial/run_kernel_stats.csv 7 > $OUT/serial_kstats.txt
fi
if [ -n "$TRACE_LIB" ]; then
  IAS_LIB=$PWD/build_var/libias_$TRACE_LIB.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
     -d $OUT/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
     --no-host-e2e --no-one-shot --no-anchor --no-weak-anchor $BENCH_ARGS > $OUT/trace.log 2>&1 || exit $?
  python3 tools/timeline.py $OUT/trace/run_kernel_trace.csv k_an_entries -2 > $OUT/timeline.txt
fi
if [ -n "$PMC_LIB" ]; then
  for c in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $c | cut -d' ' -f1)
    IAS_LIB=$PWD/build_var/libias_$PMC_LIB.so timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$n -o p -- \
       python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor --no-weak-anchor $BENCH_ARGS > $OUT/pmc_$n.log 2>&1 || exit $?
  done
  python3 tools/pmc_kernels.py $OUT "k_num2(<|$)|k_sym|k_short|k_part|k_fixup" > $OUT/pmc_summary.txt
fi
if [ -n "$HIPTRACE" ]; then
  timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/hip -o run -- \
      python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e > $OUT/hip_bench.json 2> $OUT/hip_bench.err || exit $?
  python3 tools/hip_api_summary.py $OUT/hip/run_hip_api_trace.csv 2000 > $OUT/hip_api_summary.txt
  python3 -c "import json;d=json.load(open('$OUT/hip_bench.json'));print(d['ms_per_step'],d.get('one_shot'))"
fi
