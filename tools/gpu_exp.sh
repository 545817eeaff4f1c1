#!/bin/bash
# Same-box experiments: variants (NAMES), env variants (ENVS="NAME:VAR=v ..."),
# a serial kernel profile of the base library and extra bench configs (EXTRA).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-exp}
mkdir -p $OUT
S=$OUT/summary.txt
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/bench_$name.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'],d['roofline'].get('ms_per_launch'))")" >> $S
}
for name in $NAMES; do
  run $name IAS_LIB=$PWD/build_var/libias_$name.so python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor $BENCH_ARGS || exit $?
done
for e in $ENVS; do
  run ${e%%:*} ${e#*:} IAS_LIB=$PWD/build_var/libias_base.so python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor $BENCH_ARGS || exit $?
done
for c in $SERIAL_CFGS; do
  IAS_SERIAL=1 IAS_LIB=$PWD/build_var/libias_${SERIAL_PROF}.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
     -d $OUT/serial_$c -o run --output-format csv -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline \
     --no-host-e2e --no-one-shot --no-anchor > $OUT/serial_$c.log 2>&1 || exit $?
  python3 tools/kstats.py $OUT/serial_$c/run_kernel_stats.csv 4 > $OUT/serial_${c}_kstats.txt
done
if [ -n "$SERIAL_PROF" ]; then
  IAS_SERIAL=1 IAS_LIB=$PWD/build_var/libias_${SERIAL_PROF}.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
     -d $OUT/serial -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
     --no-host-e2e --no-one-shot --no-anchor $BENCH_ARGS > $OUT/serial.log 2>&1 || exit $?
  python3 tools/kstats.py $OUT/serial/run_kernel_stats.csv 7 > $OUT/serial_kstats.txt
fi
for c in $EXTRA; do
  run ${c} IAS_LIB=$PWD/build_var/libias_${EXTRA_LIB:-base}.so python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor || exit $?
done
cat $S
