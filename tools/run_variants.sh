#!/bin/bash
# On the box: bench every build_var/libias_<name>.so (NAMES="a b c"), and with
# PROFILE=1 a serial rocprofv3 kernel-stats pass of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-var}
mkdir -p $OUT
for name in $NAMES; do
  IAS_LIB=$PWD/build_var/libias_$name.so timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 \
     --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-} > $OUT/bench_$name.json 2> $OUT/bench_$name.err || exit $?
  if [ -n "$PROFILE" ]; then
    IAS_SERIAL=1 IAS_LIB=$PWD/build_var/libias_$name.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
       -d $OUT/prof_$name -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
       --no-host-e2e ${BENCH_ARGS:-} > $OUT/prof_$name.log 2>&1 || exit $?
  fi
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/bench_$name.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'],d['roofline']['ms_per_launch'])")" >> $OUT/summary.txt
done
cat $OUT/summary.txt
