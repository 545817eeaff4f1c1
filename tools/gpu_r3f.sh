#!/bin/bash
# k_num2 cache-policy variants: serial kernel stats + FETCH/WRITE.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3f}
mkdir -p $OUT
V=${V:-base sc1nt sc01nt ldnt}
TAG=${TAG:-r3f}/var NAMES="$V" PROFILE=1 STEPS=10 bash tools/run_variants.sh || exit $?
for name in $V; do
  python3 tools/kstats.py $OUT/var/prof_$name/run_kernel_stats.csv 7 | grep -E "k_num2" | sed "s/^/$name /"
done
for name in $V; do
  for cnt in FETCH_SIZE WRITE_SIZE; do
    IAS_LIB=$PWD/build_var/libias_$name.so timeout -s KILL 120 rocprofv3 --pmc $cnt --kernel-trace --output-format csv \
      -d $OUT/pmc_$name/pmc_$(echo $cnt | cut -c1-5) -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-e2e \
      > $OUT/pmc_$name.log 2>&1 || exit $?
  done
  python3 tools/pmc_kernels.py $OUT/pmc_$name 'k_num2$' | sed "s/^/$name /"
done
