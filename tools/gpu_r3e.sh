#!/bin/bash
# k_num2 ablations (stores off / gathers off / plain stores) with serial
# kernel stats, FETCH/WRITE of k_num2 per variant, then the symbolic PMC pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3e}
mkdir -p $OUT
TAG=${TAG:-r3e}/var NAMES="base nost nogat plain" PROFILE=1 STEPS=10 bash tools/run_variants.sh || exit $?
for name in base nost nogat plain; do
  python3 tools/kstats.py $OUT/var/prof_$name/run_kernel_stats.csv 7 | grep -E "k_num2|k_fixup_large" | sed "s/^/$name /"
done
for name in base nost plain; do
  for cnt in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    IAS_LIB=$PWD/build_var/libias_$name.so timeout -s KILL 120 rocprofv3 --pmc $cnt --kernel-trace --output-format csv \
      -d $OUT/pmc_$name/pmc_$(echo $cnt | cut -c1-5) -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-e2e \
      > $OUT/pmc_$name.log 2>&1 || exit $?
  done
  python3 tools/pmc_kernels.py $OUT/pmc_$name 'k_num2$' | sed "s/^/$name /"
done
TAG=${TAG:-r3e}/sym bash tools/gpu_r3d.sh
