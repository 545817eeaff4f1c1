#!/bin/bash
# Build variants ($VARIANTS = "name:flags;..."), then per variant: the GPU
# parity subset, K3' bench and a serial kernel profile (top kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-varprof}
mkdir -p $OUT build_tim
make -C ia-spgemm_amd -j16 > /dev/null || exit 1
O=ia-spgemm_amd/build
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wno-unused-value \
     -Iinclude -Iia-spgemm_amd/csrc $flags -c ia-spgemm_amd/csrc/spgemm.hip -o build_tim/spgemm_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_tim/libias_$name.so build_tim/spgemm_$name.o \
     $O/ias_api.o $O/dia.o $O/convert_dev.o $O/mtx_io.o $O/gen.o $O/convert.o $O/mkl_baseline.o $O/matnet.o \
     -L/usr/lib/gcc/x86_64-linux-gnu/11 -lgomp -ldl || exit 1
done
for v in "${VS[@]}"; do
  name=${v%%:*}
  export IAS_LIB=$PWD/build_tim/libias_$name.so
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_$name.log 2>&1 || { tail -20 $OUT/pytest_$name.log; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-e2e --steps 10 --warmup 3 > $OUT/k3p_$name.json 2>> $OUT/err.log || exit 1
  IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e > $OUT/prof_$name.log 2>&1 || exit 1
  python3 -c "
import json; a=json.load(open('$OUT/k3p_$name.json')); print('$name', '$(tail -1 $OUT/pytest_$name.log | cut -c1-30)', a['value'], a['ms_per_step'], a['phases_ms_rank0'])"
  python3 tools/kstats.py $OUT/prof_$name/run_kernel_stats.csv 7 | grep -E "${KGREP:-fixup}"
done
