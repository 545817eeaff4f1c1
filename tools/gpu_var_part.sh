#!/bin/bash
# Partition-size variants: parity on the partitioned-row tests, K3' and the
# heaviest 8-GPU rank (scale 23, rank 0) per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-varpart}
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
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "long or tiers or collisions or wide or edges or rmat" > $OUT/pytest_$name.log 2>&1 || { tail -20 $OUT/pytest_$name.log; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/k3p_$name.json 2>> $OUT/err.log || exit 1
  timeout -k 10 300 python bench.py --gpus 8 --as-rank 0 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/r0_$name.json 2>> $OUT/err.log || exit 1
  python3 -c "
import json
a=json.load(open('$OUT/k3p_$name.json')); b=json.load(open('$OUT/r0_$name.json'))
print('$name', '$(tail -1 $OUT/pytest_$name.log | cut -c1-40)', 'k3p', a['value'], a['ms_per_step'], 'rank0', b['value'], b['ms_per_step'], b['phases_ms_rank0']['symbolic'])"
done
