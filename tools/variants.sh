#!/bin/bash
# Build libias variants from -D flag sets (VARIANTS="name:flags;name:flags")
# into build_tim/ and run the bench against each (IAS_LIB), one JSON line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-var}
mkdir -p $OUT build_tim
make -C ia-spgemm_amd -j16 > /dev/null || exit 1
O=ia-spgemm_amd/build
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wno-unused-value \
     -Iinclude -Iia-spgemm_amd/csrc $flags -c ia-spgemm_amd/csrc/spgemm.hip -o build_tim/spgemm_$name.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_tim/libias_$name.so build_tim/spgemm_$name.o \
     $O/ias_api.o $O/dia.o $O/mtx_io.o $O/gen.o $O/convert.o $O/mkl_baseline.o \
     -L/usr/lib/gcc/x86_64-linux-gnu/11 -lgomp -ldl || exit 1
done
for v in "${VS[@]}"; do
  name=${v%%:*}
  IAS_LIB=$PWD/build_tim/libias_$name.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
     --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_$name.json 2> $OUT/bench_$name.err || exit $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/bench_$name.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'],d['roofline']['ms_per_launch'])")" >> $OUT/summary.txt
done
cat $OUT/summary.txt
