#!/bin/bash
# Build libias variants HERE (CPU container; the .so files travel with the
# tree): VARIANTS="name:flags;name:flags" -> build_var/libias_<name>.so.
# Run them on the box with tools/run_variants.sh.
set -e
cd "$(dirname "$0")/.."
make -C ia-spgemm_amd -j8 > /dev/null
mkdir -p build_var
O=ia-spgemm_amd/build
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wno-unused-value \
     -Iinclude -Iia-spgemm_amd/csrc $flags -c ia-spgemm_amd/csrc/spgemm.hip -o build_var/spgemm_$name.o &
done
wait
for v in "${VS[@]}"; do
  name=${v%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_var/libias_$name.so build_var/spgemm_$name.o \
     $O/ias_api.o $O/multi.o $O/dia.o $O/convert_dev.o $O/mtx_io.o $O/gen.o $O/convert.o $O/mkl_baseline.o $O/matnet.o \
     -L/usr/lib/gcc/x86_64-linux-gnu/11 -lgomp -ldl
  echo "built build_var/libias_$name.so"
done
