#!/bin/bash
# Timing-only ablation builds of the hot kernels (-DIAS_ABLATE=<mask>, see
# spgemm_kernels.hpp): each variant's libias is linked into build_abl/, then
# the bench runs under rocprofv3 --kernel-trace --stats.  Outputs of ablated
# builds are WRONG by construction; only their kernel times are read.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abl}
mkdir -p $OUT build_abl
make -C ia-spgemm_amd -j16 > /dev/null || exit 1
O=ia-spgemm_amd/build
for m in ${MASKS:-0 1 2 4 8 16}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wno-unused-value \
     -Iinclude -Iia-spgemm_amd/csrc -DIAS_ABLATE=$m -c ia-spgemm_amd/csrc/spgemm.hip -o build_abl/spgemm_$m.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_abl/libias_$m.so build_abl/spgemm_$m.o \
     $O/ias_api.o $O/dia.o $O/mtx_io.o $O/gen.o $O/convert.o $O/mkl_baseline.o \
     -L/usr/lib/gcc/x86_64-linux-gnu/11 -lgomp -ldl || exit 1
done
for m in ${MASKS:-0 1 2 4 8 16}; do
  IAS_LIB=$PWD/build_abl/libias_$m.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/abl_$m -o p \
     --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
     > $OUT/abl_$m.log 2>&1
  rc=$?; echo "mask $m rc=$rc" >> $OUT/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
