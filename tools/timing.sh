#!/bin/bash
# Per-phase timing of the row kernels: builds libias with -DIAS_TIMING=1 into
# build_tim/ and runs tools/timing_run.py against it (K3' by default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tim}
mkdir -p $OUT build_tim
make -C ia-spgemm_amd -j16 > /dev/null || exit 1
O=ia-spgemm_amd/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wno-unused-value \
   -Iinclude -Iia-spgemm_amd/csrc -DIAS_TIMING=1 -c ia-spgemm_amd/csrc/spgemm.hip -o build_tim/spgemm.o || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_tim/libias.so build_tim/spgemm.o \
   $O/ias_api.o $O/multi.o $O/dia.o $O/convert_dev.o $O/mtx_io.o $O/gen.o $O/convert.o $O/mkl_baseline.o $O/matnet.o \
   -L/usr/lib/gcc/x86_64-linux-gnu/11 -lgomp -ldl || exit 1
IAS_SERIAL=1 IAS_LIB=$PWD/build_tim/libias.so timeout -k 10 300 python tools/timing_run.py ${TIMING_ARGS:-} > $OUT/timing.txt 2>&1
