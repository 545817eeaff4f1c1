#!/bin/bash
# Builds tools/rocsparse_cmp (rocSPARSE csrgemm beside the engine) against the
# in-tree libias.so.  Run on the GPU box: tools/bin/rocsparse_cmp [scale] [steps]
set -e
cd "$(dirname "$0")"
mkdir -p bin
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -I../include rocsparse_cmp.cpp \
  -o bin/rocsparse_cmp -L../ia-spgemm_amd -lias -lrocsparse \
  -Wl,-rpath,'$ORIGIN/../../ia-spgemm_amd' -Wl,-rpath,/opt/rocm/lib
