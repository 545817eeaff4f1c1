#!/bin/bash
# Parity of variant V (build_var/libias_$V.so: K3' per-row nnz vs the oracle,
# then the GPU parity suites on the in-tree library), then a same-box A/B of
# NAMES with V's serial kernel stats.   usage: V=name NAMES="base name" bash tools/gpu_symab.sh
set -o pipefail
V=${V:?variant}
mkdir -p gpurun_out/$V
IAS_LIB=$PWD/build_var/libias_$V.so timeout -k 10 200 python tools/row_nnz_diff.py > gpurun_out/$V/rowdiff.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fullsize.py tests/test_gpu_parity.py tests/test_gpu_branches.py > gpurun_out/$V/pytest.log 2>&1 &&
NAMES="${NAMES:-base $V}" REPS=${REPS:-3} TAG=$V SERIAL_LIB=$V bash tools/gpu_ab.sh
