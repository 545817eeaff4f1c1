#!/bin/bash
# Device transpose + conversions parity, then spgemm-gpu --aat on the inputs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-f2}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "device_transpose or device_conversions or csr_inputs_a_times_at" > $OUT/pytest_t.log 2>&1 || { tail -40 $OUT/pytest_t.log; exit 1; }
tail -1 $OUT/pytest_t.log
for m in dia.mtx b1_ss.mtx LFAT5.mtx; do
  timeout -k 10 120 ia-spgemm_amd/bin/spgemm-gpu tests/golden/inputs/$m --aat --rand10 --seed 1 > $OUT/cli_gpu_$m.txt 2>&1 || { cat $OUT/cli_gpu_$m.txt; exit 1; }
done
grep -H "verified_sum" $OUT/cli_gpu_*.txt
