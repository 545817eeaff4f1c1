#!/bin/bash
# f3 on the box: device conversion parity, full GPU suite, spgemm-cpu with
# device-side CSRtoX (trans_time) on the reference inputs and a 1M-row band.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-f3}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k device_conversions > $OUT/pytest_conv.log 2>&1 || { tail -40 $OUT/pytest_conv.log; exit 1; }
tail -1 $OUT/pytest_conv.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for m in dia.mtx b1_ss.mtx; do
  timeout -k 10 120 ia-spgemm_amd/bin/spgemm-cpu tests/golden/inputs/$m > $OUT/cli_cpu_$m.txt 2>&1 || { cat $OUT/cli_cpu_$m.txt; exit 1; }
done
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'ia-spgemm_amd'); import ias
ias.mtx_write('/tmp/band1m.mtx', ias.gen_band(1 << 20, 5, seed=3))" &&
timeout -k 10 300 ia-spgemm_amd/bin/spgemm-cpu /tmp/band1m.mtx > $OUT/cli_cpu_band1m.txt 2>&1 || { tail -30 $OUT/cli_cpu_band1m.txt; exit 1; }
grep -A3 "^Algorithm" $OUT/cli_cpu_band1m.txt
