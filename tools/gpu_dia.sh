#!/bin/bash
# DIA: parity tests, then K1 / wide-band lines through the DIA kernel, VALU
# tile kernel vs MFMA (IAS_DIA_MFMA=1), plus a serial kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dia}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "dia" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_dia.log 2>&1 || exit $?
for c in k1 k1w; do
  timeout -k 10 300 python bench.py --config $c --format dia --steps 20 --warmup 5 > $OUT/bench_${c}_dia.json 2> $OUT/bench_${c}_dia.err || exit $?
  IAS_DIA_MFMA=1 timeout -k 10 300 python bench.py --config $c --format dia --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${c}_dia_mfma.json 2> $OUT/bench_${c}_dia_mfma.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_k1_dia -o run --output-format csv -- python bench.py --config k1 --format dia --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_k1_dia.log 2>&1 || exit $?
