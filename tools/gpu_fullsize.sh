#!/bin/bash
# Full-size parity (K1, K2, K3', K3 against the oracle's digests) and the
# K3 / K3' bench lines.  Each GPU step has its own time limit; && chains them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fullsize}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_fullsize.log 2>&1 &&
timeout -k 10 600 python bench.py --config k3 --steps 5 --warmup 2 ${BENCH_ARGS:-} > $OUT/bench_k3.json 2> $OUT/bench_k3.err &&
timeout -k 10 600 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > $OUT/bench_k3p.json 2> $OUT/bench_k3p.err
