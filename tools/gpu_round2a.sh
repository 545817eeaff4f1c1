#!/bin/bash
# Full GPU suite, K3' bench line, and the K4 8-rank rehearsal (--as-rank all).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2a}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-host-e2e > $OUT/bench_k3p.json 2> $OUT/bench_k3p.err || exit $?
timeout -k 10 500 python bench.py --gpus 8 --as-rank all --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e \
    > $OUT/k4_as_rank_all.jsonl 2> $OUT/k4_as_rank_all.err || exit $?
