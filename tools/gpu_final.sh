#!/bin/bash
# Round-end measurement set: GPU suite, smoke, bench lines of every config
# (K3' default with the CPU baselines, K3, K2, K1 CSR + DIA, K1w DIA), the
# K4 eight-rank rehearsal, and the rocprofv3 stats of the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $OUT/bench_k3p.json 2> $OUT/bench_k3p.err || exit $?
timeout -k 10 400 python bench.py --config k3 --no-host-e2e > $OUT/bench_k3.json 2> $OUT/bench_k3.err || exit $?
timeout -k 10 300 python bench.py --config k2 --no-host-e2e > $OUT/bench_k2.json 2> $OUT/bench_k2.err || exit $?
timeout -k 10 300 python bench.py --config k1 --no-host-e2e > $OUT/bench_k1.json 2> $OUT/bench_k1.err || exit $?
timeout -k 10 300 python bench.py --config k1 --format dia --steps 20 --warmup 5 > $OUT/bench_k1_dia.json 2> $OUT/bench_k1_dia.err || exit $?
timeout -k 10 300 python bench.py --config k1w --format dia --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_k1w_dia.json 2> $OUT/bench_k1w_dia.err || exit $?
timeout -k 10 500 python bench.py --gpus 8 --as-rank all --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e > $OUT/k4_as_rank_all.jsonl 2> $OUT/k4_as_rank_all.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-e2e > $OUT/bench_k3p_rocprof.json 2> $OUT/bench_k3p_rocprof.err || exit $?
