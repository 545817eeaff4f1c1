set -o pipefail
mkdir -p gpurun_out/b2
IAS_SYM_BIG=2 IAS_LIB=$PWD/build_var/libias_big2.so timeout -k 10 200 python tools/row_nnz_diff.py > gpurun_out/b2/rowdiff_big2.txt 2>&1 &&
NAMES="ring2u big2 big2+IAS_SYM_BIG=2" REPS=3 TAG=b2k3p bash tools/gpu_ab.sh &&
NAMES="ring2u big2 big2+IAS_SYM_BIG=2" REPS=2 STEPS=5 TAG=b2k3 BENCH_ARGS="--config k3" bash tools/gpu_ab.sh &&
timeout -k 10 600 python bench.py --gpus 8 --as-rank all --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e > gpurun_out/b2/k4_as_rank_all.jsonl 2> gpurun_out/b2/k4_as_rank_all.err
