#!/bin/bash
# One GPU-box session: build check, GPU tests, smoke, CLIs, bench, rocprof.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure (fault, abort, timeout) ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
bash tools/probe_box.sh > $OUT/box.txt 2>&1 || true
make -C ia-spgemm_amd -j16 > $OUT/build.log 2>&1 && make -C oracle >> $OUT/build.log 2>&1 &&
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:--x} > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 120 ./ia-spgemm_amd/bin/spgemm-cpu tests/golden/inputs/dia.mtx > $OUT/cli_cpu_dia.txt 2>&1 &&
timeout -k 10 120 ./ia-spgemm_amd/bin/spgemm-gpu tests/golden/inputs/dia.mtx --aat --rand10 --seed 1 > $OUT/cli_gpu_dia.txt 2>&1 &&
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err &&
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof.log 2>&1 &&
  IAS_SERIAL=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_serial.log 2>&1
fi
