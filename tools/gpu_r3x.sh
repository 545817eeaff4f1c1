#!/bin/bash
# A/B pre vs fuse on K3 and K3' (serial kernel stats), then the full-size + parity suites
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in k3 k3p; do
  TAG=r3x/$c NAMES="pre fuse" PROFILE=1 STEPS=6 BENCH_ARGS="--config $c --no-anchor --no-one-shot" bash tools/run_variants.sh || exit $?
  for n in pre fuse; do python3 tools/kstats.py gpurun_out/r3x/$c/prof_$n/run_kernel_stats.csv 8 | grep -E "part|expand|bitmap_prefix|dup_place" | sed "s/^/$c $n /"; done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3x/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r3x/pytest_gpu.log
exit $rc
