#!/bin/bash
# pipe (row blocks) vs one block on K2, K3 and the whole K4 on one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in k2 k3 k4; do
  st=20; [ $c = k4 ] && st=5
  TAG=r3k/$c STEPS=$st BENCH_ARGS="--config $c --no-anchor --no-one-shot" EVARS="-;IAS_PIPE_BLOCKS=1;IAS_PIPE_BLOCKS=2" \
     bash tools/env_variants.sh || exit $?
done
