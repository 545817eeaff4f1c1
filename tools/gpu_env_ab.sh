#!/bin/bash
# Same-box A/B of environment settings on the in-tree library: SUITE=1 runs
# the GPU suite first; then for each config in CFGS (default k3p) and each
# setting in ENVS (space-separated VAR=value, "-" for none), REPS alternating
# bench lines.  usage: TAG=x ENVS="IAS_X=0 IAS_X=1" bash tools/gpu_env_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-envab}
mkdir -p $OUT
if [ -n "$SUITE" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
B="python bench.py --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor --steps ${STEPS:-10} --warmup 3"
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:-k3p}; do
    for e in $ENVS; do
      n=$(echo $e | tr '=' '_')
      if [ "$e" = "-" ]; then E=""; else E="$e"; fi
      env $E timeout -k 10 300 $B --config $cfg > $OUT/${cfg}_${n}_$rep.json 2> $OUT/${cfg}_${n}_$rep.err || exit $?
      echo "$cfg $e $rep $(python3 -c "import json;d=json.load(open('$OUT/${cfg}_${n}_$rep.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'])")"
    done
  done
done
