#!/bin/bash
# On the box: bench.py under each environment of EVARS (entries separated by
# ';', each a space-separated list of VAR=value, "-" = none), one JSON line per
# variant, then a summary.  BENCH_ARGS is passed to every run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-envvar}
mkdir -p $OUT
IFS=';' read -ra VS <<< "$EVARS"
i=0
for v in "${VS[@]}"; do
  i=$((i + 1))
  envs=""; [ "$v" != "-" ] && envs="$v"
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-host-e2e \
      ${BENCH_ARGS:-} > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
  echo "[$v] $(python3 -c "import json;d=json.load(open('$OUT/bench_$i.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'])")" | tee -a $OUT/summary.txt
done
