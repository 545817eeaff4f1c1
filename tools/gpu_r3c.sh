#!/bin/bash
# K3' bench with / without sym3 and the per-phase timing build of the row kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3c}
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-e2e ${BENCH_ARGS:-}"
timeout -k 10 300 $B > $OUT/bench.json 2> $OUT/bench.err &&
IAS_SYM3=0 timeout -k 10 300 $B > $OUT/bench_nosym3.json 2> $OUT/bench_nosym3.err
rc=$?
for f in bench bench_nosym3; do
  python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['ms_per_launch'])"
done
[ $rc -eq 0 ] && TAG=${TAG:-r3c}/tim bash tools/timing.sh; rc=$?
cat $OUT/tim/timing.txt
exit $rc
