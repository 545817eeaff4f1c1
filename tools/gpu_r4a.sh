#!/bin/bash
# Round-4 first probe: the K3' bench line of the starting tree and a HIP API
# trace of the one-shot calls (where the first call's time goes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4a}
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-e2e > $OUT/bench_k3p.json 2> $OUT/bench_k3p.err || exit $?
timeout -k 10 300 python tools/one_shot_probe.py > $OUT/one_shot.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/hip -o run -- \
    python tools/one_shot_probe.py > $OUT/one_shot_traced.log 2>&1 || exit $?
f=$(ls $OUT/hip/*/run_hip_api_trace.csv 2>/dev/null | head -1)
[ -z "$f" ] && f=$(find $OUT/hip -name '*hip_api_trace.csv' | head -1)
python3 tools/hip_api_summary.py "$f" 2000 > $OUT/hip_api_summary.txt
cat $OUT/one_shot.log
python3 -c "import json;d=json.load(open('$OUT/bench_k3p.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'],d['roofline']['frac'],d.get('one_shot'))"
# A/B of build_var variants (NAMES), alternating twice
if [ -n "$NAMES" ]; then
  for rep in 1 2; do
    for name in $NAMES; do
      IAS_LIB=$PWD/build_var/libias_$name.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
         --no-host-e2e --no-one-shot > $OUT/ab_${name}_$rep.json 2> $OUT/ab_${name}_$rep.err || exit $?
      echo "$name $rep $(python3 -c "import json;d=json.load(open('$OUT/ab_${name}_$rep.json'));print(d['value'],d['ms_per_step'],d['phases_ms_rank0'],d['roofline'].get('ms_per_launch'))")" >> $OUT/ab_summary.txt
    done
  done
  cat $OUT/ab_summary.txt
fi
if [ -n "$PMC_LIB" ]; then
  for c in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
    n=$(echo $c | cut -d' ' -f1)
    IAS_LIB=$PWD/build_var/libias_$PMC_LIB.so timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$n -o p -- \
       python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor > $OUT/pmc_$n.log 2>&1 || exit $?
  done
  python3 tools/pmc_kernels.py $OUT "k_sym|k_short|k_part" > $OUT/pmc_summary.txt
fi
