#!/bin/bash
# Round-end measurement set, in two parts (PART=a|b, one gpurun call each).
#  a: GPU suite, smoke, the K3' bench line (CPU baselines, one-shot and host
#     end-to-end), its rocprofv3 kernel stats, PMC passes of the same command.
#  b: K3 (full ILP64 MKL baseline), K2, K1 CSR + DIA, K1w DIA, the whole K4 on
#     one GPU, K3' in sorted order, the K4 eight-rank rehearsal on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
B="python bench.py"
if [ "${PART:-a}" = a ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
  timeout -k 10 500 $B > $OUT/bench_k3p.json 2> $OUT/bench_k3p.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-e2e --no-one-shot --no-weak-anchor > $OUT/bench_k3p_rocprof.json 2> $OUT/bench_k3p_rocprof.err || exit $?
  for c in FETCH_SIZE WRITE_SIZE "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$n -o p -- \
       python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor --no-weak-anchor > $OUT/pmc_$n.log 2>&1 || exit $?
  done
  python3 tools/pmc_kernels.py $OUT "k_num2(<|$)|k_sym|k_short|k_part|k_fixup|k_expand" > $OUT/pmc_summary.txt
  python3 tools/timeline.py $OUT/prof/run_kernel_trace.csv k_an_entries -2 > $OUT/timeline_k3p.txt
  IAS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor --no-weak-anchor > $OUT/serial.log 2>&1 || exit $?
  python3 tools/kstats.py $OUT/serial/run_kernel_stats.csv 7 > $OUT/serial_kstats_k3p.txt
else
  timeout -k 10 600 $B --config k3 --no-host-e2e --cpu-full > $OUT/bench_k3.json 2> $OUT/bench_k3.err || exit $?
  timeout -k 10 300 $B --config k2 --no-host-e2e > $OUT/bench_k2.json 2> $OUT/bench_k2.err || exit $?
  timeout -k 10 300 $B --config k1 --no-host-e2e > $OUT/bench_k1.json 2> $OUT/bench_k1.err || exit $?
  timeout -k 10 300 $B --config k1 --format dia --steps 200 --warmup 20 > $OUT/bench_k1_dia.json 2> $OUT/bench_k1_dia.err || exit $?
  timeout -k 10 300 $B --config k1w --format dia --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_k1w_dia.json 2> $OUT/bench_k1w_dia.err || exit $?
  timeout -k 10 300 $B --order sorted --steps 10 --warmup 2 --no-cpu-baseline --no-host-e2e --no-one-shot > $OUT/bench_k3p_sorted.json 2> $OUT/bench_k3p_sorted.err || exit $?
  timeout -k 10 900 $B --config k4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot > $OUT/bench_k4_1gpu.json 2> $OUT/bench_k4_1gpu.err || exit $?
  timeout -k 10 600 $B --gpus 8 --as-rank all --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e > $OUT/k4_as_rank_all.jsonl 2> $OUT/k4_as_rank_all.err || exit $?
fi
for f in $OUT/bench_*.json; do python3 -c "
import json,sys
d=json.load(open('$f')); r=d.get('roofline',{}); cb=d.get('cpu_baseline') or {}
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d.get('phases_ms_rank0'), r.get('frac'), cb.get('value'))"; done
