# K4 (whole, one GPU): per-kernel serial stats of one step — where K4's
# symbolic time goes (tools/kstats.py summary)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-k4prof}
mkdir -p $OUT
IAS_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/serial -o run --output-format csv -- \
  python bench.py --config k4 --steps 2 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor \
  > $OUT/serial.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/serial/run_kernel_stats.csv 3 > $OUT/serial_kstats.txt
head -30 $OUT/serial_kstats.txt
