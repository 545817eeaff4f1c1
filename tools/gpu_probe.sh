#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/fetch_probe.hip)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-probe}
mkdir -p $OUT
[ -x tools/fetch_probe ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/fetch_probe tools/fetch_probe.hip || exit 1
for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$n -o p -- tools/fetch_probe > $OUT/probe_$n.log 2>&1 || exit $?
done
cat $OUT/probe_FETCH_SIZE.log
python3 tools/pmc_kernels.py $OUT "." | tee $OUT/summary.txt
