#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of k_num2 per library variant (NAMES), K3'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fetch}
mkdir -p $OUT
for name in $NAMES; do
  for c in FETCH_SIZE WRITE_SIZE; do
    IAS_LIB=$PWD/build_var/libias_$name.so timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${name}_$c -o p -- \
       python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-e2e --no-one-shot --no-anchor > $OUT/pmc_${name}_$c.log 2>&1 || exit $?
  done
  python3 - $OUT $name <<'PY'
import csv, glob, sys, collections
out, name = sys.argv[1], sys.argv[2]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{out}/pmc_{name}_{c}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_num2(" in r["Kernel_Name"] or r["Kernel_Name"].startswith("ias::dev::k_num2"):
            acc[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    vals = [sum(v) for v in acc.values()]
    print(name, c, "launches", len(vals), "KiB per launch mean %.4g" % (sum(vals) / max(len(vals), 1)))
PY
done
