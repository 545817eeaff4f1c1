#!/usr/bin/env python3
"""Per-kernel mean of every collected counter (rocprofv3 --pmc CSVs under
<root>/pmc_*), for kernels whose name matches a regex.
usage: tools/pmc_kernels.py <root> [regex]"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "").replace("ias::dev::", "")
        if not pat.search(k):
            continue
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(vals.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-28s %14.4g" % (c, sum(v) / len(v)))
