#!/usr/bin/env python3
"""Short per-kernel table from a rocprofv3 --stats kernel_stats.csv.
usage: tools/kstats.py <kernel_stats.csv> [calls_per_step_divisor]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:30]:
    n = re.sub(r"ias::dev::", "", r["Name"])
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    print("%-48s %6s %10.1f us/call %9.3f ms/step %6.2f%%" % (
        n[:48], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6 / div,
        100 * float(r["TotalDurationNs"]) / tot))
