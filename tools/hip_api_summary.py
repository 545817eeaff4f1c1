#!/usr/bin/env python3
"""Per-call HIP API time from a rocprofv3 --hip-trace CSV, split at the
one-shot probe's calls (the windows between big gaps are not needed: every
API call is listed with its start relative to the first one, and the totals
per function name are printed at the end).
usage: hip_api_summary.py run_hip_api_trace.csv [min_us]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 500.0
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    tot = defaultdict(lambda: [0, 0.0])
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[r["Function"]][0] += 1
        tot[r["Function"]][1] += d
        if d >= min_us:
            print(f"{(int(r['Start_Timestamp']) - t0) / 1e6:10.3f} ms  {d / 1e3:9.3f} ms  {r['Function']}")
    print("--- totals")
    for k, (n, d) in sorted(tot.items(), key=lambda x: -x[1][1])[:30]:
        print(f"{k:40s} {n:7d} {d / 1e3:10.3f} ms")


if __name__ == "__main__":
    main()
