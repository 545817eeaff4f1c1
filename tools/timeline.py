#!/usr/bin/env python3
"""Timeline of one pipeline run from a rocprofv3 --kernel-trace CSV: kernels
of the LAST occurrence of the anchor kernel's run (default k_an_entries, the
first kernel of analysis), with start / end offsets in us and the gaps
between kernels (host syncs show up as gaps).

usage: tools/timeline.py <kernel_trace.csv> [anchor]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_an_entries"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    n = re.sub(r"ias::dev::", "", n)
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n


idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
if len(idx) < 2:
    sys.exit("anchor %s found %d times" % (anchor, len(idx)))
lo, hi = idx[-2], idx[-1]
t0 = int(rows[lo]["Start_Timestamp"])
busy_end = t0
for r in rows[lo:hi]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - busy_end) / 1e3
    print("%9.1f %9.1f %8.1f  q%-3s %s%s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"],
                                            short(r["Kernel_Name"])[:56],
                                            ("   <gap %.1f us>" % gap) if gap > 5 else ""))
    busy_end = max(busy_end, e)
print("span %.1f us" % ((busy_end - t0) / 1e3))
