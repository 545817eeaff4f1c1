#!/usr/bin/env python3
"""Timeline of one step from a rocprofv3 --kernel-trace CSV: each kernel's
start / end (us from the step's first kernel), queue and stream, plus the
busy time (union of kernel intervals) vs the step's span.
usage: timeline.py run_kernel_trace.csv MARKER [occurrence] [max_rows]
MARKER is a kernel-name substring that starts a step (e.g. k_row_blocks)."""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*$", "", n)
    n = re.sub(r"^void ", "", n)
    return n[:70]


def main():
    path, marker = sys.argv[1], sys.argv[2]
    occ = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    maxr = int(sys.argv[4]) if len(sys.argv) > 4 else 400
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    i0 = starts[occ]
    nxt = [i for i in starts if i > i0]
    i1 = nxt[0] if nxt else len(rows)
    step = rows[i0:i1]
    t0 = int(step[0]["Start_Timestamp"])
    iv = []
    for r in step[:maxr]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        iv.append((s, e))
        print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:8.1f}  q{r['Queue_Id']:>2} s{r['Stream_Id']:>2}  {short(r['Kernel_Name'])}")
    iv = sorted((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0) for r in step)
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = max(e for _, e in iv)
    print(f"kernels {len(step)}  span {span/1e6:.3f} ms  busy {busy/1e6:.3f} ms  idle {(span-busy)/1e6:.3f} ms")


if __name__ == "__main__":
    main()
