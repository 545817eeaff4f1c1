#!/usr/bin/env python3
"""Turn a tools/pmc_summary.py --json output into profiles/pmc_<config>_n<N>.json,
the file bench.py reads roofline.traffic from (HBM bytes per launch of the
roofline kernel, k_numeric_flat).

FETCH_SIZE / WRITE_SIZE are KiB in rocprofv3.  MI355X_MICROARCH.md (HBM):
FETCH_SIZE reports half the bytes of a wide coalesced *16-B-per-lane* stream;
other access widths are uncalibrated.  k_numeric_flat reads with 4- and 8-byte
lanes (product columns, gathered B values, bitmap words), so the raw counter
is used for `hbm_bytes_per_launch` and the x2 figure is kept beside it.

usage: tools/pmc_to_profile.py summary.json out.json [source-note]
"""
import json
import sys

summ = json.load(open(sys.argv[1]))
out = {"source": sys.argv[3] if len(sys.argv) > 3 else sys.argv[1]}
for k, m in summ.items():
    if "FETCH_SIZE" not in m or "WRITE_SIZE" not in m:
        continue
    fetch = 1024.0 * m["FETCH_SIZE"]
    write = 1024.0 * m["WRITE_SIZE"]
    out[k] = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes_raw": round(fetch),
              "fetch_bytes_x2": round(2 * fetch), "write_bytes": round(write),
              "dur_us": round(m.get("dur_us", 0.0), 1), "l2_hit": m.get("l2_hit")}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out.get("k_numeric_flat", {})))
