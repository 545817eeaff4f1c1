#!/usr/bin/env python3
"""Per-kernel PMC means (rocprofv3 --pmc CSVs under <root>/pmc_*) ->
profiles/pmc_<config>_n<N>.json, the file bench.py reads roofline.traffic and
lds_bank_conflict_ratio from.

FETCH_SIZE / WRITE_SIZE are KiB.  Calibrated on this GPU with
tools/fetch_probe.hip (profiles/r03/fetch_probe.txt): every 128-B read
request beyond L2 is tallied as 64 B, for 4-, 8- and 16-byte lanes alike
(4 GiB streamed: FETCH_SIZE = 2.097e6 KiB, TCC_EA0_RDREQ = 2^25 = 4 GiB / 128 B),
so read bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for 4- and 16-byte
stores.  `hbm_bytes_per_launch` = 2 x FETCH + WRITE: bytes beyond L2 (the
Infinity Cache may still serve part of the reads).

usage: tools/pmc_to_profile.py <root> out.json [note]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

root, dst = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "").replace("ias::dev::", "")
        k = re.sub(r"^k_num2<.*>$", "k_num2", k)   # the streaming pass's instantiations (bench.py's key)
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {"source": sys.argv[3] if len(sys.argv) > 3 else root,
       "calibration": "read bytes = 2 x FETCH_SIZE (tools/fetch_probe.hip); WRITE_SIZE exact"}
lds = {}
for k, cs in sorted(vals.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    e = {}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        fetch, write = 2 * 1024.0 * m["FETCH_SIZE"], 1024.0 * m["WRITE_SIZE"]
        e.update(hbm_bytes_per_launch=round(fetch + write), read_bytes=round(fetch), write_bytes=round(write),
                 fetch_size_kib_raw=round(m["FETCH_SIZE"], 1))
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m and m["TCC_HIT_sum"] + m["TCC_MISS_sum"] > 0:
        e["l2_hit"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
    if m.get("SQ_LDS_IDX_ACTIVE", 0) > 0:
        e["lds_bank_conflict_ratio"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 4)
        lds[k] = e["lds_bank_conflict_ratio"]
    if e:
        out[k] = e
out["lds_bank_conflict_ratio"] = lds
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out.get("k_num2", {})))
