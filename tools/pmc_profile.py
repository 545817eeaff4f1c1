#!/usr/bin/env python3
"""PMC passes (tools/pmc.sh output) -> the profile bench.py reads
(profiles/pmc_<config>_n<N>.json): per kernel the mean counters per launch,
HBM traffic per launch (FETCH_SIZE + WRITE_SIZE, KiB -> bytes; FETCH_SIZE raw
and x2 — the MI355X_MICROARCH.md gfx950 correction for 16-B-per-lane streams —
side by side, `hbm_bytes_per_launch` uses the raw value: the row kernels read
with 4- and 8-B lanes), L2 hit rate, and SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE; top-level `lds_bank_conflict_ratio` maps the symbolic /
numeric LDS-table kernels to that ratio.

usage: tools/pmc_profile.py gpurun_out/<tag> profiles/pmc_auto_n1.json "source text"
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    name = re.sub(r"ias::dev::", "", name)
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")


def main():
    root, out_path = sys.argv[1], sys.argv[2]
    source = sys.argv[3] if len(sys.argv) > 3 else root
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "pmc_*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            if row["Counter_Name"] in ("SQ_WAVES", "FETCH_SIZE"):
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
    out = {"source": source}
    ratios = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dur[k]
        m["dur_us"] = sum(d) / len(d) if d else 0.0
        if "FETCH_SIZE" in m:
            m["fetch_bytes_raw"] = 1024 * m["FETCH_SIZE"]
            m["fetch_bytes_x2"] = 2 * 1024 * m["FETCH_SIZE"]
        if "WRITE_SIZE" in m:
            m["write_bytes"] = 1024 * m["WRITE_SIZE"]
        if "fetch_bytes_raw" in m and "write_bytes" in m:
            m["hbm_bytes_per_launch"] = int(m["fetch_bytes_raw"] + m["write_bytes"])
        if "TCC_HIT_sum" in m and m.get("TCC_MISS_sum"):
            m["l2_hit"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_bank_conflict_ratio"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
            if re.match(r"k_(sym2|short_sym|short_num|symbolic_part|num2|numeric_val|numeric_dw|numeric_part)", k):
                ratios[k] = round(m["lds_bank_conflict_ratio"], 4)
        out[k] = m
    out["lds_bank_conflict_ratio"] = ratios
    json.dump(out, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(ratios, indent=1))


if __name__ == "__main__":
    main()
