#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc CSVs (tools/pmc.sh) per kernel: mean counter
value per dispatch, plus derived ratios.  FETCH_SIZE is doubled for gfx950
wide streaming reads (MI355X_MICROARCH.md §HBM: it reports half the bytes);
both sizes are in KiB in rocprofv3 and converted to bytes here.

usage: tools/pmc_summary.py gpurun_out/pmc1 [--json out.json]
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
    return name.replace("void ", "")[:48]


def main():
    root = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "pmc_*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            if row["Counter_Name"] in ("SQ_WAVES", "FETCH_SIZE"):
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
    out = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dur[k]
        m["dur_us"] = sum(d) / len(d) if d else 0.0
        if "FETCH_SIZE" in m:
            m["fetch_bytes_x2"] = 2 * 1024 * m["FETCH_SIZE"]
        if "WRITE_SIZE" in m:
            m["write_bytes"] = 1024 * m["WRITE_SIZE"]
        if "TCC_HIT_sum" in m and m.get("TCC_MISS_sum"):
            m["l2_hit"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        if m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    m[c + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
        out[k] = m
    keys = sorted(out, key=lambda k: -out[k]["dur_us"])
    cols = ["dur_us", "SQ_WAVES", "SQ_WAIT_ANY_frac", "SQ_WAIT_INST_ANY_frac", "SQ_ACTIVE_INST_ANY_frac",
            "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
            "fetch_bytes_x2", "write_bytes", "l2_hit"]
    print("%-48s " % "kernel" + " ".join("%12s" % c[:12] for c in cols))
    for k in keys:
        print("%-48s " % k + " ".join("%12.4g" % out[k].get(c, float("nan")) for c in cols))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
