#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (compile-only, no GPU).

usage: tools/resources.py [source.hip]   (default ia-spgemm_amd/csrc/spgemm.hip)
"""
import os
import re
import subprocess
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "ia-spgemm_amd/csrc/spgemm.hip")
pkg = os.path.join(root, "ia-spgemm_amd")
cmd = ["hipcc", "-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-std=c++17", "-fPIC",
       "-I" + os.path.join(root, "include"), "-I" + os.path.join(pkg, "csrc"), "--cuda-device-only",
       "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("RES_FLAGS", "").split()
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                     text=True).stdout.splitlines()
print("%-60s %5s %5s %5s %7s %4s" % ("kernel", "vgpr", "sspl", "vspl", "lds", "occ"))
for r, d in zip(rows, dem):
    d = re.sub(r"ias::dev::", "", d)
    d = re.sub(r"\(.*", "", d).replace("void ", "")
    print("%-60s %5s %5s %5s %7s %4s" % (d[:60], r.get("VGPRs"), r.get("SGPRs Spill"), r.get("VGPRs Spill"),
                                         r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]")))
