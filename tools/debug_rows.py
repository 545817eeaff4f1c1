#!/usr/bin/env python3
"""Debug aid (GPU box): C = A*A on the device for a generator config, then the
rows whose product count lies in [PLO, PHI] compared bit for bit with the
oracle (A restricted to those rows times A).  Prints the first mismatching
rows: products, nnz, first differing position, columns / values there.

usage: PLO=8193 PHI=16384 python tools/debug_rows.py k3p_rmat20_ef20_s2"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ias  # noqa: E402
import oracle_bind as ob  # noqa: E402
from test_fullsize import STATS, device_spgemm, make  # noqa: E402
import torch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "k3p_rmat20_ef20_s2"
plo, phi = int(os.environ.get("PLO", "8193")), int(os.environ.get("PHI", "16384"))
A = make(STATS[name])
blen = np.diff(A.row_ptr)
prod = np.zeros(A.rows, np.int64)
np.add.at(prod, np.repeat(np.arange(A.rows), blen), blen[A.col])
sel = np.nonzero((prod >= plo) & (prod <= phi))[0]
print("rows selected", len(sel), "products", int(prod[sel].sum()), flush=True)
c_rp, c_ci, c_va, _ = device_spgemm(torch, A)
rp = c_rp.cpu().numpy()
# oracle on the selected rows
sub_len = blen[sel]
sub_rp = np.zeros(len(sel) + 1, np.int64)
sub_rp[1:] = np.cumsum(sub_len)
idx = np.concatenate([np.arange(A.row_ptr[r], A.row_ptr[r + 1]) for r in sel])
As = ob.Mat(len(sel), A.cols, sub_rp, A.col[idx], A.val[idx])
Bm = ob.Mat(A.rows, A.cols, A.row_ptr, A.col, A.val)
R = ob.csr_mul_csr(As, Bm)
bad = 0
for i, r in enumerate(sel):
    s, e = int(rp[r]), int(rp[r + 1])
    oc = R.col[R.row_ptr[i]:R.row_ptr[i + 1]]
    ov = R.val[R.row_ptr[i]:R.row_ptr[i + 1]]
    gc = c_ci[s:e].cpu().numpy()
    gv = c_va[s:e].cpu().numpy()
    if len(oc) != len(gc) or not np.array_equal(oc, gc) or not np.array_equal(ov.view(np.int64), gv.view(np.int64)):
        bad += 1
        if bad <= 8:
            n = min(len(oc), len(gc))
            dc = np.nonzero(oc[:n] != gc[:n])[0]
            dv = np.nonzero(ov[:n].view(np.int64) != gv[:n].view(np.int64))[0]
            print("row", int(r), "products", int(prod[r]), "nnz gpu/oracle", len(gc), len(oc),
                  "col diffs", len(dc), dc[:6].tolist(), "val diffs", len(dv), dv[:6].tolist())
            if len(dv):
                j = int(dv[0])
                print("   at", j, "col", int(oc[j]), int(gc[j]), "val", ov[j], gv[j], "ratio", gv[j] / ov[j] if ov[j] else None)
print("bad rows", bad, "of", len(sel))
