#!/usr/bin/env python3
"""Per-row nnz of C = A*A (K3' unless told otherwise) from a library variant
(IAS_LIB) against the oracle's CSR_MUL_CSR row counts: which rows differ, and
in which symbolic bin (by products) they sit — localises a wrong count to the
kernel that produced it.
usage: IAS_LIB=... python tools/row_nnz_diff.py [scale ef seed]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

BINS = [(0, 256, "short"), (257, 2048, "sym3"), (2049, 4096, "sym4"), (4097, 16384, "sym5"),
        (16385, 1 << 40, "cbm / partitions")]


def main():
    import torch
    import ias
    import oracle_bind as ob
    sc, ef, seed = (int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (20, 20.0, 2)
    A = ias.gen_rmat(sc, ef, 0.45, 0.15, 0.15, seed, 0)
    rp_ref, _ = ob.csr_mul_csr_digest(ob.Mat.of(A), ob.Mat.of(A))
    ref = np.diff(rp_ref)
    ln = np.diff(A.row_ptr)
    cs = np.concatenate([[0], np.cumsum(ln[A.col])])
    prod = cs[A.row_ptr[1:]] - cs[A.row_ptr[:-1]]
    dev = torch.device("cuda", 0)
    rp = torch.from_numpy(A.row_ptr).to(dev)
    ci = torch.from_numpy(A.col).to(dev)
    va = torch.from_numpy(A.val).to(dev)
    M = ias.Csr(A.rows, A.cols, A.nnz, C.cast(C.c_void_p(rp.data_ptr()), ias.i64p),
                C.cast(C.c_void_p(ci.data_ptr()), ias.i32p), C.cast(C.c_void_p(va.data_ptr()), ias.f64p),
                ias.MEMORY_DEVICE, 0)
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
    out = torch.empty(A.rows + 1, dtype=torch.int64, device=dev)
    for call in range(2):
        n = C.c_int64(0)
        st = ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(M), C.byref(M), C.byref(n),
                                         C.cast(C.c_void_p(out.data_ptr()), ias.i64p), None)
        if st != 0:
            print("call", call, "status", st, ias.lib.ias_last_error().decode(), flush=True)
            return 1
        got = np.diff(out.cpu().numpy())
        bad = np.nonzero(got != ref)[0]
        print(f"call {call}: nnz {int(n.value)} want {int(rp_ref[-1])}; rows differing {bad.size}", flush=True)
        for lo, hi, name in BINS:
            m = (prod[bad] >= lo) & (prod[bad] <= hi)
            if m.any():
                d = got[bad[m]] - ref[bad[m]]
                print(f"   {name:18s} rows {m.sum():7d}  extra nnz {int(d.sum()):9d}  e.g. rows {bad[m][:5].tolist()} "
                      f"products {prod[bad[m]][:5].tolist()} got {got[bad[m]][:5].tolist()} want {ref[bad[m]][:5].tolist()}",
                      flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
