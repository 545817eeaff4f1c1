#!/usr/bin/env python3
"""Rows each sym3 / sym4 / sym5 bin hands to sym2 on K3' (IAS_RETRY_PRINT=1
makes the library print them after each symbolic pass).
usage: IAS_LIB=... IAS_RETRY_PRINT=1 python tools/retry_counts.py [scale ef seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))


def main():
    import ctypes as C
    import torch
    import ias
    sc, ef, seed = (int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (20, 20.0, 2)
    A = ias.gen_rmat(sc, ef, 0.45, 0.15, 0.15, seed, 0)
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
    n = C.c_int64(0)
    st = ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(M), C.byref(M), C.byref(n),
                                     C.cast(C.c_void_p(out.data_ptr()), ias.i64p), None)
    print("status", st, "nnz", n.value, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
