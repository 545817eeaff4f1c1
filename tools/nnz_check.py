#!/usr/bin/env python3
"""nnz(C) of K3' / K3 through the two-phase device ABI, repeated: a quick
consistency check of a library variant (IAS_LIB) against the recorded oracle
counts (tests/golden/generator_stats.json) before a full test run.
usage: IAS_LIB=... python tools/nnz_check.py [k3p k3 ...]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))

CFG = {"k3p": (20, 20, 2), "k3": (20, 32, 1)}


def main():
    import torch
    import ias
    stats = json.load(open(os.path.join(ROOT, "tests", "golden", "generator_stats.json")))
    names = sys.argv[1:] or ["k3p"]
    dev = torch.device("cuda", 0)
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
    ok = True
    for nm in names:
        sc, ef, seed = CFG[nm]
        A = ias.gen_rmat(sc, ef, 0.45, 0.15, 0.15, seed, 0)
        rec = [v for k, v in stats.items() if k.startswith(f"{nm}_") or k == nm]
        want = rec[0]["nnz_c"] if rec else None
        rp = torch.from_numpy(A.row_ptr).to(dev)
        ci = torch.from_numpy(A.col).to(dev)
        va = torch.from_numpy(A.val).to(dev)
        M = ias.Csr(A.rows, A.cols, A.nnz, C.cast(C.c_void_p(rp.data_ptr()), ias.i64p),
                    C.cast(C.c_void_p(ci.data_ptr()), ias.i32p), C.cast(C.c_void_p(va.data_ptr()), ias.f64p),
                    ias.MEMORY_DEVICE, 0)
        got = []
        for _ in range(3):
            n = C.c_int64(0)
            ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(M), C.byref(M), C.byref(n), None, None), "nnz")
            got.append(int(n.value))
        good = want is not None and all(g == want for g in got)
        ok = ok and good
        print(f"{os.path.basename(os.environ.get('IAS_LIB', 'in-tree'))} {nm}: nnz {got} want {want} "
              f"{'OK' if good else 'MISMATCH'}", flush=True)
    ias.lib.ias_plan_destroy(plan)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
