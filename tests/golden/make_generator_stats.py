"""Records the exact statistics of the deterministic generators
(ia-spgemm_amd/csrc/gen.cpp) into generator_stats.json; tests/test_generators.py
checks the library still produces them.  nnz(C) comes from the oracle."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "ia-spgemm_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
import ias  # noqa: E402
import oracle_bind as ob  # noqa: E402

CASES = {
    "rmat12_ef16_s1": ("rmat", (12, 16.0, 0.45, 0.15, 0.15, 1, 0)),
    "rmat14_ef20_s2_int": ("rmat", (14, 20.0, 0.45, 0.15, 0.15, 2, 1)),
    "band4096_h3_s7": ("band", (4096, 3, 7, 0)),
    "ell8192_k16_s7": ("ell", (8192, 16, 7, 0)),
    "k3p_rmat20_ef20_s2": ("rmat", (20, 20.0, 0.45, 0.15, 0.15, 2, 0)),
}


def make(kind, args):
    return {"rmat": ias.gen_rmat, "band": ias.gen_band, "ell": ias.gen_ell}[kind](*args)


def digest(A):
    h = hashlib.sha256()
    for a in (A.row_ptr, A.col, A.val):
        h.update(a.tobytes())
    return h.hexdigest()


if __name__ == "__main__":
    out = {}
    for name, (kind, args) in CASES.items():
        A = make(kind, args)
        rec = {"kind": kind, "args": list(args), "rows": A.rows, "nnz": A.nnz,
               "flops": ias.flops(A, A), "sha256": digest(A)}
        if A.nnz < 5_000_000:
            rec["nnz_c"] = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A)).nnz
        out[name] = rec
        print(name, rec)
    with open(os.path.join(HERE, "generator_stats.json"), "w") as f:
        json.dump(out, f, indent=1)
