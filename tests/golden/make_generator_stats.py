"""Records the exact statistics of the deterministic generators
(ia-spgemm_amd/csrc/gen.cpp) into generator_stats.json; tests/test_generators.py
checks the library still produces them.  nnz(C), the sha256 of C's row
pointer and the order-sensitive digest of C (tests/fulldigest.py) come from
the oracle's CSR_MUL_CSR restatement, folded row by row
(ora_csr_mul_csr_digest), so the full-size configurations K1-K3 and K3'
 are pinned even where C does not fit host memory; the GPU
tests (tests/test_fullsize.py) compare the engine's C against these."""
import hashlib
import json
import os
import sys
import time

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
    # the BASELINE.json configurations at full size
    "k1_band262144_h3_s7": ("band", (1 << 18, 3, 7, 0)),
    "k2_ell1048576_k16_s7": ("ell", (1 << 20, 16, 7, 0)),
    "k3p_rmat20_ef20_s2": ("rmat", (20, 20.0, 0.45, 0.15, 0.15, 2, 0)),
    "k3_rmat20_ef32_s1": ("rmat", (20, 32.0, 0.45, 0.15, 0.15, 1, 0)),
    # K4: the 8-GPU configuration (R-MAT 2^23, edge factor 24, seed 3); C has
    # ~1.2e10 entries (~143 GB), so only the streaming digest is recorded
    "k4_rmat23_ef24_s3": ("rmat", (23, 24.0, 0.45, 0.15, 0.15, 3, 0)),
}


# configurations whose sorted-order digest is recorded too
SORTED = {"rmat12_ef16_s1", "k2_ell1048576_k16_s7", "k3p_rmat20_ef20_s2"}


def make(kind, args):
    return {"rmat": ias.gen_rmat, "band": ias.gen_band, "ell": ias.gen_ell}[kind](*args)


def digest(A):
    h = hashlib.sha256()
    for a in (A.row_ptr, A.col, A.val):
        h.update(a.tobytes())
    return h.hexdigest()


if __name__ == "__main__":
    only = set(sys.argv[1:])
    path = os.path.join(HERE, "generator_stats.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name, (kind, args) in CASES.items():
        if only and name not in only:
            continue
        t = time.time()
        A = make(kind, args)
        rec = {"kind": kind, "args": list(args), "rows": A.rows, "nnz": A.nnz,
               "flops": ias.flops(A, A), "sha256": digest(A)}
        rp, dg = ob.csr_mul_csr_digest(ob.Mat.of(A), ob.Mat.of(A))
        rec["nnz_c"] = int(rp[-1])
        rec["c_row_ptr_sha256"] = hashlib.sha256(rp.tobytes()).hexdigest()
        rec["c_digest"] = dg
        if name in SORTED:   # the IAS_ORDER_SORTED pin (tests/test_fullsize.py)
            _, rec["c_digest_sorted"] = ob.csr_mul_csr_digest(ob.Mat.of(A), ob.Mat.of(A), sorted_rows=True)
        out[name] = rec
        print(name, rec, f"{time.time() - t:.1f}s", flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
