"""The full-size digest (tests/fulldigest.py) agrees with the oracle's
streaming digest (ora_csr_mul_csr_digest) on products small enough to
materialise, and its torch form (run on the GPU's C by test_fullsize.py)
agrees with the numpy form — so a digest match at full size means C matches
the oracle entry for entry."""
import numpy as np
import pytest

import ias
import oracle_bind as ob
from fulldigest import digest_numpy, digest_torch


@pytest.mark.parametrize("A", [ias.gen_rmat(12, 16, seed=1), ias.gen_band(4096, 3, seed=7),
                               ias.gen_ell(8192, 16, seed=7), ias.gen_rmat(11, 8, seed=4, value_mode=1)],
                         ids=["rmat12", "band4k", "ell8k", "rmat11_int"])
def test_digest_matches_materialised_oracle(A):
    M = ob.Mat.of(A)
    ref = ob.csr_mul_csr(M, M)
    rp, dg = ob.csr_mul_csr_digest(M, M)
    np.testing.assert_array_equal(rp, ref.row_ptr)
    assert digest_numpy(ref.row_ptr, ref.col, ref.val) == dg
    # order and value bits matter: swapping two entries of a row, or one ulp, changes it
    i = int(np.argmax(np.diff(ref.row_ptr) >= 2))
    s = int(ref.row_ptr[i])
    col2 = ref.col.copy()
    col2[s], col2[s + 1] = col2[s + 1], col2[s]
    assert digest_numpy(ref.row_ptr, col2, ref.val) != dg
    val2 = ref.val.copy()
    val2[s] = np.nextafter(val2[s], np.inf)
    assert digest_numpy(ref.row_ptr, ref.col, val2) != dg


def test_torch_digest_equals_numpy():
    torch = pytest.importorskip("torch")
    A = ias.gen_rmat(12, 16, seed=1)
    M = ob.Mat.of(A)
    ref = ob.csr_mul_csr(M, M)
    want = digest_numpy(ref.row_ptr, ref.col, ref.val)
    got = digest_torch(torch.from_numpy(ref.row_ptr), torch.from_numpy(ref.col), torch.from_numpy(ref.val),
                       chunk=100_000)
    assert got == want


def test_digest_adds_over_row_blocks():
    """A row-block split of C (the K4 shards, tests/test_k4.py) digests to the
    whole C's digest when each block's rows carry their global index (row0)."""
    torch = pytest.importorskip("torch")
    A = ias.gen_rmat(12, 16, seed=1)
    M = ob.Mat.of(A)
    ref = ob.csr_mul_csr(M, M)
    want = digest_numpy(ref.row_ptr, ref.col, ref.val)
    rp = torch.from_numpy(ref.row_ptr)
    col, val = torch.from_numpy(ref.col), torch.from_numpy(ref.val)
    bounds = [0, 7, 700, 2048, 4000, A.rows]
    total = 0
    for r0, r1 in zip(bounds[:-1], bounds[1:]):
        s, e = int(rp[r0]), int(rp[r1])
        total += digest_torch(rp[r0:r1 + 1], col[s:e], val[s:e], chunk=50_000, row0=r0)
    assert total % (1 << 64) == want
    # without the global row index the blocks do not add up
    s, e = int(rp[700]), int(rp[A.rows])
    assert digest_torch(rp[:701], col[:s], val[:s]) + digest_torch(rp[700:], col[s:e], val[s:e]) != want


@pytest.mark.parametrize("A", [ias.gen_rmat(12, 16, seed=1), ias.gen_ell(8192, 16, seed=7)], ids=["rmat12", "ell8k"])
def test_sorted_digest_matches_sorted_oracle(A):
    """ora_csr_mul_csr_digest_sorted (the IAS_ORDER_SORTED pin of
    test_fullsize_sorted_row_pointer) = the digest of the materialised oracle C
    with each row sorted by column, and differs from the reference-order digest."""
    M = ob.Mat.of(A)
    ref = ob.csr_mul_csr(M, M)
    col, val = ref.col.copy(), ref.val.copy()
    for i in range(A.rows):
        s, e = int(ref.row_ptr[i]), int(ref.row_ptr[i + 1])
        o = np.argsort(col[s:e], kind="stable")
        col[s:e], val[s:e] = col[s:e][o], val[s:e][o]
    rp, dg = ob.csr_mul_csr_digest(M, M, sorted_rows=True)
    np.testing.assert_array_equal(rp, ref.row_ptr)
    assert digest_numpy(ref.row_ptr, col, val) == dg
    assert dg != ob.csr_mul_csr_digest(M, M)[1]


def test_recorded_sorted_digest_small():
    """the recorded c_digest_sorted of the small R-MAT case reproduces"""
    import json, os
    rec = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "generator_stats.json")))["rmat12_ef16_s1"]
    A = ias.gen_rmat(*rec["args"])
    assert ob.csr_mul_csr_digest(ob.Mat.of(A), ob.Mat.of(A), sorted_rows=True)[1] == rec["c_digest_sorted"]
