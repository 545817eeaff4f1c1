"""Pin the oracle (oracle/ias_oracle.c, CPU restatement of the reference) to
(1) the known answers recorded from the reference itself (SURVEY.md §4 ->
tests/golden/survey_known_answers.json) and (2) MKL mkl_sparse_sp2m, the
third-party routine behind the reference's Algorithm 1, on the same inputs.
CPU only."""
import json
import os

import numpy as np
import pytest

import ias
import oracle_bind as ob


@pytest.fixture(scope="module")
def known(golden_dir):
    with open(os.path.join(golden_dir, "survey_known_answers.json")) as f:
        return json.load(f)


def transpose(M):
    order = np.lexsort((np.repeat(np.arange(M.rows), np.diff(M.row_ptr)), M.col))
    rows = np.repeat(np.arange(M.rows), np.diff(M.row_ptr))
    cnt = np.bincount(M.col, minlength=M.cols)
    rp = np.zeros(M.cols + 1, np.int64)
    rp[1:] = np.cumsum(cnt)
    return ob.Mat(M.cols, M.rows, rp, rows[order], M.val[order])


def close(a, b):
    return abs(a - b) <= 1e-6 * max(1.0, abs(b))


@pytest.mark.parametrize("name", ["dia.mtx", "small.mtx", "b1_ss.mtx", "Ragusa18.mtx", "LFAT5.mtx",
                                  "Trec5.mtx", "ch3-3-b2.mtx", "relat3.mtx", "sample.mtx"])
def test_known_answers(known, inputs_dir, name):
    k = known["inputs"][name]
    A, _ = ob.mtx_read(os.path.join(inputs_dir, name))
    assert [A.rows, A.cols] == k["shape"] and A.nnz == k["nnz_a"]
    if "aa" in k:
        C = ob.csr_mul_csr(A, A)
        assert ob.flops(A, A) == k["aa"]["flops"]
        assert C.nnz == k["aa"]["nnz"]
        assert close(C.val.sum(), k["aa"]["sum"])
    AT = transpose(A)
    C = ob.csr_mul_csr(A, AT)
    assert ob.flops(A, AT) == k["aat"]["flops"]
    assert C.nnz == k["aat"]["nnz"]
    assert close(C.val.sum(), k["aat"]["sum"])


def test_dia_probe_arrays(known, inputs_dir):
    p = known["dia_mtx_aa_probe"]
    A, _ = ob.mtx_read(os.path.join(inputs_dir, "dia.mtx"))
    C = ob.csr_mul_csr(A, A)
    assert C.row_ptr.tolist() == p["row_ptr"]
    assert C.col.tolist() == p["col"]          # reverse first-touch, exactly the reference's order
    assert C.val.tolist() == [float(v) for v in p["val"]]


def test_cancellation_keeps_structural_zeros():
    A = ob.Mat(2, 2, [0, 2, 4], [0, 1, 0, 1], [1.0, 1.0, 1.0, -1.0])
    C = ob.csr_mul_csr(A, A)
    assert C.nnz == 4 and sorted(C.val.tolist()) == [0.0, 0.0, 2.0, 2.0]


def test_coo_order_forward_first_touch(inputs_dir):
    A, _ = ob.mtx_read(os.path.join(inputs_dir, "dia.mtx"))
    C, rows = ob.coo_mul_coo(A, A)
    assert C.col.tolist() == [0, 1, 2, 1, 2, 3, 2, 3, 3]
    assert rows.tolist() == [0, 0, 0, 1, 1, 1, 2, 2, 3]


def test_ell_matches_csr(inputs_dir):
    A, _ = ob.mtx_read(os.path.join(inputs_dir, "Ragusa18.mtx"))
    C = ob.csr_mul_csr(A, A)
    E = ob.ell_mul_ell(A, A)
    assert E["nnz"] == C.nnz and E["K"] == int(np.diff(C.row_ptr).max())
    for i in range(A.rows):
        n = E["nnz_row"][i]
        s, e = C.row_ptr[i], C.row_ptr[i + 1]
        assert E["col"][i, :n].tolist() == C.col[s:e].tolist()
        assert E["val"][i, :n].tolist() == C.val[s:e].tolist()
        assert not E["col"][i, n:].any() and not E["val"][i, n:].any()


def test_dia_band_pattern():
    """7-diagonal band: C is the full 13-diagonal band (SURVEY §8d K1 shape)."""
    A = ob.Mat.of(ias.gen_band(512, 3, seed=7, value_mode=1))
    D = ob.dia_mul_dia(A, A)
    assert D["nd"] == 13 and D["offsets"].tolist() == list(range(-6, 7))
    C = ob.csr_mul_csr(A, A)
    # every stored CSR entry equals the DIA slot (integer values: exact)
    for i in range(0, 512, 37):
        for p in range(C.row_ptr[i], C.row_ptr[i + 1]):
            slot = D["ind"][C.col[p] - i + 512 - 1]
            assert D["val"][i, slot] == C.val[p]


def test_dia_duplicate_overwrites():
    """CSRtoDIA keeps the last of duplicate (i,j) entries (dia:73-83)."""
    A = ob.Mat(2, 2, [0, 2, 3], [0, 0, 1], [5.0, 7.0, 1.0])
    D = ob.csr_to_dia(A)
    assert D["offsets"].tolist() == [0] and D["val"][0, 0] == 7.0


def test_gates():
    A = ob.Mat.of(ias.gen_band(256, 3, seed=1))
    coo, ell, dia = ob.gate_choices(A, 50.0)
    assert coo and ell and dia
    # one long row makes ELL padding explode; scattered entries make DIA explode
    n = 2000
    rp = np.zeros(n + 1, np.int64)
    rp[1] = n
    rp[2:] = n + np.arange(1, n)
    col = np.concatenate([np.arange(n), (np.arange(1, n) * 7919) % n]).astype(np.int32)
    B = ob.Mat(n, n, rp, col, np.ones(col.size))
    coo, ell, dia = ob.gate_choices(B, 50.0)
    assert coo and not ell and not dia


@pytest.mark.parametrize("maker", [lambda: ias.gen_rmat(12, 16, seed=1),
                                   lambda: ias.gen_ell(4096, 16, seed=7),
                                   lambda: ias.gen_band(4096, 3, seed=7)], ids=["rmat12", "ell4k", "band4k"])
def test_oracle_vs_mkl(maker):
    ok, _ = ias.mkl_available()
    if not ok:
        pytest.skip("MKL runtime not present")
    A = maker()
    C = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    M, _ = ias.mkl_sp2m(A, A, threads=4)
    np.testing.assert_array_equal(C.row_ptr, M.row_ptr)
    for i in range(0, A.rows, max(1, A.rows // 500)):
        s, e = C.row_ptr[i], C.row_ptr[i + 1]
        oc, om = np.argsort(C.col[s:e]), np.argsort(M.col[s:e])
        np.testing.assert_array_equal(C.col[s:e][oc], M.col[s:e][om])
        np.testing.assert_allclose(C.val[s:e][oc], M.val[s:e][om], rtol=1e-10, atol=1e-12)
