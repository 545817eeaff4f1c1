"""Matrix-Market reader/writer and the format layer (host code) against the
oracle restatement of main.cpp:143-458 and CSRtoCOO/ELL/DIA.  CPU only."""
import ctypes as C
import os

import numpy as np
import pytest

import ias
import oracle_bind as ob

NAMES = ["dia.mtx", "small.mtx", "b1_ss.mtx", "Ragusa18.mtx", "LFAT5.mtx", "Trec5.mtx",
         "ch3-3-b2.mtx", "relat3.mtx", "sample.mtx"]


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


@pytest.mark.parametrize("name", NAMES)
def test_reader_matches_oracle(inputs_dir, name):
    path = os.path.join(inputs_dir, name)
    got, info = ias.mtx_read(path)
    ref, flags = ob.mtx_read(path)
    assert (got.rows, got.cols) == (ref.rows, ref.cols)
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
    np.testing.assert_array_equal(got.col, ref.col)
    np.testing.assert_array_equal(got.val, ref.val)
    assert [info.is_pattern, info.is_real, info.is_integer, info.is_symmetric] == flags


def test_reader_semantics(tmp_path):
    # symmetric mirror (same value), diagonal once, comments skipped, file order kept
    p = write(tmp_path, "s.mtx", "%%MatrixMarket matrix coordinate real symmetric\n% c\n%\n"
                                 "3 3 4\n2 1 5.5\n1 1 2\n3 2 -1\n3 3 7\n")
    A, info = ias.mtx_read(p)
    assert info.is_symmetric == 1 and A.nnz == 6
    assert A.row_ptr.tolist() == [0, 2, 4, 6]
    assert A.col.tolist() == [1, 0, 0, 2, 1, 2]
    assert A.val.tolist() == [5.5, 2.0, 5.5, -1.0, -1.0, 7.0]
    # skew-symmetric is NOT mirrored (main.cpp:317-332)
    p = write(tmp_path, "k.mtx", "%%MatrixMarket matrix coordinate real skew-symmetric\n2 2 1\n2 1 3\n")
    A, info = ias.mtx_read(p)
    assert info.is_symmetric == 0 and A.nnz == 1
    # pattern -> 1.0, duplicates kept, unsorted columns kept, case-insensitive banner
    p = write(tmp_path, "p.mtx", "%%MatrixMarket MATRIX Coordinate PATTERN General\n2 3 4\n1 3\n1 1\n1 3\n2 2\n")
    A, info = ias.mtx_read(p)
    assert info.is_pattern and A.col.tolist() == [2, 0, 2, 1] and A.val.tolist() == [1.0] * 4
    # integer values
    p = write(tmp_path, "i.mtx", "%%MatrixMarket matrix coordinate integer general\n1 1 1\n1 1 -4\n")
    A, info = ias.mtx_read(p)
    assert info.is_integer and A.val.tolist() == [-4.0]


@pytest.mark.parametrize("text,status", [
    ("%%MatrixMarket matrix coordinate complex general\n1 1 1\n1 1 1 0\n", 7),
    ("%%MatrixMarket matrix array real general\n1 1\n1\n", 7),
    ("MatrixMarket matrix coordinate real general\n1 1 1\n1 1 1\n", 6),
    ("%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1\n", 6),
    ("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1\n", 6),
])
def test_reader_errors(tmp_path, text, status):
    p = write(tmp_path, "e.mtx", text)
    with pytest.raises(ias.IasError) as e:
        ias.mtx_read(p)
    assert e.value.status == status


def test_read_pair_forces_b_rows(inputs_dir, tmp_path):
    a = os.path.join(inputs_dir, "Trec5.mtx")          # 3 x 7
    b = write(tmp_path, "b.mtx", "%%MatrixMarket matrix coordinate real general\n5 2 2\n1 1 1\n5 2 2\n")
    A, B, ia_, ib = ias.mtx_read_pair(a, b)
    assert (B.rows, B.cols) == (7, 2)                  # B.row = A.col (main.cpp:482)
    assert ib.rows == 5


def test_write_roundtrip(tmp_path):
    A = ias.gen_rmat(8, 4, seed=3)
    p = str(tmp_path / "w.mtx")
    s = A.struct()
    ias.check(ias.lib.ias_mtx_write(p.encode(), C.byref(s)), "write")
    B, info = ias.mtx_read(p)
    np.testing.assert_array_equal(B.row_ptr, A.row_ptr)
    np.testing.assert_array_equal(B.col, A.col)
    np.testing.assert_allclose(B.val, A.val, rtol=1e-15)


# ------------------------------------------------------------------ format layer
def test_csr_to_dia_matches_oracle(inputs_dir):
    for name in ["dia.mtx", "Ragusa18.mtx", "b1_ss.mtx"]:
        A, _ = ias.mtx_read(os.path.join(inputs_dir, name))
        ref = ob.csr_to_dia(ob.Mat.of(A))
        s, d = A.struct(), ias.Dia()
        ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(d), 0.0), "to_dia")
        nd = d.num_diagonals
        assert nd == ref["nd"]
        np.testing.assert_array_equal(ias._np(d.diagonal_offsets, nd, np.int32), ref["offsets"])
        np.testing.assert_array_equal(ias._np(d.diagonal_ind, d.rows + d.cols - 1, np.int32), ref["ind"])
        np.testing.assert_array_equal(ias._np(d.val, d.rows * nd, np.float64).reshape(d.rows, nd), ref["val"])
        assert ias.lib.ias_sizeof_dia(C.byref(d)) == pytest.approx(
            4.0 * (d.rows + d.cols - 1 + nd + 3) + 8.0 * d.rows * nd)
        ias.lib.ias_dia_free(C.byref(d))


def test_gates_match_oracle():
    for A in [ias.gen_band(300, 3), ias.gen_rmat(10, 8, seed=1), ias.gen_ell(500, 7)]:
        want = ob.gate_choices(ob.Mat.of(A), 50.0)
        s = A.struct()
        co, el, di = ias.Coo(), ias.Ell(), ias.Dia()
        got = (ias.lib.ias_csr_to_coo(C.byref(s), C.byref(co), 50.0) == 0,
               ias.lib.ias_csr_to_ell(C.byref(s), C.byref(el), 50.0) == 0,
               ias.lib.ias_csr_to_dia(C.byref(s), C.byref(di), 50.0) == 0)
        assert got == want
        assert co.choice == want[0] and el.choice == want[1] and di.choice == want[2]
        ias.lib.ias_coo_free(C.byref(co)); ias.lib.ias_ell_free(C.byref(el)); ias.lib.ias_dia_free(C.byref(di))


def test_format_roundtrips():
    A = ias.gen_rmat(9, 6, seed=4)
    s = A.struct()
    co, el, back = ias.Coo(), ias.Ell(), ias.Csr()
    ias.check(ias.lib.ias_csr_to_coo(C.byref(s), C.byref(co), 0.0), "coo")
    ias.check(ias.lib.ias_coo_to_csr(C.byref(co), C.byref(back)), "coo->csr")
    b = ias.csr_to_numpy(back)
    np.testing.assert_array_equal(b.col, A.col)
    rows = ias._np(co.row, co.nnz, np.int32)
    np.testing.assert_array_equal(rows, np.repeat(np.arange(A.rows), np.diff(A.row_ptr)))
    ias.check(ias.lib.ias_csr_to_ell(C.byref(s), C.byref(el), 0.0), "ell")
    assert el.max_nnz_per_row == np.diff(A.row_ptr).max()
    back = ias.Csr()
    ias.check(ias.lib.ias_ell_to_csr(C.byref(el), C.byref(back)), "ell->csr")
    b = ias.csr_to_numpy(back)
    np.testing.assert_array_equal(b.row_ptr, A.row_ptr)
    np.testing.assert_array_equal(b.val, A.val)
    ias.lib.ias_coo_free(C.byref(co)); ias.lib.ias_ell_free(C.byref(el))


def test_dia_to_csr_band():
    A = ias.gen_band(100, 2, seed=1)
    s, d, back = A.struct(), ias.Dia(), ias.Csr()
    ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(d), 0.0), "dia")
    ias.check(ias.lib.ias_dia_to_csr(C.byref(d), C.byref(back)), "dia->csr")
    b = ias.csr_to_numpy(back)
    np.testing.assert_array_equal(b.row_ptr, A.row_ptr)
    np.testing.assert_array_equal(b.col, A.col)
    np.testing.assert_array_equal(b.val, A.val)
    ias.lib.ias_dia_free(C.byref(d))


def test_transpose():
    A = ias.gen_rmat(9, 6, seed=5)
    s, t = A.struct(), ias.Csr()
    ias.check(ias.lib.ias_csr_transpose(C.byref(s), C.byref(t)), "T")
    T = ias.csr_to_numpy(t)
    dense = np.zeros((A.rows, A.cols))
    np.add.at(dense, (np.repeat(np.arange(A.rows), np.diff(A.row_ptr)), A.col), A.val)
    dt = np.zeros((T.rows, T.cols))
    np.add.at(dt, (np.repeat(np.arange(T.rows), np.diff(T.row_ptr)), T.col), T.val)
    np.testing.assert_array_equal(dt, dense.T)
    for i in range(T.rows):   # ascending source rows (mkl_dcsrcsc order)
        seg = T.col[T.row_ptr[i]:T.row_ptr[i + 1]]
        assert np.all(np.diff(seg) >= 0)


def test_flops_sums_partition():
    A = ias.gen_rmat(11, 8, seed=6)
    assert ias.flops(A, A) == ob.flops(ob.Mat.of(A), ob.Mat.of(A))
    s = A.struct()
    v = C.c_double(0)
    ias.check(ias.lib.ias_sum_csr(C.byref(s), C.byref(v)), "sum")
    assert v.value == pytest.approx(A.val.sum(), rel=1e-12)
    for parts in (1, 2, 3, 8):
        b = (C.c_int64 * (parts + 1))()
        ias.check(ias.lib.ias_partition_rows(C.byref(s), C.byref(s), parts, b), "partition")
        bl = list(b)
        assert bl[0] == 0 and bl[-1] == A.rows and all(x <= y for x, y in zip(bl, bl[1:]))
        rl = np.diff(A.row_ptr)
        prod = np.zeros(A.rows, np.int64)
        np.add.at(prod, np.repeat(np.arange(A.rows), rl), rl[A.col])
        # the documented cost model (include/ias.h, convert.cpp): 1710 per row +
        # 10 per product, 34 per product of rows beyond 16384 products
        cost = 1710 + prod * np.where(prod > 16384, 34, 10)
        w = [cost[bl[k]:bl[k + 1]].sum() for k in range(parts)]
        assert max(w) <= (sum(w) / parts) * 1.05 + cost.max() + 1
