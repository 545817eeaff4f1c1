"""GPU parity: the HIP path (through the C-ABI) against the oracle restatement
of the reference (oracle/ias_oracle.c) on the same seeded inputs.

Bar: integer / index work bit-exact; values bit-exact too, because the HIP
kernels sum every output entry in the reference's product order without FMA
(the reference's CSR_MUL_CSR / COO_MUL_COO / ELL_MUL_ELL / DIA_mul_DIA
semantics).  The MKL cross-check uses the north-star tolerance
|dC| <= 1e-10 * max(|c|, sum|a_ik*b_kj|).
"""
import ctypes as C
import os

import numpy as np
import pytest

import ias
import oracle_bind as ob

pytestmark = pytest.mark.gpu

SQUARE = ["dia.mtx", "small.mtx", "b1_ss.mtx", "Ragusa18.mtx", "LFAT5.mtx"]
ALL = SQUARE + ["Trec5.mtx", "ch3-3-b2.mtx", "relat3.mtx", "sample.mtx"]


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if ias.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X box")


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.int64)


def assert_csr_identical(got, ref, what=""):
    assert got.rows == ref.rows and got.cols == ref.cols, what
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(got.col, ref.col, err_msg=f"{what} col order")
    np.testing.assert_array_equal(bits(got.val), bits(ref.val), err_msg=f"{what} values (bitwise)")


def sorted_form(m):
    rp, col, val = m.row_ptr, m.col, m.val
    oc, ov = np.empty_like(col), np.empty_like(val)
    for i in range(m.rows):
        s, e = rp[i], rp[i + 1]
        o = np.argsort(col[s:e], kind="stable")
        oc[s:e], ov[s:e] = col[s:e][o], val[s:e][o]
    return oc, ov


def transpose(m):
    s = ias.HostCsr(m.rows, m.cols, m.row_ptr, m.col, m.val).struct()
    t = ias.Csr()
    ias.check(ias.lib.ias_csr_transpose(C.byref(s), C.byref(t)), "transpose")
    return ias.csr_to_numpy(t)


def cases_small():
    """(name, A, B) synthetic cases at oracle-friendly sizes."""
    out = []
    out.append(("band4k", ias.gen_band(4096, 3, seed=7), None))
    out.append(("band4k_int", ias.gen_band(4096, 3, seed=7, value_mode=1), None))
    out.append(("ell8k", ias.gen_ell(8192, 16, seed=7), None))
    out.append(("rmat12", ias.gen_rmat(12, 16, seed=1), None))
    out.append(("rmat14_int", ias.gen_rmat(14, 20, seed=2, value_mode=1), None))
    out.append(("rmat15", ias.gen_rmat(15, 8, seed=3), None))
    # cancellation: A=[[1,1],[1,-1]] -> C has 4 stored entries, two of them 0.0
    out.append(("cancel", ias.HostCsr(2, 2, np.array([0, 2, 4]), np.array([0, 1, 0, 1]),
                                      np.array([1.0, 1.0, 1.0, -1.0])), None))
    # duplicates inside rows, empty rows, unsorted columns
    rp = np.array([0, 4, 4, 7, 9, 9])
    col = np.array([3, 1, 3, 0, 2, 2, 4, 1, 0])
    val = np.array([1.5, -2.0, 0.25, 3.0, 1.0, -1.0, 2.0, 0.5, -0.5])
    out.append(("dups", ias.HostCsr(5, 5, rp, col, val), None))
    # signed zeros: 0.0 * negative = -0.0 first product (CSR: 0.0 + -0.0 = +0.0)
    out.append(("negzero", ias.HostCsr(2, 2, np.array([0, 2, 3]), np.array([0, 1, 1]),
                                       np.array([0.0, 1.0, -3.0])), None))
    return out


def long_rows(n=40000, head=3000, per=10, seed=5):
    """Row 0 has `head` entries into rows of `per` columns each: products beyond
    every LDS bin, so the global-memory tables (symbolic and numeric) run."""
    rng = np.random.default_rng(seed)
    rows = [np.arange(head)] + [np.sort(rng.choice(n, per, replace=False)) for _ in range(n - 1)]
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.integers(1, 10, size=col.size).astype(np.float64)
    return ias.HostCsr(n, n, rp, col, val)


# ------------------------------------------------------------------ CSR
@pytest.mark.parametrize("name", SQUARE)
def test_csr_inputs_a_times_a(inputs_dir, name):
    A, _ = ias.mtx_read(os.path.join(inputs_dir, name))
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    got, rep = ias.spgemm(A)
    assert_csr_identical(got, ref, name)
    assert rep.flops == ob.flops(ob.Mat.of(A), ob.Mat.of(A))
    assert rep.nnz_c == ref.nnz


@pytest.mark.parametrize("name", ALL)
def test_csr_inputs_a_times_at(inputs_dir, name):
    A, _ = ias.mtx_read(os.path.join(inputs_dir, name))
    AT = transpose(A)
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(AT))
    got, _ = ias.spgemm(A, AT)
    assert_csr_identical(got, ref, name + " A*At")


@pytest.mark.parametrize("case", cases_small(), ids=lambda c: c[0])
def test_csr_synthetic(case):
    name, A, B = case
    B = A if B is None else B
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    got, rep = ias.spgemm(A, B)
    assert_csr_identical(got, ref, name)
    assert rep.flops == ob.flops(ob.Mat.of(A), ob.Mat.of(B))


def test_csr_long_rows_global_tables():
    A = long_rows()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    got, rep = ias.spgemm(A)
    assert rep.max_row_products > 21840 and rep.max_row_nnz > 5460
    assert_csr_identical(got, ref, "long rows")


def duplicate_tiers(seed=11):
    """A·B whose first rows hit every duplicate-handling path: each A row i
    takes m_i distinct rows of its own group of B, whose 100 columns are drawn
    from a pool sized for the wanted duplicate count (d ~ P^2 / 2 pool):
      P=1000 ~30 dups (one-wave fix-up), P=8000 ~500 (sorted fix-up, LDS bin),
      P=30000 ~1700 (partitioned row, streaming, 256-lane sorted fix-up),
      P=20000 ~4300 (partitioned row, streaming: list cap P/4), P=2000 ~500
      (LDS row beyond its list: direct-write table), P=30000 ~5300
      (partitioned, streaming, the 1024-lane sorted fix-up), P=20000 ~6200
      (partitioned row beyond its list: table path); then 2000 ordinary rows."""
    rng = np.random.default_rng(seed)
    per = 100
    plan = [(1000, 16000), (8000, 64000), (30000, 250000), (20000, 40000), (2000, 3333), (30000, 75000),
            (20000, 25000)]
    brows, arows = [], []
    ncols = 300000
    for prods, pool in plan:
        m = prods // per
        base = len(brows)
        for _ in range(m):
            brows.append(rng.choice(pool, per, replace=False))
        arows.append(np.arange(base, base + m))
    nb_special = len(brows)
    for _ in range(4000):
        brows.append(rng.choice(ncols, 12, replace=False))
    for _ in range(2000):
        arows.append(rng.choice(np.arange(nb_special, len(brows)), 8, replace=False))

    def csr(rows, ncol):
        rp = np.zeros(len(rows) + 1, np.int64)
        rp[1:] = np.cumsum([len(r) for r in rows])
        col = np.concatenate(rows).astype(np.int32)
        val = rng.uniform(-1.0, 1.0, size=col.size)
        return ias.HostCsr(len(rows), ncol, rp, col, val)

    return csr(arows, len(brows)), csr(brows, ncols)


def long_row_tiers(seed=5):
    """Rows for the one-wave / few-wave long-row symbolic kernels (sym4: 2,049 -
    4,096 products, sym5: 4,097 - 16,384), each with few duplicates, with a
    possible-duplicate list beyond the kernel's (handed to sym2's teams), and
    with more entries than sym4 stages (200 entries of 15 columns).  Each tier:
    (products, B-row length, column pool)."""
    rng = np.random.default_rng(seed)
    plan = [(3000, 100, 90000), (3000, 100, 5000), (3000, 15, 90000), (4000, 100, 2500),
            (6000, 100, 200000), (6000, 100, 9000), (8000, 100, 400000), (8000, 100, 6000),
            (12000, 100, 500000), (12000, 100, 20000), (16000, 100, 700000), (16000, 100, 12000)]
    brows, arows = [], []
    for prods, per, pool in plan:
        base = len(brows)
        for _ in range(prods // per):
            brows.append(rng.choice(pool, per, replace=False))
        arows.append(np.arange(base, len(brows)))
    nb = len(brows)
    for _ in range(3000):
        brows.append(rng.choice(50000, 20, replace=False))
    for _ in range(500):   # ordinary rows beside them (sym3 / short)
        arows.append(rng.choice(np.arange(nb, len(brows)), int(rng.integers(4, 60)), replace=False))

    def csr(rows, ncol):
        rp = np.zeros(len(rows) + 1, np.int64)
        rp[1:] = np.cumsum([len(r) for r in rows])
        col = np.concatenate(rows).astype(np.int32)
        val = rng.uniform(-1.0, 1.0, size=col.size)
        return ias.HostCsr(len(rows), ncol, rp, col, val)

    return csr(arows, len(brows)), csr(brows, 700000)


def test_csr_long_row_tiers():
    A, B = long_row_tiers()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    got, rep = ias.spgemm(A, B)
    assert rep.max_row_products == 16000
    assert_csr_identical(got, ref, "long-row tiers")


def test_csr_duplicate_tiers():
    A, B = duplicate_tiers()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    got, rep = ias.spgemm(A, B)
    assert rep.max_row_products == 30000
    assert_csr_identical(got, ref, "duplicate tiers")
    # the same product through COO (forward first-touch order, first product assigned)
    refc, ref_rows = ob.coo_mul_coo(ob.Mat.of(A), ob.Mat.of(B))
    ca, cb, cc = _coo_of(A), _coo_of(B), ias.Coo()
    o = ias.opts(output_memory=ias.MEMORY_HOST)
    ias.check(ias.lib.ias_coo_mul_coo(C.byref(ca), C.byref(cb), C.byref(cc), C.byref(o), None), "coo")
    n = cc.nnz
    got_c = ias._np(cc.col, n, np.int32)
    got_v = ias._np(cc.val, n, np.float64)
    for m in (ca, cb, cc):
        ias.lib.ias_coo_free(C.byref(m))
    np.testing.assert_array_equal(got_c, refc.col)
    np.testing.assert_array_equal(bits(got_v), bits(refc.val))


def test_csr_duplicate_tiers_hash_partitions():
    """The same tiers with B declared 1.2M columns wide: beyond one LDS column
    bitmap (k_sym_cbm), so the partitioned rows take the hash partitions."""
    A, B = duplicate_tiers()
    B = ias.HostCsr(B.rows, 1_200_000, B.row_ptr, B.col, B.val)
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    got, rep = ias.spgemm(A, B)
    assert rep.max_row_products == 30000
    assert_csr_identical(got, ref, "duplicate tiers, hash partitions")


def wide_row(n=1 << 20, head=1000, per=600):
    """Row 0 reaches head*per = 600k distinct columns: beyond the 19-bit rank
    field of the LDS/partition tables, so the 64-bit global-table path runs."""
    rp = np.zeros(n + 1, np.int64)
    lens = np.zeros(n, np.int64)
    lens[0] = head
    lens[1:head] = per
    rp[1:] = np.cumsum(lens)
    col = [np.arange(head)] + [np.arange(i * head, i * head + per) for i in range(1, head)]
    col = np.concatenate(col).astype(np.int32)
    val = ((np.arange(col.size) % 7) + 1).astype(np.float64)
    return ias.HostCsr(n, n, rp, col, val)


def heavy_collisions(n=4096, head=3000, per=10, seed=3):
    """Row 0: 30k products onto 10 columns (long ordered sums in one LDS slot);
    symbolic takes the hash-partition path (P > 5460), numeric the smallest bin."""
    rng = np.random.default_rng(seed)
    rp = np.zeros(n + 1, np.int64)
    lens = np.full(n, per, np.int64)
    lens[0] = head
    rp[1:] = np.cumsum(lens)
    col = np.concatenate([rng.choice(np.arange(1, n), head, replace=False)] +
                         [np.arange(per)] * (n - 1)).astype(np.int32)
    val = rng.uniform(-1, 1, col.size)
    return ias.HostCsr(n, n, rp, col, val)


def test_csr_wide_row_global_table():
    A = wide_row()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    got, rep = ias.spgemm(A)
    assert rep.max_row_nnz >= (1 << 19)
    assert_csr_identical(got, ref, "wide row")
    got_s, _ = ias.spgemm(A, order=ias.ORDER_SORTED)
    rc, rv = sorted_form(ref)
    np.testing.assert_array_equal(got_s.col, rc)
    np.testing.assert_array_equal(bits(got_s.val), bits(rv))


def test_csr_heavy_collisions_ordered_sums():
    A = heavy_collisions()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    got, rep = ias.spgemm(A)
    assert rep.max_row_products >= 30000
    assert_csr_identical(got, ref, "heavy collisions")


@pytest.mark.parametrize("case", cases_small()[:6], ids=lambda c: c[0])
def test_csr_sorted_order(case):
    name, A, _ = case
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    got, _ = ias.spgemm(A, order=ias.ORDER_SORTED)
    rc, rv = sorted_form(ref)
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
    np.testing.assert_array_equal(got.col, rc)
    np.testing.assert_array_equal(bits(got.val), bits(rv))


def test_csr_sorted_long_rows():
    A = long_rows()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    got, _ = ias.spgemm(A, order=ias.ORDER_SORTED)
    rc, rv = sorted_form(ref)
    np.testing.assert_array_equal(got.col, rc)
    np.testing.assert_array_equal(bits(got.val), bits(rv))


def test_csr_empty_and_zero_rows():
    A = ias.HostCsr(3, 4, np.zeros(4, np.int64), np.zeros(0, np.int32), np.zeros(0))
    B = ias.HostCsr(4, 2, np.zeros(5, np.int64), np.zeros(0, np.int32), np.zeros(0))
    got, rep = ias.spgemm(A, B)
    assert got.nnz == 0 and got.rows == 3 and got.cols == 2 and rep.flops == 0


def test_csr_dimension_mismatch():
    A = ias.gen_band(16, 1)
    B = ias.HostCsr(8, 8, np.zeros(9, np.int64), np.zeros(0, np.int32), np.zeros(0))
    with pytest.raises(ias.IasError) as e:
        ias.spgemm(A, B)
    assert e.value.status == 2


# ------------------------------------------------------------------ COO / ELL / DIA
def _coo_of(A):
    s = A.struct()
    c = ias.Coo()
    ias.check(ias.lib.ias_csr_to_coo(C.byref(s), C.byref(c), 0.0), "to_coo")
    return c


@pytest.mark.parametrize("case", cases_small(), ids=lambda c: c[0])
def test_coo_synthetic(case):
    name, A, _ = case
    ref, ref_rows = ob.coo_mul_coo(ob.Mat.of(A), ob.Mat.of(A))
    ca = _coo_of(A)
    cc = ias.Coo()
    o = ias.opts(output_memory=ias.MEMORY_HOST)
    ias.check(ias.lib.ias_coo_mul_coo(C.byref(ca), C.byref(ca), C.byref(cc), C.byref(o), None), "coo")
    n = cc.nnz
    got_rp = ias._np(cc.row_offset, cc.rows + 1, np.int64)
    got_r = ias._np(cc.row, n, np.int32)
    got_c = ias._np(cc.col, n, np.int32)
    got_v = ias._np(cc.val, n, np.float64)
    ias.lib.ias_coo_free(C.byref(ca))
    ias.lib.ias_coo_free(C.byref(cc))
    np.testing.assert_array_equal(got_rp, ref.row_ptr)
    np.testing.assert_array_equal(got_r, ref_rows)
    np.testing.assert_array_equal(got_c, ref.col)
    np.testing.assert_array_equal(bits(got_v), bits(ref.val))


@pytest.mark.parametrize("case", cases_small(), ids=lambda c: c[0])
def test_ell_synthetic(case):
    name, A, _ = case
    ref = ob.ell_mul_ell(ob.Mat.of(A), ob.Mat.of(A))
    s = A.struct()
    ea, ec = ias.Ell(), ias.Ell()
    ias.check(ias.lib.ias_csr_to_ell(C.byref(s), C.byref(ea), 0.0), "to_ell")
    o = ias.opts(output_memory=ias.MEMORY_HOST)
    ias.check(ias.lib.ias_ell_mul_ell(C.byref(ea), C.byref(ea), C.byref(ec), C.byref(o), None), "ell")
    K = ec.max_nnz_per_row
    assert K == ref["K"] and ec.nnz == ref["nnz"]
    got_n = ias._np(ec.nnz_row, ec.rows, np.int32)
    got_c = ias._np(ec.col, ec.rows * K, np.int32).reshape(ec.rows, K)
    got_v = ias._np(ec.val, ec.rows * K, np.float64).reshape(ec.rows, K)
    ias.lib.ias_ell_free(C.byref(ea))
    ias.lib.ias_ell_free(C.byref(ec))
    np.testing.assert_array_equal(got_n, ref["nnz_row"])
    np.testing.assert_array_equal(got_c, ref["col"])
    np.testing.assert_array_equal(bits(got_v), bits(ref["val"]))


def _sparse_band(n=3000, seed=4):
    """Non-contiguous diagonal set (offsets -40, -7, 0, 3, 11, 90) with a few
    holes on each diagonal: the offset -> slot maps have gaps."""
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        cols = [i + o for o in (-40, -7, 0, 3, 11, 90) if 0 <= i + o < n and rng.random() > 0.05]
        rows.append(np.array(sorted(cols), np.int64))
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    return ias.HostCsr(n, n, rp, col, rng.standard_normal(col.size))


DIA_CASES = [("band4k", lambda: ias.gen_band(4096, 3, seed=7)),
             ("band_w1", lambda: ias.gen_band(1000, 1, seed=3, value_mode=1)),
             ("band_wide65", lambda: ias.gen_band(5000, 32, seed=5)),
             ("band_sparse_offsets", _sparse_band),
             ("dia.mtx", None), ("small.mtx", None), ("b1_ss.mtx", None)]


def _dia_run(A, mfma, monkeypatch):
    monkeypatch.setenv("IAS_DIA_MFMA", "1" if mfma else "0")
    s = A.struct()
    da, dc = ias.Dia(), ias.Dia()
    ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(da), 0.0), "to_dia")
    o = ias.opts(output_memory=ias.MEMORY_HOST)
    ias.check(ias.lib.ias_dia_mul_dia(C.byref(da), C.byref(da), C.byref(dc), C.byref(o), None), "dia")
    nd = dc.num_diagonals
    out = dict(nd=nd, offsets=ias._np(dc.diagonal_offsets, nd, np.int32).copy(),
               ind=ias._np(dc.diagonal_ind, dc.rows + dc.cols - 1, np.int32).copy(),
               val=ias._np(dc.val, dc.rows * nd, np.float64).reshape(dc.rows, nd).copy())
    ias.lib.ias_dia_free(C.byref(da))
    ias.lib.ias_dia_free(C.byref(dc))
    return out


@pytest.mark.parametrize("case", DIA_CASES, ids=lambda c: c[0])
def test_dia(case, inputs_dir, monkeypatch):
    """The LDS-tiled kernel (default): bitwise the reference's DIA_mul_DIA."""
    name, mk = case
    A = mk() if mk else ias.mtx_read(os.path.join(inputs_dir, name))[0]
    ref = ob.dia_mul_dia(ob.Mat.of(A), ob.Mat.of(A))
    got = _dia_run(A, False, monkeypatch)
    assert got["nd"] == ref["nd"]
    np.testing.assert_array_equal(got["offsets"], ref["offsets"])
    np.testing.assert_array_equal(got["ind"], ref["ind"])
    np.testing.assert_array_equal(bits(got["val"]), bits(ref["val"]))


@pytest.mark.parametrize("case", DIA_CASES, ids=lambda c: c[0])
def test_dia_mfma(case, inputs_dir, monkeypatch):
    """The MFMA form (IAS_DIA_MFMA=1, fused sums in the matrix core's order):
    same diagonal set, values within the north-star tolerance
    |dC| <= 1e-10 * max(|c|, sum |a*b|)."""
    name, mk = case
    A = mk() if mk else ias.mtx_read(os.path.join(inputs_dir, name))[0]
    ref = ob.dia_mul_dia(ob.Mat.of(A), ob.Mat.of(A))
    absA = ias.HostCsr(A.rows, A.cols, A.row_ptr, A.col, np.abs(A.val))
    bound = ob.dia_mul_dia(ob.Mat.of(absA), ob.Mat.of(absA))["val"]
    got = _dia_run(A, True, monkeypatch)
    assert got["nd"] == ref["nd"]
    np.testing.assert_array_equal(got["offsets"], ref["offsets"])
    tol = 1e-10 * np.maximum(np.abs(ref["val"]), bound) + 1e-300
    assert np.all(np.abs(got["val"] - ref["val"]) <= tol)


# ------------------------------------------------------------------ device-side conversions (f3)
def _dup_matrix():
    """Rows with repeated columns (later duplicate wins in CSRtoDIA) and empty rows."""
    rp = np.array([0, 3, 3, 6, 6, 8], np.int64)
    col = np.array([1, 1, 4, 0, 2, 0, 3, 3], np.int32)
    val = np.array([1.5, -2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0])
    return ias.HostCsr(5, 6, rp, col, val)


CONV_CASES = [("dia.mtx", None), ("small.mtx", None),
              ("band", lambda: ias.gen_band(3000, 4, seed=5)),
              ("rmat12", lambda: ias.gen_rmat(12, 8, seed=3)),
              ("dups", _dup_matrix),
              ("empty", lambda: ias.HostCsr(7, 9, np.zeros(8, np.int64), np.zeros(0, np.int32), np.zeros(0)))]

_CONV = {"coo": (ias.Coo, "ias_csr_to_coo", "ias_coo_copy", "ias_coo_free"),
         "ell": (ias.Ell, "ias_csr_to_ell", "ias_ell_copy", "ias_ell_free"),
         "dia": (ias.Dia, "ias_csr_to_dia", "ias_dia_copy", "ias_dia_free")}


def _conv_arrays(kind, m):
    """All arrays of a host-resident converted matrix, as numpy."""
    if kind == "coo":
        n = m.nnz
        return dict(rp=ias._np(m.row_offset, m.rows + 1, np.int64), r=ias._np(m.row, n, np.int32),
                    c=ias._np(m.col, n, np.int32), v=bits(ias._np(m.val, n, np.float64)))
    if kind == "ell":
        rk = m.rows * m.max_nnz_per_row
        return dict(K=m.max_nnz_per_row, n=ias._np(m.nnz_row, m.rows, np.int32),
                    c=ias._np(m.col, rk, np.int32), v=bits(ias._np(m.val, rk, np.float64)))
    nd = m.num_diagonals
    return dict(nd=nd, off=ias._np(m.diagonal_offsets, nd, np.int32),
                ind=ias._np(m.diagonal_ind, max(m.rows + m.cols - 1, 0), np.int32),
                v=bits(ias._np(m.val, m.rows * nd, np.float64)))


def _convert(kind, src, gate=0.0):
    T, conv, copy, free = _CONV[kind]
    out = T()
    st = getattr(ias.lib, conv)(C.byref(src), C.byref(out), gate)
    if st != 0:
        return st, None, (out.rows, out.cols, out.choice)
    if out.memory == ias.MEMORY_DEVICE:
        h = T()
        ias.check(getattr(ias.lib, copy)(C.byref(out), C.byref(h), ias.MEMORY_HOST, 0), "copy back")
        getattr(ias.lib, free)(C.byref(out))
        out = h
    arrays = _conv_arrays(kind, out)
    meta = (out.rows, out.cols, out.choice)
    getattr(ias.lib, free)(C.byref(out))
    return st, arrays, meta


@pytest.mark.parametrize("kind", ["coo", "ell", "dia"])
@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: c[0])
def test_device_conversions(case, kind, inputs_dir):
    """CSRtoCOO/ELL/DIA of a device CSR (convert_dev.hip) == the host conversion, byte for byte,
    for the whole matrix and for a row view (row_ptr[0] != 0)."""
    name, mk = case
    A = mk() if mk else ias.mtx_read(os.path.join(inputs_dir, name))[0]
    hs = A.struct()
    dA = ias.Csr()
    ias.check(ias.lib.ias_csr_copy(C.byref(hs), C.byref(dA), ias.MEMORY_DEVICE, 0), "copy")
    try:
        lo, hi = (A.rows // 3, A.rows - A.rows // 4) if A.rows > 2 else (0, A.rows)
        hv, dv = ias.Csr(), ias.Csr()
        ias.check(ias.lib.ias_csr_row_view(C.byref(hs), lo, hi, C.byref(hv)), "view")
        ias.check(ias.lib.ias_csr_row_view(C.byref(dA), lo, hi, C.byref(dv)), "view")
        for host_src, dev_src in ((hs, dA), (hv, dv)):
            sh, want, mh = _convert(kind, host_src)
            sd, got, md = _convert(kind, dev_src)
            assert sh == sd == 0 and mh == md, (name, kind, sh, sd, mh, md)
            for k in want:
                np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(want[k]), err_msg=f"{name} {kind} {k}")
        # the size gate (coo/ell/dia common headers): same verdict both sides
        for gate in (0.5, 1.0, 4.0):
            sh, _, mh = _convert(kind, hs, gate)
            sd, _, md = _convert(kind, dA, gate)
            assert sh == sd and mh[2] == md[2], (name, kind, gate, sh, sd)
    finally:
        ias.lib.ias_csr_free(C.byref(dA))


@pytest.mark.parametrize("case", CONV_CASES + [("rect", lambda: ias.HostCsr(
    3, 70000, np.array([0, 2, 2, 5], np.int64), np.array([69999, 5, 5, 0, 69999], np.int32),
    np.array([1.0, 2.0, 3.0, 4.0, 5.0])))], ids=lambda c: c[0])
def test_device_transpose(case, inputs_dir):
    """Aᵀ of a device CSR (stable radix sort, convert_dev.hip) == the host counting sort, byte for byte."""
    name, mk = case
    A = mk() if mk else ias.mtx_read(os.path.join(inputs_dir, name))[0]
    hs = A.struct()
    dA = ias.Csr()
    ias.check(ias.lib.ias_csr_copy(C.byref(hs), C.byref(dA), ias.MEMORY_DEVICE, 0), "copy")
    try:
        lo, hi = (A.rows // 3, A.rows) if A.rows > 2 else (0, A.rows)
        hv, dv = ias.Csr(), ias.Csr()
        ias.check(ias.lib.ias_csr_row_view(C.byref(hs), lo, hi, C.byref(hv)), "view")
        ias.check(ias.lib.ias_csr_row_view(C.byref(dA), lo, hi, C.byref(dv)), "view")
        for host_src, dev_src in ((hs, dA), (hv, dv)):
            th, td = ias.Csr(), ias.Csr()
            ias.check(ias.lib.ias_csr_transpose(C.byref(host_src), C.byref(th)), "host T")
            ias.check(ias.lib.ias_csr_transpose(C.byref(dev_src), C.byref(td)), "device T")
            assert td.memory == ias.MEMORY_DEVICE
            want, got = ias.csr_to_numpy(th), ias.csr_to_numpy(td)
            assert (got.rows, got.cols) == (want.rows, want.cols)
            np.testing.assert_array_equal(got.row_ptr, want.row_ptr, err_msg=name)
            np.testing.assert_array_equal(got.col, want.col, err_msg=name)
            np.testing.assert_array_equal(bits(got.val), bits(want.val), err_msg=name)
    finally:
        ias.lib.ias_csr_free(C.byref(dA))


# ------------------------------------------------------------------ device-resident two-phase
def test_two_phase_device_resident():
    A = ias.gen_rmat(14, 16, seed=4)
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    hs = A.struct()
    dA = ias.Csr()
    ias.check(ias.lib.ias_csr_copy(C.byref(hs), C.byref(dA), ias.MEMORY_DEVICE, 0), "copy")
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
    try:
        for _ in range(3):   # plan reuse across calls
            nnz = C.c_int64(0)
            ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(dA), C.byref(dA), C.byref(nnz), None, None), "nnz")
            assert nnz.value == ref.nnz
            dC = ias.Csr()
            ias.check(ias.lib.ias_csr_alloc(C.byref(dC), A.rows, A.cols, nnz.value, ias.MEMORY_DEVICE, 0), "alloc")
            ias.check(ias.lib.ias_csr_mul_csr_compute(plan, C.byref(dA), C.byref(dA), C.byref(dC),
                                                      ias.ORDER_REFERENCE, None), "compute")
            got = ias.csr_to_numpy(dC)
            assert_csr_identical(got, ref, "two-phase")
    finally:
        ias.lib.ias_plan_destroy(plan)
        ias.lib.ias_csr_free(C.byref(dA))


def test_row_views_concatenate():
    """Row-block shards (the multi-GPU unit) concatenate to the 1-GPU result."""
    A = ias.gen_rmat(13, 16, seed=9)
    full, _ = ias.spgemm(A)
    bounds = (C.c_int64 * 5)()
    sa = A.struct()
    ias.check(ias.lib.ias_partition_rows(C.byref(sa), C.byref(sa), 4, bounds), "partition")
    cols, vals, lens = [], [], []
    for k in range(4):
        v = ias.Csr()
        ias.check(ias.lib.ias_csr_row_view(C.byref(sa), bounds[k], bounds[k + 1], C.byref(v)), "view")
        c, o = ias.Csr(), ias.opts(output_memory=ias.MEMORY_HOST, device=0)
        ias.check(ias.lib.ias_csr_mul_csr(C.byref(v), C.byref(sa), C.byref(c), C.byref(o), None), "shard")
        part = ias.csr_to_numpy(c)
        cols.append(part.col); vals.append(part.val); lens.append(np.diff(part.row_ptr))
    np.testing.assert_array_equal(np.concatenate(lens), np.diff(full.row_ptr))
    np.testing.assert_array_equal(np.concatenate(cols), full.col)
    np.testing.assert_array_equal(bits(np.concatenate(vals)), bits(full.val))


# ------------------------------------------------------------------ MKL cross-check
def test_against_mkl_tolerance():
    ok, _ = ias.mkl_available()
    if not ok:
        pytest.skip("MKL runtime not present on this box")
    A = ias.gen_rmat(14, 16, seed=2)
    got, _ = ias.spgemm(A, order=ias.ORDER_SORTED)
    mk, _ = ias.mkl_sp2m(A, A)
    mc, mv = sorted_form(mk)
    np.testing.assert_array_equal(got.row_ptr, mk.row_ptr)
    np.testing.assert_array_equal(got.col, mc)
    # |dC| <= 1e-10 * sum |a||b| (absolute products) per entry
    absA = ias.HostCsr(A.rows, A.cols, A.row_ptr, A.col, np.abs(A.val))
    bound, _ = ias.spgemm(absA, order=ias.ORDER_SORTED)
    assert np.all(np.abs(got.val - mv) <= 1e-10 * np.maximum(np.abs(mv), bound.val) + 1e-300)


# ------------------------------------------------------------------ single pass (ias_csr_mul_csr_into)
def _dev(A):
    hs = A.struct()
    d = ias.Csr()
    ias.check(ias.lib.ias_csr_copy(C.byref(hs), C.byref(d), ias.MEMORY_DEVICE, 0), "copy")
    return d


def _into(plan, dA, dB, rows, cols, cap, order=ias.ORDER_REFERENCE):
    dC = ias.Csr()
    ias.check(ias.lib.ias_csr_alloc(C.byref(dC), rows, cols, cap, ias.MEMORY_DEVICE, 0), "alloc")
    st = ias.lib.ias_csr_mul_csr_into(plan, C.byref(dA), C.byref(dB), C.byref(dC), order, None)
    return st, dC


def chunk_edges(seed=21):
    """Rows that stress the chunking of the single pass: > OP_RMAX consecutive
    empty rows, rows of exactly OP_BIG (2048) and OP_BIG + 1 products, rows of
    1 product, rows whose product prefix straddles chunk windows, a band block
    (3-4x compression: most products are duplicates) and an R-MAT block."""
    rng = np.random.default_rng(seed)
    n = 20000
    rows = [[] for _ in range(n)]
    blen = 16
    # rows 0..1499 empty (beyond OP_RMAX consecutive)
    for i in range(1500, 1600):             # exactly 2048 products: 128 entries x 16
        rows[i] = list(rng.choice(np.arange(12000, n), 128, replace=False))
    for i in range(1600, 1610):             # 2048 + 16 products: big row path
        rows[i] = list(rng.choice(np.arange(12000, n), 129, replace=False))
    for i in range(1610, 1615):             # 6400 products: big row path
        rows[i] = list(rng.choice(np.arange(12000, n), 400, replace=False))
    for i in range(1615, 3000):             # 1 entry: 16 products
        rows[i] = [int(rng.integers(12000, n))]
    for i in range(3000, 12000):            # band: entries i-3..i+3 -> heavy duplicates
        rows[i] = [j for j in range(i - 3, i + 4)]
    for i in range(12000, n):               # 16 random entries (B rows of A = B)
        rows[i] = list(rng.choice(n, blen, replace=False))
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate([np.asarray(r, np.int64) for r in rows]).astype(np.int32)
    val = rng.integers(-4, 5, size=col.size).astype(np.float64) + 0.5
    return ias.HostCsr(n, n, rp, col, val)


@pytest.mark.parametrize("which", ["rmat14", "edges", "dups", "long"])
def test_into_single_call(which):
    A = {"rmat14": lambda: ias.gen_rmat(14, 16, seed=4), "edges": chunk_edges,
         "dups": lambda: duplicate_tiers()[0], "long": long_rows}[which]()
    B = duplicate_tiers()[1] if which == "dups" else A
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    fl = ob.flops(ob.Mat.of(A), ob.Mat.of(B))
    dA, dB = _dev(A), _dev(B)
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
    try:
        for _ in range(2):   # plan reuse
            st, dC = _into(plan, dA, dB, A.rows, B.cols, max(fl, 1))
            ias.check(st, "into")
            assert dC.nnz == ref.nnz
            assert_csr_identical(ias.csr_to_numpy(dC), ref, "into " + which)
        st, dC = _into(plan, dA, dB, A.rows, B.cols, max(fl, 1), ias.ORDER_SORTED)
        ias.check(st, "into sorted")
        got = ias.csr_to_numpy(dC)
        rc, rv = sorted_form(ref)
        np.testing.assert_array_equal(got.col, rc)
        np.testing.assert_array_equal(bits(got.val), bits(rv))
        # too little capacity: row pointer complete, needed nnz reported, nothing written beyond
        if ref.nnz > 1:
            st, dC = _into(plan, dA, dB, A.rows, B.cols, ref.nnz - 1)
            assert st == 11 and dC.nnz == ref.nnz
            ias.check(ias.lib.ias_csr_free(C.byref(dC)), "free")
    finally:
        ias.lib.ias_plan_destroy(plan)
        ias.lib.ias_csr_free(C.byref(dA))
        ias.lib.ias_csr_free(C.byref(dB))


def test_chunk_edges_all_paths():
    A = chunk_edges()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
    got, rep = ias.spgemm(A)
    assert_csr_identical(got, ref, "chunk edges")
    refc, _ = ob.coo_mul_coo(ob.Mat.of(A), ob.Mat.of(A))
    ca, cc = _coo_of(A), ias.Coo()
    o = ias.opts(output_memory=ias.MEMORY_HOST)
    ias.check(ias.lib.ias_coo_mul_coo(C.byref(ca), C.byref(ca), C.byref(cc), C.byref(o), None), "coo")
    n = cc.nnz
    np.testing.assert_array_equal(ias._np(cc.col, n, np.int32), refc.col)
    np.testing.assert_array_equal(bits(ias._np(cc.val, n, np.float64)), bits(refc.val))
    for m in (ca, cc):
        ias.lib.ias_coo_free(C.byref(m))


def test_host_operand_transfer_times():
    """Host operands: the report carries the PCIe staging times (ias.h ms_upload / ms_download)."""
    A = ias.gen_rmat(12, 8, seed=5)
    _, rep = ias.spgemm(A)
    assert rep.ms_upload > 0 and rep.ms_download > 0 and rep.ms_total > 0
    hs = A.struct()
    dA = ias.Csr()
    ias.check(ias.lib.ias_csr_copy(C.byref(hs), C.byref(dA), ias.MEMORY_DEVICE, 0), "copy")
    try:
        c, r2 = ias.Csr(), ias.Report()
        o = ias.opts(output_memory=ias.MEMORY_DEVICE, device=0)
        ias.check(ias.lib.ias_csr_mul_csr(C.byref(dA), C.byref(dA), C.byref(c), C.byref(o), C.byref(r2)), "dev")
        assert r2.ms_upload == 0 and r2.ms_download == 0
        ias.lib.ias_csr_free(C.byref(c))
    finally:
        ias.lib.ias_csr_free(C.byref(dA))


# ------------------------------------------------------------------ sorted order, wide rows
def many_wide_rows(rows=40000, n=40000, nwide=60, mmax=230, seed=9):
    """A*B with `nwide` rows of A whose C rows hold ~2000-20000 entries
    (radix-sort segments of different sizes with short rows between them);
    B rows ~100 entries, the other A rows 0-3 entries."""
    rng = np.random.default_rng(seed)
    wide = set(rng.choice(rows, nwide, replace=False).tolist())
    arows = []
    for i in range(rows):
        m = int(rng.integers(22, mmax)) if i in wide else int(rng.integers(0, 4))
        arows.append(np.sort(rng.choice(n, m, replace=False)))
    brows = [np.sort(rng.choice(n, int(rng.integers(80, 120)), replace=False)) for _ in range(n)]

    def mk(rs):
        rp = np.zeros(len(rs) + 1, np.int64)
        rp[1:] = np.cumsum([len(r) for r in rs])
        col = np.concatenate(rs).astype(np.int32)
        val = rng.standard_normal(col.size)
        return ias.HostCsr(len(rs), n, rp, col, val)

    return mk(arows), mk(brows)


def _wide_rows_ref():
    A, B = many_wide_rows()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    nnz_row = np.diff(ref.row_ptr)
    assert ((nnz_row > 2048) & (nnz_row <= 20000)).sum() >= 40 and nnz_row.max() > 8192
    return A, B, ref


@pytest.mark.parametrize("force_global", ["0", "1"])
def test_sorted_wide_rows_csr(force_global, monkeypatch):
    """Rows past the LDS sort bins: the segmented radix sort (default) and
    the per-row bitonic workspace (IAS_SORT_GLOBAL=1)."""
    monkeypatch.setenv("IAS_SORT_GLOBAL", force_global)
    A, B, ref = _wide_rows_ref()
    got, _ = ias.spgemm(A, B, order=ias.ORDER_SORTED)
    rc, rv = sorted_form(ref)
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
    np.testing.assert_array_equal(got.col, rc)
    np.testing.assert_array_equal(bits(got.val), bits(rv))


@pytest.mark.parametrize("force_global", ["0", "1"])
def test_sorted_wide_rows_coo(force_global, monkeypatch):
    monkeypatch.setenv("IAS_SORT_GLOBAL", force_global)
    A, B = many_wide_rows()
    ref, ref_rows = ob.coo_mul_coo(ob.Mat.of(A), ob.Mat.of(B))
    ca, cb, cc = _coo_of(A), _coo_of(B), ias.Coo()
    o = ias.opts(order=ias.ORDER_SORTED, output_memory=ias.MEMORY_HOST)
    ias.check(ias.lib.ias_coo_mul_coo(C.byref(ca), C.byref(cb), C.byref(cc), C.byref(o), None), "coo")
    n = cc.nnz
    got_r = ias._np(cc.row, n, np.int32)
    got_c = ias._np(cc.col, n, np.int32)
    got_v = ias._np(cc.val, n, np.float64)
    for m in (ca, cb, cc):
        ias.lib.ias_coo_free(C.byref(m))
    rc, rv = sorted_form(ref)
    np.testing.assert_array_equal(got_r, ref_rows)
    np.testing.assert_array_equal(got_c, rc)
    np.testing.assert_array_equal(bits(got_v), bits(rv))


@pytest.mark.parametrize("force_global", ["0", "1"])
def test_sorted_wide_rows_ell(force_global, monkeypatch):
    """ELL output: the sort spans (row * K, nnz_row) instead of row pointers."""
    monkeypatch.setenv("IAS_SORT_GLOBAL", force_global)
    A, B = many_wide_rows(rows=1000, n=30000, nwide=40, mmax=130)   # C: 1000 x K<=13000 padded
    ref = ob.ell_mul_ell(ob.Mat.of(A), ob.Mat.of(B))
    assert (ref["nnz_row"] > 2048).sum() >= 25
    sa, sb = A.struct(), B.struct()
    ea, eb, ec = ias.Ell(), ias.Ell(), ias.Ell()
    ias.check(ias.lib.ias_csr_to_ell(C.byref(sa), C.byref(ea), 0.0), "to_ell")
    ias.check(ias.lib.ias_csr_to_ell(C.byref(sb), C.byref(eb), 0.0), "to_ell")
    o = ias.opts(order=ias.ORDER_SORTED, output_memory=ias.MEMORY_HOST)
    ias.check(ias.lib.ias_ell_mul_ell(C.byref(ea), C.byref(eb), C.byref(ec), C.byref(o), None), "ell")
    K = ec.max_nnz_per_row
    assert K == ref["K"]
    got_n = ias._np(ec.nnz_row, ec.rows, np.int32)
    got_c = ias._np(ec.col, ec.rows * K, np.int32).reshape(ec.rows, K)
    got_v = ias._np(ec.val, ec.rows * K, np.float64).reshape(ec.rows, K)
    for m in (ea, eb, ec):
        ias.lib.ias_ell_free(C.byref(m))
    np.testing.assert_array_equal(got_n, ref["nnz_row"])
    for i in np.nonzero(got_n)[0]:
        k = got_n[i]
        o_ = np.argsort(ref["col"][i, :k], kind="stable")
        np.testing.assert_array_equal(got_c[i, :k], ref["col"][i, :k][o_], err_msg=f"row {i}")
        np.testing.assert_array_equal(bits(got_v[i, :k]), bits(ref["val"][i, :k][o_]), err_msg=f"row {i}")
