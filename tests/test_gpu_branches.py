"""Targeted GPU tests of branches the full-size inputs do not reach (or reach
without an entry-by-entry check), each bitwise against the oracle's
CSR_MUL_CSR restatement (IA-SPGEMM-CPU_release/detail/csr/common_csr.h:85-193):

  * the column-bitmap symbolic (k_sym_cbm) of rows beyond 16,384 products:
    every branch — minima table in LDS or in the row's work space, duplicates
    found from the list or by a sweep, kept for the fix-ups or left to the
    table path, first-touch words in LDS or in global memory — natural and
    forced (IAS_CBM_FORCE), asserted reached through ias_last_diag();
  * the LDS bucket sort (IAS_ORDER_SORTED) on rows whose columns cluster with
    far outliers (most keys in a few buckets: the bitonic-keys fallback);
  * ias_dia_mul_dia_into refusing a C that shares memory with an operand, and
    ias_dia_mul_dia_ndiag refusing invalid operands;
  * the block cache of library-allocated device outputs under several host
    threads allocating and freeing at once;
  * rows of 16,385 .. 32,768 products when B is too wide for the column
    bitmap (k_sym5<32768>, 8 waves, dynamic LDS) and their fall-back through
    global-memory tables (k_sym_gtab: list overflows, > 1,024 entries, and
    every row of the bins when forced with IAS_GTAB_ALL=1, the branch taken
    when B's entries exceed 32-bit offsets);
  * sym2's retry teams sized from the plan's previous call (rows the sym3 /
    sym4 / sym5 bins handed back then): a plan whose last call had no retries
    meets a product whose rows all overflow their lists, and the reverse;
  * B rows selected beyond 2^29 and 2^30 entries (a padded B): the streaming
    numeric pass with 64-bit gather addresses, and the symbolic bins that
    take over from the 32-bit-offset ones; the 64-bit pass forced on an
    ordinary input (IAS_WIDE_V=1).
"""
import ctypes as C
import threading

import numpy as np
import pytest

import ias
import oracle_bind as ob

pytestmark = pytest.mark.gpu

GLOBAL_OWN, UNLISTED_KEEP, UNLISTED_DROP, GLOBAL_WORDS, LISTED_KEEP, LISTED_DROP, LDS_OWN = 1, 2, 4, 8, 16, 32, 64


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


def _csr(rows, ncol, rng):
    rp = np.zeros(len(rows) + 1, np.int64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.uniform(-1.0, 1.0, size=col.size)
    return ias.HostCsr(len(rows), ncol, rp, col, val)


def cbm_rows(seed=17):
    """A*B with B 2^20 columns wide (one LDS column bitmap, 3,968 LDS minima
    slots beside it) whose first A rows exceed 16,384 products (k_sym_cbm):
    each takes `prods` products from B rows of 100 columns drawn from a pool
    of `pool` columns — (P, pool):
      (60000, 200000) ~7.4k repeated columns > 3,968: global minima, ~8k
                      duplicates <= P/4: listed, kept;
      (40000,  40000) global minima, ~15k duplicates > P/4: listed, dropped;
      (40000,   5000) global minima, 35k duplicates: unlisted, dropped;
      (30000, 250000) few repeated columns: LDS minima, listed, kept;
      (20000,   1000) LDS minima, 19k duplicates: unlisted, dropped;
    then 1,500 ordinary rows."""
    rng = np.random.default_rng(seed)
    per = 100
    brows, arows = [], []
    for prods, pool in [(60000, 200000), (40000, 40000), (40000, 5000), (30000, 250000), (20000, 1000)]:
        base = len(brows)
        for _ in range(prods // per):
            brows.append(rng.choice(pool, per, replace=False))
        arows.append(np.arange(base, len(brows)))
    nb = len(brows)
    for _ in range(3000):
        brows.append(rng.choice(1 << 20, 12, replace=False))
    for _ in range(1500):
        arows.append(rng.choice(np.arange(nb, len(brows)), 8, replace=False))
    return _csr(arows, len(brows), rng), _csr(brows, 1 << 20, rng)


@pytest.fixture(scope="module")
def cbm_case():
    A, B = cbm_rows()
    return A, B, ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))


# (IAS_CBM_FORCE, branches that must have run)
FORCED = [
    (0, GLOBAL_OWN | LDS_OWN | LISTED_KEEP | LISTED_DROP | UNLISTED_DROP),
    (1, GLOBAL_OWN | LISTED_KEEP | LISTED_DROP | UNLISTED_DROP),          # every row's minima in global memory
    (2, GLOBAL_OWN | LDS_OWN | UNLISTED_KEEP | UNLISTED_DROP | GLOBAL_WORDS),   # no list: sweeps
    (4, GLOBAL_WORDS | LISTED_KEEP | LISTED_DROP),                        # listed rows' words in global memory
    (3, GLOBAL_OWN | UNLISTED_KEEP | UNLISTED_DROP | GLOBAL_WORDS),
    (5, GLOBAL_OWN | GLOBAL_WORDS | LISTED_KEEP | LISTED_DROP),
    (7, GLOBAL_OWN | UNLISTED_KEEP | UNLISTED_DROP | GLOBAL_WORDS),
]


@pytest.mark.parametrize("force,want", FORCED, ids=[f"force{f}" for f, _ in FORCED])
def test_cbm_branches(cbm_case, monkeypatch, force, want):
    A, B, ref = cbm_case
    monkeypatch.setenv("IAS_CBM_FORCE", str(force))
    got, rep = ias.spgemm(A, B)
    hits = int(ias.lib.ias_last_diag())
    assert rep.max_row_products == 60000
    assert_csr_identical(got, ref, f"column-bitmap symbolic, IAS_CBM_FORCE={force}")
    assert hits & want == want, f"branches reached {hits:#x}, wanted {want:#x}"
    if force & 1:
        assert not hits & LDS_OWN
    if force & 2:
        assert not hits & (LISTED_KEEP | LISTED_DROP)
    # and the same product in sorted order (rows of the bitmap path sorted after)
    if force == 7:
        got_s, _ = ias.spgemm(A, B, order=ias.ORDER_SORTED)
        for i in range(5):
            s, e = ref.row_ptr[i], ref.row_ptr[i + 1]
            o = np.argsort(ref.col[s:e], kind="stable")
            np.testing.assert_array_equal(got_s.col[s:e], ref.col[s:e][o])
            np.testing.assert_array_equal(bits(got_s.val[s:e]), bits(ref.val[s:e][o]))


def test_cbm_diag_off_without_knob(cbm_case, monkeypatch):
    A, B, ref = cbm_case
    monkeypatch.delenv("IAS_CBM_FORCE", raising=False)
    got, _ = ias.spgemm(A, B)
    assert_csr_identical(got, ref, "column-bitmap symbolic")
    assert ias.lib.ias_last_diag() == 0


def skewed_rows(seed=23):
    """C rows whose columns cluster with far outliers, for every bucket-sort
    team size (rows of ~100 .. ~8,000 entries): A row i takes m_i B rows whose
    columns lie in [0, 4000) except one column near 2^20 - 1 (the long rows put
    hundreds of keys in each of a few buckets)."""
    rng = np.random.default_rng(seed)
    brows = [np.concatenate([rng.choice(4000, 15, replace=False), [(1 << 20) - 1 - i]]) for i in range(3000)]
    arows = [rng.choice(3000, m, replace=False) for m in (8, 30, 60, 120, 250, 500, 1000, 2000)]
    arows += [rng.choice(3000, 10, replace=False) for _ in range(200)]
    return _csr(arows, 3000, rng), _csr(brows, 1 << 20, rng)


def test_sort_skewed_buckets():
    A, B = skewed_rows()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    got, _ = ias.spgemm(A, B, order=ias.ORDER_SORTED)
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
    assert int(np.diff(ref.row_ptr).max()) > 4096
    for i in range(A.rows):
        s, e = ref.row_ptr[i], ref.row_ptr[i + 1]
        o = np.argsort(ref.col[s:e], kind="stable")
        np.testing.assert_array_equal(got.col[s:e], ref.col[s:e][o], err_msg=f"row {i}")
        np.testing.assert_array_equal(bits(got.val[s:e]), bits(ref.val[s:e][o]), err_msg=f"row {i}")


def _device_dia(A):
    s = A.struct()
    ha, da = ias.Dia(), ias.Dia()
    ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(ha), 0.0), "to_dia")
    ias.check(ias.lib.ias_dia_copy(C.byref(ha), C.byref(da), ias.MEMORY_DEVICE, 0), "upload")
    ias.lib.ias_dia_free(C.byref(ha))
    return da


def test_dia_into_rejects_aliased_c():
    A = ias.gen_band(2048, 2, seed=3)
    da = _device_dia(A)
    try:
        nd = C.c_int32(0)
        ias.check(ias.lib.ias_dia_mul_dia_ndiag(C.byref(da), C.byref(da), C.byref(nd)), "ndiag")
        assert nd.value == 9
        # C = A in place: every array of C is one of A's
        Ca = ias.Dia(rows=0, cols=0, num_diagonals=da.num_diagonals, choice=0,
                     diagonal_offsets=da.diagonal_offsets, diagonal_ind=da.diagonal_ind, val=da.val,
                     memory=ias.MEMORY_DEVICE, device=0)
        assert ias.lib.ias_dia_mul_dia_into(C.byref(da), C.byref(da), C.byref(Ca), None, None) == 1
        assert b"overlap" in ias.lib.ias_last_error()
        # only the values overlap (C.val inside A's value array)
        import torch
        offs = torch.empty(nd.value, dtype=torch.int32, device="cuda:0")
        ind = torch.empty(2 * 2048 - 1, dtype=torch.int32, device="cuda:0")
        Cb = ias.Dia(rows=0, cols=0, num_diagonals=nd.value, choice=0,
                     diagonal_offsets=C.cast(C.c_void_p(offs.data_ptr()), ias.i32p),
                     diagonal_ind=C.cast(C.c_void_p(ind.data_ptr()), ias.i32p),
                     val=C.cast(C.c_void_p(C.cast(da.val, C.c_void_p).value + 8 * 100), ias.f64p),
                     memory=ias.MEMORY_DEVICE, device=0)
        assert ias.lib.ias_dia_mul_dia_into(C.byref(da), C.byref(da), C.byref(Cb), None, None) == 1
        # invalid operands of the ndiag query
        bad = ias.Dia(rows=da.rows, cols=da.cols, num_diagonals=-1, choice=1, diagonal_offsets=da.diagonal_offsets,
                      diagonal_ind=da.diagonal_ind, val=da.val, memory=ias.MEMORY_DEVICE, device=0)
        assert ias.lib.ias_dia_mul_dia_ndiag(C.byref(bad), C.byref(da), C.byref(nd)) == 1
        bad.num_diagonals, bad.choice = da.num_diagonals, 0
        assert ias.lib.ias_dia_mul_dia_ndiag(C.byref(bad), C.byref(da), C.byref(nd)) == 8
    finally:
        ias.lib.ias_dia_free(C.byref(da))


def test_block_cache_concurrent_threads():
    """Four host threads, each with its own plan, multiply and free
    library-allocated device outputs (block-cache sized) at once; every result
    matches the oracle's nnz and value sum, so no thread got a block another
    thread's kernels were still writing."""
    mats = [ias.gen_rmat(12, 8, seed=s, value_mode=1) for s in (31, 32, 33, 34)]
    refs = []
    for A in mats:
        r = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
        refs.append((r.nnz, float(r.val.sum())))
    errors = []

    def work(k):
        try:
            A = mats[k]
            plan = C.c_void_p()
            ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
            s = A.struct()
            o = ias.opts(output_memory=ias.MEMORY_DEVICE, device=0, plan=plan)
            for it in range(25):
                c = ias.Csr()
                ias.check(ias.lib.ias_csr_mul_csr(C.byref(s), C.byref(s), C.byref(c), C.byref(o), None), "mul")
                h = ias.Csr()
                ias.check(ias.lib.ias_csr_copy(C.byref(c), C.byref(h), ias.MEMORY_HOST, 0), "download")
                ias.lib.ias_csr_free(C.byref(c))
                got = ias.csr_to_numpy(h)
                if got.nnz != refs[k][0] or float(got.val.sum()) != refs[k][1]:
                    errors.append((k, it, got.nnz, refs[k]))
            ias.lib.ias_plan_destroy(plan)
        except Exception as e:   # noqa: BLE001 — reported below
            errors.append((k, repr(e)))

    th = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:4]


def retry_rows(crowded, seed=41):
    """Rows in every sym3 / sym4 / sym5 bin (400 .. 12,000 products, 40
    columns per B row).  crowded=False: columns drawn from 2^20 (no list
    overflows); crowded=True: each row's B rows draw from a pool of P/3
    columns (two thirds of the products repeat a column: every such row
    overflows its possible-duplicate list and is handed to sym2)."""
    rng = np.random.default_rng(seed + crowded)
    per = 40
    brows, arows = [], []
    for m in (10, 30, 45, 60, 90, 150, 300):
        for _ in range(12):
            base = len(brows)
            pool = max(per, (m * per) // 3) if crowded else 1 << 20
            for _ in range(m):
                brows.append(rng.choice(pool, per, replace=False))
            arows.append(np.arange(base, len(brows)))
    return _csr(arows, len(brows), rng), _csr(brows, 1 << 20, rng)


def test_retry_grid_follows_plan_history():
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
    try:
        o = ias.opts(output_memory=ias.MEMORY_HOST, device=0, plan=plan)
        for crowded in (False, True, True, False, True):
            A, B = retry_rows(crowded)
            ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
            sa, sb = A.struct(), B.struct()
            c = ias.Csr()
            ias.check(ias.lib.ias_csr_mul_csr(C.byref(sa), C.byref(sb), C.byref(c), C.byref(o), None), "mul")
            got = ias.csr_to_numpy(c)
            assert_csr_identical(got, ref, f"crowded={crowded}")
    finally:
        ias.lib.ias_plan_destroy(plan)


def big_rows(seed=53):
    """B 2^21 columns wide (beyond the column bitmap), A rows of 16,385 ..
    32,768 products: plain (columns over 2^21), crowded (each row's B rows
    from a pool of P/3 columns: list overflow), many-entry (1,500 entries of
    20 products: more entries than sym5 stages), then ordinary rows."""
    rng = np.random.default_rng(seed)
    brows, arows = [], []
    def add(m, per, pool):
        base = len(brows)
        for _ in range(m):
            brows.append(rng.choice(pool, per, replace=False))
        arows.append(np.arange(base, len(brows)))
    for m in (420, 500, 640, 780, 830):            # 16.8k .. 33.2k products (the last one beyond: partitions)
        add(m, 40, 1 << 21)
    for m in (450, 700):
        add(m, 40, (m * 40) // 3)
    add(1500, 20, 1 << 21)
    nb = len(brows)
    for _ in range(2000):
        brows.append(rng.choice(1 << 21, 10, replace=False))
    for _ in range(800):
        arows.append(rng.choice(np.arange(nb, len(brows)), 12, replace=False))
    return _csr(arows, len(brows), rng), _csr(brows, 1 << 21, rng)


@pytest.mark.parametrize("force", [0, 1], ids=["sym5-big", "gtab-all"])
def test_big_rows_wide_b(monkeypatch, force):
    A, B = big_rows()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    if force:
        monkeypatch.setenv("IAS_GTAB_ALL", "1")
    else:
        monkeypatch.delenv("IAS_GTAB_ALL", raising=False)
    got, rep = ias.spgemm(A, B)
    assert rep.max_row_products == 830 * 40
    assert_csr_identical(got, ref, f"rows beyond 16,384 products, IAS_GTAB_ALL={force}")
    got_s, _ = ias.spgemm(A, B, order=ias.ORDER_SORTED)
    for i in range(8):
        s, e = ref.row_ptr[i], ref.row_ptr[i + 1]
        o = np.argsort(ref.col[s:e], kind="stable")
        np.testing.assert_array_equal(got_s.col[s:e], ref.col[s:e][o])
        np.testing.assert_array_equal(bits(got_s.val[s:e]), bits(ref.val[s:e][o]))


def test_big_rows_beyond_32bit_offsets():
    """The 16,385 - 32,768-product rows of a wide B whose entries sit beyond
    2^30: the analysis is redone with those rows in the hash partitions (not
    the global tables); bitwise."""
    A, B = big_rows()
    ref = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))
    A2 = ias.HostCsr(A.rows, A.cols + 1, A.row_ptr, A.col + 1, A.val)
    got, rep = ias.spgemm(A2, _padded_b(B, (1 << 30) + 1000))
    assert rep.max_row_products == 830 * 40
    assert_csr_identical(got, ref, "rows beyond 16,384 products, B beyond 2^30 entries")


def _padded_b(B, pad):
    """B behind a first row of `pad` entries (column 0, value 0) that A never
    selects: every selected row's entries sit beyond `pad`."""
    rp = np.concatenate([[0], B.row_ptr + pad]).astype(np.int64)
    col = np.zeros(pad + B.col.size, np.int32)   # untouched pages stay unallocated
    col[pad:] = B.col
    val = np.zeros(pad + B.val.size, np.float64)
    val[pad:] = B.val
    return ias.HostCsr(B.rows + 1, B.cols, rp, col, val)


def _check_sorted(got_s, ref, rows):
    for i in rows:
        s, e = ref.row_ptr[i], ref.row_ptr[i + 1]
        o = np.argsort(ref.col[s:e], kind="stable")
        np.testing.assert_array_equal(got_s.col[s:e], ref.col[s:e][o])
        np.testing.assert_array_equal(bits(got_s.val[s:e]), bits(ref.val[s:e][o]))


@pytest.mark.parametrize("pad", [(1 << 29) + 1000, (1 << 30) + 1000], ids=["beyond-2^29", "beyond-2^30"])
def test_b_entries_beyond_32bit_offsets(pad):
    """B's selected rows start beyond 2^29 entries (the streaming numeric pass
    gathers through 64-bit addresses: k_num2<true, …>) and beyond 2^30 (no
    sym3 / sym4 / sym5: sym2 and the global tables)."""
    R = ias.gen_rmat(13, 16, seed=71)
    ref = ob.csr_mul_csr(ob.Mat.of(R), ob.Mat.of(R))
    A = ias.HostCsr(R.rows, R.cols + 1, R.row_ptr, R.col + 1, R.val)
    B = _padded_b(R, pad)
    got, _ = ias.spgemm(A, B)
    assert_csr_identical(got, ref, f"B entries from {pad}")
    got_s, _ = ias.spgemm(A, B, order=ias.ORDER_SORTED)
    _check_sorted(got_s, ref, range(0, R.rows, 97))


@pytest.mark.parametrize("order", [0, 1], ids=["reference", "sorted"])
def test_wide_v_knob(monkeypatch, order):
    """IAS_WIDE_V=1: the 64-bit-address streaming pass on an ordinary input."""
    R = ias.gen_rmat(14, 16, seed=73)
    ref = ob.csr_mul_csr(ob.Mat.of(R), ob.Mat.of(R))
    monkeypatch.setenv("IAS_WIDE_V", "1")
    if order == 0:
        got, _ = ias.spgemm(R, R)
        assert_csr_identical(got, ref, "IAS_WIDE_V=1")
    else:
        got_s, _ = ias.spgemm(R, R, order=ias.ORDER_SORTED)
        np.testing.assert_array_equal(got_s.row_ptr, ref.row_ptr)
        _check_sorted(got_s, ref, range(R.rows))


def cbs_rows(seed=29):
    """A*B with B 3,158,000 columns wide (four column-bitmap slices of 2^20
    columns, the last partial: k_sym_cbm<true>) whose first A rows exceed
    32,768 products (the rows that took the hash partitions before round 6),
    each from B rows of 100 columns drawn from a pool — (products, pool):
      spread over every slice, few repeated columns (LDS minima, kept);
      40,000 columns across the slice 0 / 1 boundary (duplicates dropped);
      5,000 columns over all slices (most products duplicates: dropped);
      200,000 columns of slice 2 (kept);
      10,000 columns of the partial last slice;
      1,000 columns of slice 0 (every other slice empty for this row);
    then 1,500 ordinary rows."""
    rng = np.random.default_rng(seed)
    per, ncols, sw = 100, 3_158_000, 1 << 20
    pools = [(60000, rng.choice(ncols, 2_000_000, replace=False)),
             (50000, np.arange(sw - 20000, sw + 20000)),
             (40000, rng.choice(ncols, 5000, replace=False)),
             (40000, np.arange(2 * sw, 2 * sw + 200000)),
             (36000, np.arange(3 * sw, 3 * sw + 10000)),
             (36000, np.arange(1000))]
    brows, arows = [], []
    for prods, pool in pools:
        base = len(brows)
        for _ in range(prods // per):
            brows.append(rng.choice(pool, per, replace=False))
        arows.append(np.arange(base, len(brows)))
    nb = len(brows)
    for _ in range(3000):
        brows.append(rng.choice(ncols, 12, replace=False))
    for _ in range(1500):
        arows.append(rng.choice(np.arange(nb, len(brows)), 8, replace=False))
    return _csr(arows, len(brows), rng), _csr(brows, ncols, rng)


@pytest.fixture(scope="module")
def cbs_case():
    A, B = cbs_rows()
    return A, B, ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(B))


@pytest.mark.parametrize("force", [0, 1, 2, 3, "hash"], ids=["cbs", "cbs-global-own", "cbs-unlisted",
                                                              "cbs-both", "hash-partitions"])
def test_column_slices_wide_b(cbs_case, monkeypatch, force):
    """Rows beyond 32,768 products on a C wider than one LDS bitmap: the
    column-sliced k_sym_cbm<true> (opt-in, IAS_SYM_CBS=1; its first-touch
    words always in global memory: GLOBAL_WORDS in ias_last_diag proves it
    ran), its forced branches, and the default hash partitions — all
    bitwise, both orders."""
    A, B, ref = cbs_case
    if force == "hash":
        monkeypatch.delenv("IAS_SYM_CBS", raising=False)   # the default path
        monkeypatch.setenv("IAS_CBM_FORCE", "0")
    else:
        monkeypatch.setenv("IAS_SYM_CBS", "1")
        monkeypatch.setenv("IAS_CBM_FORCE", str(force))
    got, rep = ias.spgemm(A, B)
    hits = int(ias.lib.ias_last_diag())
    assert rep.max_row_products == 60000
    assert_csr_identical(got, ref, f"column slices, force={force}")
    if force == "hash":
        assert hits == 0
    else:
        assert hits & GLOBAL_WORDS, f"{hits:#x}"
        if force & 1:
            assert hits & GLOBAL_OWN and not hits & LDS_OWN
        if force & 2:
            assert not hits & (LISTED_KEEP | LISTED_DROP)
        if force == 0:
            assert hits & (LISTED_KEEP | LISTED_DROP) and hits & LDS_OWN and hits & GLOBAL_OWN
    got_s, _ = ias.spgemm(A, B, order=ias.ORDER_SORTED)
    for i in range(6):
        s, e = ref.row_ptr[i], ref.row_ptr[i + 1]
        o = np.argsort(ref.col[s:e], kind="stable")
        np.testing.assert_array_equal(got_s.col[s:e], ref.col[s:e][o])
        np.testing.assert_array_equal(bits(got_s.val[s:e]), bits(ref.val[s:e][o]))
