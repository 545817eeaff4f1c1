"""DIA robustness on the DEFAULT kernel choice (no IAS_DIA_MFMA override) and
the caller-provided-C entry point.

The reference's DIA_mul_DIA (IA-SPGEMM-CPU_release/detail/dia/common_dia.h:
101-195) takes any offset set and any value, finite or not: every in-range
pair (A diagonal, B diagonal) is multiplied and summed in loop order, so a
stored 0.0 next to an Inf gives NaN there too.  Checked here against the
oracle's restatement of it:

  * a wide dense band (65 diagonals: the library picks the MFMA kernel) with
    an Inf and a NaN in it: the tiles holding them fall back to the VALU pair
    sums (k_dia_mfma's non-finite path, dia.hip), which are bitwise the
    reference; the other tiles are MFMA dense blocks, within the north-star
    tolerance.  NaN entries are compared as NaN (the payload of a NaN made on
    the GPU need not equal the x86 one), everything else bit for bit on the
    fallback tiles;
  * >= 16 diagonals spread over +-several thousand offsets: the dense-block
    gate refuses the MFMA form (its blocks would be almost all padding), the
    library takes the tiled or the pair kernel, bitwise;
  * ias_dia_mul_dia_into (caller-provided device C, no allocation in the call):
    bitwise equal to ias_dia_mul_dia, the capacity error when C is too small;
  * the DIA plan cache past its 256 entries (evicts, keeps working).
"""
import ctypes as C

import numpy as np
import pytest

import ias
import oracle_bind as ob

pytestmark = pytest.mark.gpu

TILE = 1    # IAS_DIA_KERNEL_TILE
MFMA = 2    # IAS_DIA_KERNEL_MFMA
PAIRS = 3   # IAS_DIA_KERNEL_PAIRS


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if ias.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X box")


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.int64)


def _run(A, monkeypatch):
    """C = A*A through ias_dia_mul_dia with the library's own kernel choice."""
    monkeypatch.delenv("IAS_DIA_MFMA", raising=False)
    s = A.struct()
    da, dc = ias.Dia(), ias.Dia()
    ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(da), 0.0), "to_dia")
    o = ias.opts(output_memory=ias.MEMORY_HOST, device=0)
    rep = ias.Report()
    ias.check(ias.lib.ias_dia_mul_dia(C.byref(da), C.byref(da), C.byref(dc), C.byref(o), C.byref(rep)), "dia")
    nd = dc.num_diagonals
    out = dict(nd=nd, kernel=int(rep.kernel), offsets=ias._np(dc.diagonal_offsets, nd, np.int32),
               ind=ias._np(dc.diagonal_ind, dc.rows + dc.cols - 1, np.int32),
               val=ias._np(dc.val, dc.rows * nd, np.float64).reshape(dc.rows, nd))
    ias.lib.ias_dia_free(C.byref(da))
    ias.lib.ias_dia_free(C.byref(dc))
    return out


def _band_with_nonfinite(n=4096, h=32, seed=11):
    A = ias.gen_band(n, h, seed=seed)
    val = A.val.copy()
    # an Inf and a NaN inside the band (rows 1000 and 2500), a -Inf near the end
    for row, x in ((1000, np.inf), (2500, np.nan), (n - 40, -np.inf)):
        s = int(A.row_ptr[row])
        val[s + 5] = x
    return ias.HostCsr(A.rows, A.cols, A.row_ptr, A.col, val)


def test_dia_mfma_nonfinite_default_path(monkeypatch):
    A = _band_with_nonfinite()
    ref = ob.dia_mul_dia(ob.Mat.of(A), ob.Mat.of(A))
    got = _run(A, monkeypatch)
    assert got["kernel"] == MFMA, "65 dense diagonals: the default choice is the MFMA kernel"
    assert got["nd"] == ref["nd"]
    np.testing.assert_array_equal(got["offsets"], ref["offsets"])
    np.testing.assert_array_equal(got["ind"], ref["ind"])
    rv, gv = ref["val"], got["val"]
    # non-finite results exist, and sit exactly where the reference has them
    assert np.isnan(rv).any() and np.isinf(rv).any()
    np.testing.assert_array_equal(np.isnan(gv), np.isnan(rv))
    np.testing.assert_array_equal(np.isposinf(gv), np.isposinf(rv))
    np.testing.assert_array_equal(np.isneginf(gv), np.isneginf(rv))
    # 16-row tiles holding a non-finite operand take the VALU pair sums: bitwise
    bad_rows = np.unique(np.nonzero(~np.isfinite(rv))[0])
    tiles = np.unique(bad_rows // 16)
    fin = np.isfinite(rv)
    for t in tiles:
        r0, r1 = 16 * t, min(16 * t + 16, rv.shape[0])
        m = fin[r0:r1]
        np.testing.assert_array_equal(bits(gv[r0:r1][m]), bits(rv[r0:r1][m]),
                                      err_msg=f"fallback tile {t}: finite entries bitwise")
    # the finite rest within the north-star tolerance (MFMA's fused sums)
    absA = ias.HostCsr(A.rows, A.cols, A.row_ptr, A.col, np.nan_to_num(np.abs(A.val), posinf=0.0))
    bound = ob.dia_mul_dia(ob.Mat.of(absA), ob.Mat.of(absA))["val"]
    tol = 1e-10 * np.maximum(np.abs(np.where(fin, rv, 0.0)), bound) + 1e-300
    assert np.all(np.abs(gv[fin] - rv[fin]) <= tol[fin])


def _spread_band(n=20000, seed=9):
    """17 diagonals at offsets 0, +-937, +-1874, ... up to +-7496 (a few
    entries missing on each): the MFMA gate's dense blocks would be ~97 %
    padding."""
    rng = np.random.default_rng(seed)
    offs = [937 * k for k in range(-8, 9)]
    rows = []
    for i in range(n):
        cols = [i + o for o in offs if 0 <= i + o < n and rng.random() > 0.03]
        rows.append(np.array(sorted(cols), np.int64))
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    return ias.HostCsr(n, n, rp, col, rng.standard_normal(col.size))


def test_dia_spread_offsets_default_path(monkeypatch):
    A = _spread_band()
    ref = ob.dia_mul_dia(ob.Mat.of(A), ob.Mat.of(A))
    got = _run(A, monkeypatch)
    assert got["kernel"] in (TILE, PAIRS), got["kernel"]
    assert got["nd"] == ref["nd"] and ref["nd"] >= 16
    np.testing.assert_array_equal(got["offsets"], ref["offsets"])
    np.testing.assert_array_equal(got["ind"], ref["ind"])
    np.testing.assert_array_equal(bits(got["val"]), bits(ref["val"]))


def _device_dia_of(A, torch):
    """A as a device DIA (library-allocated through ias_dia_copy)."""
    s = A.struct()
    ha, da = ias.Dia(), ias.Dia()
    ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(ha), 0.0), "to_dia")
    ias.check(ias.lib.ias_dia_copy(C.byref(ha), C.byref(da), ias.MEMORY_DEVICE, 0), "upload")
    ias.lib.ias_dia_free(C.byref(ha))
    return da


@pytest.mark.parametrize("mk", [lambda: ias.gen_band(5000, 3, seed=7), lambda: ias.gen_band(3000, 32, seed=5),
                                _spread_band], ids=["k1like", "wide65", "spread"])
def test_dia_into_matches_allocating_call(mk):
    import torch
    A = mk()
    da = _device_dia_of(A, torch)
    nd = C.c_int32(0)
    ias.check(ias.lib.ias_dia_mul_dia_ndiag(C.byref(da), C.byref(da), C.byref(nd)), "ndiag")
    ndc = int(nd.value)
    rows, cols = int(da.rows), int(da.cols)
    dev = torch.device("cuda", 0)
    offs = torch.zeros(max(ndc, 1), dtype=torch.int32, device=dev)
    ind = torch.zeros(rows + cols - 1, dtype=torch.int32, device=dev)
    val = torch.full((rows * max(ndc, 1),), 7.0, dtype=torch.float64, device=dev)
    Cd = ias.Dia(rows=0, cols=0, num_diagonals=ndc, choice=0,
                 diagonal_offsets=C.cast(C.c_void_p(offs.data_ptr()), ias.i32p),
                 diagonal_ind=C.cast(C.c_void_p(ind.data_ptr()), ias.i32p),
                 val=C.cast(C.c_void_p(val.data_ptr()), ias.f64p), memory=ias.MEMORY_DEVICE, device=0)
    # one diagonal short: the capacity error, with the needed count returned
    Cs = ias.Dia.from_buffer_copy(Cd)
    Cs.num_diagonals = ndc - 1
    assert ias.lib.ias_dia_mul_dia_into(C.byref(da), C.byref(da), C.byref(Cs), None, None) == 11
    assert Cs.num_diagonals == ndc
    rep = ias.Report()
    ias.check(ias.lib.ias_dia_mul_dia_into(C.byref(da), C.byref(da), C.byref(Cd), None, C.byref(rep)), "into")
    torch.cuda.synchronize()
    assert Cd.num_diagonals == ndc and Cd.rows == rows and Cd.cols == cols and Cd.choice == 1
    hc = ias.Dia()
    o = ias.opts(output_memory=ias.MEMORY_HOST, device=0)
    ias.check(ias.lib.ias_dia_mul_dia(C.byref(da), C.byref(da), C.byref(hc), C.byref(o), None), "dia")
    assert hc.num_diagonals == ndc
    np.testing.assert_array_equal(offs.cpu().numpy()[:ndc], ias._np(hc.diagonal_offsets, ndc, np.int32))
    np.testing.assert_array_equal(ind.cpu().numpy(), ias._np(hc.diagonal_ind, rows + cols - 1, np.int32))
    np.testing.assert_array_equal(bits(val.cpu().numpy()[:rows * ndc]),
                                  bits(ias._np(hc.val, rows * ndc, np.float64)))
    ias.lib.ias_dia_free(C.byref(hc))
    ias.lib.ias_dia_free(C.byref(da))


def test_dia_plan_cache_eviction(monkeypatch):
    """More distinct offset sets / shapes than the plan cache holds (256): the
    least recently used plans are evicted and every call stays correct."""
    monkeypatch.delenv("IAS_DIA_MFMA", raising=False)
    o = ias.opts(output_memory=ias.MEMORY_HOST, device=0)
    for i in range(300):
        A = ias.gen_band(64 + i, 1 + i % 3, seed=i)
        s = A.struct()
        da, dc = ias.Dia(), ias.Dia()
        ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(da), 0.0), "to_dia")
        ias.check(ias.lib.ias_dia_mul_dia(C.byref(da), C.byref(da), C.byref(dc), C.byref(o), None), f"dia {i}")
        if i % 37 == 0 or i >= 295:
            ref = ob.dia_mul_dia(ob.Mat.of(A), ob.Mat.of(A))
            nd = dc.num_diagonals
            assert nd == ref["nd"]
            np.testing.assert_array_equal(bits(ias._np(dc.val, dc.rows * nd, np.float64)),
                                          bits(ref["val"].ravel()))
        ias.lib.ias_dia_free(C.byref(da))
        ias.lib.ias_dia_free(C.byref(dc))


def _diag_matrix(n, offs, seed):
    rng = np.random.default_rng(seed)
    rows = [np.array(sorted(i + o for o in offs if 0 <= i + o < n), np.int64) for i in range(n)]
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    return ias.HostCsr(n, n, rp, col, rng.standard_normal(col.size))


def test_dia_into_reused_plan_sees_changed_offsets(monkeypatch):
    """ias_dia_mul_dia_into with device offsets reuses the last call's plan
    without reading them back (dia.hip, DiaFast); the device-side check must
    catch offsets rewritten in place between calls (same arrays, same counts):
    each call bitwise equal to the oracle of what the arrays hold."""
    import torch
    monkeypatch.delenv("IAS_DIA_MFMA", raising=False)
    n = 4096
    mats = [_diag_matrix(n, [-3, -2, -1, 0, 1, 2, 3], 1), _diag_matrix(n, [-9, -6, -3, 0, 3, 6, 9], 2),
            _diag_matrix(n, [-3, -2, -1, 0, 1, 2, 3], 3)]
    dev = torch.device("cuda", 0)
    host = []
    for A in mats:
        s, h = A.struct(), ias.Dia()
        ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(h), 0.0), "to_dia")
        assert h.num_diagonals == 7
        host.append((ias._np(h.diagonal_offsets, 7, np.int32).copy(), ias._np(h.val, n * 7, np.float64).copy(),
                     ias._np(h.diagonal_ind, 2 * n - 1, np.int32).copy()))
        ias.lib.ias_dia_free(C.byref(h))
    a_off = torch.from_numpy(host[0][0]).to(dev)
    a_val = torch.from_numpy(host[0][1]).to(dev)
    a_ind = torch.from_numpy(host[0][2]).to(dev)
    da = ias.Dia(rows=n, cols=n, num_diagonals=7, choice=1,
                 diagonal_offsets=C.cast(C.c_void_p(a_off.data_ptr()), ias.i32p),
                 diagonal_ind=C.cast(C.c_void_p(a_ind.data_ptr()), ias.i32p),
                 val=C.cast(C.c_void_p(a_val.data_ptr()), ias.f64p), memory=ias.MEMORY_DEVICE, device=0)
    cap = 13
    offs = torch.zeros(cap, dtype=torch.int32, device=dev)
    ind = torch.zeros(2 * n - 1, dtype=torch.int32, device=dev)
    val = torch.zeros(n * cap, dtype=torch.float64, device=dev)
    for step, k in enumerate([0, 0, 1, 1, 2, 0]):
        a_off.copy_(torch.from_numpy(host[k][0]))
        a_val.copy_(torch.from_numpy(host[k][1]))
        a_ind.copy_(torch.from_numpy(host[k][2]))
        torch.cuda.synchronize()
        Cd = ias.Dia(rows=0, cols=0, num_diagonals=cap, choice=0,
                     diagonal_offsets=C.cast(C.c_void_p(offs.data_ptr()), ias.i32p),
                     diagonal_ind=C.cast(C.c_void_p(ind.data_ptr()), ias.i32p),
                     val=C.cast(C.c_void_p(val.data_ptr()), ias.f64p), memory=ias.MEMORY_DEVICE, device=0)
        ias.check(ias.lib.ias_dia_mul_dia_into(C.byref(da), C.byref(da), C.byref(Cd), None, None), f"into {step}")
        torch.cuda.synchronize()
        ref = ob.dia_mul_dia(ob.Mat.of(mats[k]), ob.Mat.of(mats[k]))
        nd = int(Cd.num_diagonals)
        assert nd == ref["nd"], (step, nd, ref["nd"])
        np.testing.assert_array_equal(offs.cpu().numpy()[:nd], ref["offsets"], err_msg=f"step {step}")
        np.testing.assert_array_equal(ind.cpu().numpy(), ref["ind"], err_msg=f"step {step}")
        np.testing.assert_array_equal(bits(val.cpu().numpy()[:n * nd]), bits(ref["val"].ravel()),
                                      err_msg=f"step {step}")
