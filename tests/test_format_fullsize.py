"""Full-size parity through the format entry points:

  * K2 (ELL 1M x 1M, 16 per row) through ias_ell_mul_ell — the configuration
    the reference's ELL_MUL_ELL cannot run (its malloc2d byte count overflows
    int, CPU/detail/ell/common_ell.h:117-128, CPU/detail/common.h:19-31).  ELL
    rows hold each C row in CSR_MUL_CSR's order (common_ell.h:80-189 restates
    common_csr.h:85-193 over padded rows), so the device ELL result, compacted
    row by row, must give the oracle's recorded CSR digest of K2
    (tests/golden/generator_stats.json) and a padded width of 256.
  * K1 (band 256k x 256k, 7 diagonals) through ias_dia_mul_dia: the tiled VALU
    kernel bitwise against the oracle's DIA_mul_DIA restatement
    (common_dia.h:101-195), and the MFMA form (forced) within the north-star
    tolerance.
"""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import ias
import oracle_bind as ob
from fulldigest import digest_torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
STATS = json.load(open(os.path.join(HERE, "golden", "generator_stats.json")))


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if ias.device_count() < 1 or not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X box")
    return torch


def test_ell_k2_fullsize(torch_dev):
    torch = torch_dev
    rec = STATS["k2_ell1048576_k16_s7"]
    A = ias.gen_ell(*rec["args"])
    s = A.struct()
    he, de, dc = ias.Ell(), ias.Ell(), ias.Ell()
    ias.check(ias.lib.ias_csr_to_ell(C.byref(s), C.byref(he), 0.0), "to_ell")
    ias.check(ias.lib.ias_ell_copy(C.byref(he), C.byref(de), ias.MEMORY_DEVICE, 0), "upload")
    ias.lib.ias_ell_free(C.byref(he))
    o = ias.opts(output_memory=ias.MEMORY_DEVICE, device=0)
    rep = ias.Report()
    try:
        ias.check(ias.lib.ias_ell_mul_ell(C.byref(de), C.byref(de), C.byref(dc), C.byref(o), C.byref(rep)), "ell")
        K, rows = int(dc.max_nnz_per_row), int(dc.rows)
        assert K == 256 and int(dc.nnz) == rec["nnz_c"]
        dev = torch.device("cuda", 0)
        # the library's device arrays, viewed (not copied) by torch
        n_row = torch.empty(rows, dtype=torch.int32, device=dev)
        col = torch.empty(rows * K, dtype=torch.int32, device=dev)
        val = torch.empty(rows * K, dtype=torch.float64, device=dev)
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        for dst, src, nb in ((n_row, dc.nnz_row, 4 * rows), (col, dc.col, 4 * rows * K), (val, dc.val, 8 * rows * K)):
            assert hip.hipMemcpy(ctypes.c_void_p(dst.data_ptr()), ctypes.cast(src, ctypes.c_void_p), ctypes.c_size_t(nb),
                                 3) == 0   # hipMemcpyDeviceToDevice
        torch.cuda.synchronize()
        keep = (torch.arange(K, device=dev)[None, :] < n_row[:, None].long()).reshape(-1)
        c_ci, c_va = col[keep], val[keep]
        c_rp = torch.zeros(rows + 1, dtype=torch.int64, device=dev)
        c_rp[1:] = torch.cumsum(n_row.long(), 0)
        assert rep.flops == rec["flops"]
        assert hashlib.sha256(c_rp.cpu().numpy().tobytes()).hexdigest() == rec["c_row_ptr_sha256"]
        assert digest_torch(c_rp, c_ci, c_va) == rec["c_digest"], "ELL C differs from the oracle (digest)"
    finally:
        ias.lib.ias_ell_free(C.byref(de))
        ias.lib.ias_ell_free(C.byref(dc))
        torch.cuda.empty_cache()


def _k1_dia(monkeypatch, mfma):
    rec = STATS["k1_band262144_h3_s7"]
    A = ias.gen_band(*rec["args"])
    monkeypatch.setenv("IAS_DIA_MFMA", "1" if mfma else "0")
    s = A.struct()
    hd, dd, dc, hc = ias.Dia(), ias.Dia(), ias.Dia(), ias.Dia()
    ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(hd), 0.0), "to_dia")
    ias.check(ias.lib.ias_dia_copy(C.byref(hd), C.byref(dd), ias.MEMORY_DEVICE, 0), "upload")
    ias.lib.ias_dia_free(C.byref(hd))
    o = ias.opts(output_memory=ias.MEMORY_DEVICE, device=0)
    rep = ias.Report()
    ias.check(ias.lib.ias_dia_mul_dia(C.byref(dd), C.byref(dd), C.byref(dc), C.byref(o), C.byref(rep)), "dia")
    assert rep.kernel == (2 if mfma else 1), rep.kernel   # IAS_DIA_KERNEL_MFMA / _TILE
    ias.check(ias.lib.ias_dia_copy(C.byref(dc), C.byref(hc), ias.MEMORY_HOST, 0), "download")
    nd = int(hc.num_diagonals)
    got = dict(nd=nd, offsets=ias._np(hc.diagonal_offsets, nd, np.int32),
               ind=ias._np(hc.diagonal_ind, hc.rows + hc.cols - 1, np.int32),
               val=ias._np(hc.val, hc.rows * nd, np.float64).reshape(hc.rows, nd))
    for x in (dd, dc, hc):
        ias.lib.ias_dia_free(C.byref(x))
    return A, got


def test_dia_k1_fullsize(monkeypatch):
    A, got = _k1_dia(monkeypatch, False)
    ref = ob.dia_mul_dia(ob.Mat.of(A), ob.Mat.of(A))
    assert got["nd"] == ref["nd"] == 13
    np.testing.assert_array_equal(got["offsets"], ref["offsets"])
    np.testing.assert_array_equal(got["ind"], ref["ind"])
    np.testing.assert_array_equal(got["val"].view(np.int64), ref["val"].view(np.int64))


def test_dia_k1_fullsize_mfma(monkeypatch):
    A, got = _k1_dia(monkeypatch, True)
    ref = ob.dia_mul_dia(ob.Mat.of(A), ob.Mat.of(A))
    absA = ias.HostCsr(A.rows, A.cols, A.row_ptr, A.col, np.abs(A.val))
    bound = ob.dia_mul_dia(ob.Mat.of(absA), ob.Mat.of(absA))["val"]
    assert got["nd"] == ref["nd"]
    np.testing.assert_array_equal(got["offsets"], ref["offsets"])
    tol = 1e-10 * np.maximum(np.abs(ref["val"]), bound) + 1e-300
    assert np.all(np.abs(got["val"] - ref["val"]) <= tol)
