"""Full-size parity on the GPU: the BASELINE.json configurations K1, K2, K3'
and K3 through the device-resident two-phase C-ABI
(ias_csr_mul_csr_nnz + ias_csr_mul_csr_compute, and the one-call
ias_csr_mul_csr_into), checked against the
oracle's CSR_MUL_CSR restatement recorded in tests/golden/generator_stats.json
by make_generator_stats.py:

  * flops and nnz(C) exact — K3's nnz(C) = 2,284,461,849 > 2^31, the size the
    reference's int row pointers cannot hold (CPU/detail/format.h:36-38);
  * sha256 of C's int64 row pointer (every row's nnz);
  * the order-sensitive digest of C (tests/fulldigest.py): every entry's row,
    position in its row, column and value bits — reverse first-touch order
    and sums in product order, bit for bit;
  * plus a bitwise comparison with the oracle of the hub rows at the top of
    the R-MAT matrices and of the last rows (past entry 2^31 for K3).
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
CASES = ["k1_band262144_h3_s7", "k2_ell1048576_k16_s7", "k3p_rmat20_ef20_s2", "k3_rmat20_ef32_s1"]


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if ias.device_count() < 1 or not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X box")
    return torch


def make(rec):
    return {"rmat": ias.gen_rmat, "band": ias.gen_band, "ell": ias.gen_ell}[rec["kind"]](*rec["args"])


def device_spgemm(torch, A, order=ias.ORDER_REFERENCE, via="twophase"):
    """C = A*A with A and C in HBM; returns (row_ptr, col, val) torch tensors and
    the symbolic report.  via="twophase": ias_csr_mul_csr_nnz + _compute;
    via="into": one ias_csr_mul_csr_into call into C of capacity flops(A*A)."""
    dev = torch.device("cuda", 0)
    rp = torch.from_numpy(A.row_ptr).to(dev)
    ci = torch.from_numpy(A.col).to(dev)
    va = torch.from_numpy(A.val).to(dev)

    def csr(r, c, v, rows, nnz):
        return ias.Csr(rows, A.cols, nnz, C.cast(C.c_void_p(r.data_ptr()), ias.i64p),
                       C.cast(C.c_void_p(c.data_ptr()), ias.i32p),
                       C.cast(C.c_void_p(v.data_ptr()), ias.f64p), ias.MEMORY_DEVICE, 0)

    Am = csr(rp, ci, va, A.rows, A.nnz)
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
    try:
        n = C.c_int64(0)
        rs, rep = ias.Report(), ias.Report()
        ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Am), C.byref(Am), C.byref(n), None, C.byref(rs)),
                  "nnz")
        nnz = int(n.value)
        cap = nnz if via == "twophase" else int(rs.flops)
        c_rp = torch.empty(A.rows + 1, dtype=torch.int64, device=dev)
        c_ci = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        c_va = torch.empty(max(cap, 1), dtype=torch.float64, device=dev)
        Cm = csr(c_rp, c_ci, c_va, A.rows, cap)
        if via == "twophase":
            ias.check(ias.lib.ias_csr_mul_csr_compute(plan, C.byref(Am), C.byref(Am), C.byref(Cm), order,
                                                      C.byref(rep)), "compute")
        else:
            ias.check(ias.lib.ias_csr_mul_csr_into(plan, C.byref(Am), C.byref(Am), C.byref(Cm), order,
                                                   C.byref(rep)), "into")
            assert Cm.nnz == nnz, (Cm.nnz, nnz)
        torch.cuda.synchronize()
    finally:
        ias.lib.ias_plan_destroy(plan)
    return c_rp, c_ci[:nnz], c_va[:nnz], rs


def rows_block(A, r0, r1):
    s, e = int(A.row_ptr[r0]), int(A.row_ptr[r1])
    return ob.Mat(r1 - r0, A.cols, A.row_ptr[r0:r1 + 1] - s, A.col[s:e], A.val[s:e])


@pytest.mark.parametrize("via", ["twophase", "into"])
@pytest.mark.parametrize("name", CASES)
def test_fullsize_against_oracle(torch_dev, name, via):
    torch = torch_dev
    rec = STATS[name]
    A = make(rec)
    assert A.nnz == rec["nnz"]
    c_rp, c_ci, c_va, rs = device_spgemm(torch, A, via=via)
    try:
        assert rs.flops == rec["flops"]
        rp = c_rp.cpu().numpy()
        nnz = int(rp[-1])
        assert nnz == rec["nnz_c"], (nnz, rec["nnz_c"])
        assert hashlib.sha256(rp.tobytes()).hexdigest() == rec["c_row_ptr_sha256"], "row pointer differs"
        assert digest_torch(c_rp, c_ci, c_va) == rec["c_digest"], "C differs from the oracle (digest)"
        # hub rows at the top and the last rows, entry by entry against the oracle
        Bm = ob.Mat.of(A)
        for r0, r1 in ((0, 64), (A.rows - 2048, A.rows)):
            ref = ob.csr_mul_csr(rows_block(A, r0, r1), Bm)
            s, e = int(rp[r0]), int(rp[r1])
            np.testing.assert_array_equal(rp[r0:r1 + 1] - s, ref.row_ptr, err_msg=f"rows {r0}:{r1} row_ptr")
            np.testing.assert_array_equal(c_ci[s:e].cpu().numpy(), ref.col, err_msg=f"rows {r0}:{r1} col")
            np.testing.assert_array_equal(c_va[s:e].cpu().numpy().view(np.int64), ref.val.view(np.int64),
                                          err_msg=f"rows {r0}:{r1} values")
        if name.startswith("k3_"):
            assert int(rp[-2049]) > 2**31, "the tail rows should sit past entry 2^31"
    finally:
        del c_rp, c_ci, c_va
        torch.cuda.empty_cache()


@pytest.mark.parametrize("name", ["k2_ell1048576_k16_s7", "k3p_rmat20_ef20_s2"])
def test_fullsize_sorted_row_pointer(torch_dev, name):
    """IAS_ORDER_SORTED at full size (K2, K3'): same row pointer, every row
    ascending, and the order-sensitive digest of C equal to the oracle's with
    every row sorted by column (c_digest_sorted: the cuSPARSE-like order of
    GPU/detail/cusparse/common_cusparse.h:78-91, values bit for bit); plus the
    hub rows entry by entry."""
    torch = torch_dev
    rec = STATS[name]
    A = make(rec)
    c_rp, c_ci, c_va, _ = device_spgemm(torch, A, order=ias.ORDER_SORTED)
    try:
        rp = c_rp.cpu().numpy()
        assert hashlib.sha256(rp.tobytes()).hexdigest() == rec["c_row_ptr_sha256"]
        assert digest_torch(c_rp, c_ci, c_va) == rec["c_digest_sorted"], "sorted C differs from the oracle (digest)"
        # ascending inside every row: a descent may only happen at a row start
        d = (c_ci[1:] <= c_ci[:-1]).nonzero().flatten() + 1
        starts = torch.from_numpy(rp[1:-1]).to(d.device)
        assert bool(torch.isin(d, starts).all()), "a row of the sorted output is not ascending"
        ref = ob.csr_mul_csr(rows_block(A, 0, 64), ob.Mat.of(A))
        for i in range(64):
            s, e = int(rp[i]), int(rp[i + 1])
            got_c = c_ci[s:e].cpu().numpy()
            o = np.argsort(ref.col[ref.row_ptr[i]:ref.row_ptr[i + 1]], kind="stable")
            np.testing.assert_array_equal(got_c, ref.col[ref.row_ptr[i]:ref.row_ptr[i + 1]][o])
            np.testing.assert_array_equal(c_va[s:e].cpu().numpy().view(np.int64),
                                          ref.val[ref.row_ptr[i]:ref.row_ptr[i + 1]][o].view(np.int64))
    finally:
        del c_rp, c_ci, c_va
        torch.cuda.empty_cache()
