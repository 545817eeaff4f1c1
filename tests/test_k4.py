"""K4 — BASELINE.json configs[4], the 8-GPU configuration (R-MAT 2^23, edge
factor 24, seed 3: 8.4 M rows, 201 M entries, 1.19e10 products, nnz(C) =
11,851,855,388, ~142 GB of C) — pinned against the oracle's CSR_MUL_CSR
restatement (IA-SPGEMM-CPU_release/detail/csr/common_csr.h:85-193), whose
streaming digest tests/golden/make_generator_stats.py recorded in
generator_stats.json:

  * the whole K4 on one MI355X (288 GB of HBM hold A, B and all of C) through
    the device-resident two-phase ABI: flops, nnz(C), the sha256 of C's
    row pointer and the order-sensitive digest of every entry; the hub rows at
    the top and the last rows bitwise against the oracle;
  * the row blocks the eight ranks of `bench.py --gpus 8` compute
    (ias_partition_rows, P = 8), each through its own call on a row view of A
    with all of B, as each rank runs it (multi.hip / ias_dist_csr_mul_csr do
    the same per rank): the blocks' row pointers, shifted by the blocks' nnz
    offsets and concatenated, hash to the recorded sha256, and their digests
    with global row indices add up to the recorded digest — so the sharded C
    concatenated by the allgatherv is the oracle's C.
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
REC = json.load(open(os.path.join(HERE, "golden", "generator_stats.json")))["k4_rmat23_ef24_s3"]
NPARTS = 8


@pytest.fixture(scope="module")
def k4():
    import torch
    if ias.device_count() < 1 or not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X box")
    A = ias.gen_rmat(*REC["args"])
    assert (A.rows, A.nnz) == (REC["rows"], REC["nnz"])
    dev = torch.device("cuda", 0)
    d = dict(A=A, torch=torch, dev=dev, rp=torch.from_numpy(A.row_ptr).to(dev),
             ci=torch.from_numpy(A.col).to(dev), va=torch.from_numpy(A.val).to(dev))
    yield d
    del d["rp"], d["ci"], d["va"]
    torch.cuda.empty_cache()


def view(k, r0, r1):
    """rows r0:r1 of the device-resident A as a row view (col/val addressed
    absolutely, as ias_csr_row_view makes them)"""
    A = k["A"]
    return ias.Csr(r1 - r0, A.cols, int(A.row_ptr[r1] - A.row_ptr[r0]),
                   C.cast(C.c_void_p(k["rp"].data_ptr() + 8 * r0), ias.i64p),
                   C.cast(C.c_void_p(k["ci"].data_ptr()), ias.i32p),
                   C.cast(C.c_void_p(k["va"].data_ptr()), ias.f64p), ias.MEMORY_DEVICE, 0)


def block_product(k, plan, r0, r1):
    """C = A[r0:r1] * A via ias_csr_mul_csr_nnz + _compute into torch tensors"""
    torch, dev, A = k["torch"], k["dev"], k["A"]
    Am, Bm = view(k, r0, r1), view(k, 0, A.rows)
    n, rs, rep = C.c_int64(0), ias.Report(), ias.Report()
    ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Am), C.byref(Bm), C.byref(n), None, C.byref(rs)), "nnz")
    nnz = int(n.value)
    c_rp = torch.empty(r1 - r0 + 1, dtype=torch.int64, device=dev)
    c_ci = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    c_va = torch.empty(max(nnz, 1), dtype=torch.float64, device=dev)
    Cm = ias.Csr(r1 - r0, A.cols, nnz, C.cast(C.c_void_p(c_rp.data_ptr()), ias.i64p),
                 C.cast(C.c_void_p(c_ci.data_ptr()), ias.i32p), C.cast(C.c_void_p(c_va.data_ptr()), ias.f64p),
                 ias.MEMORY_DEVICE, 0)
    ias.check(ias.lib.ias_csr_mul_csr_compute(plan, C.byref(Am), C.byref(Bm), C.byref(Cm), ias.ORDER_REFERENCE,
                                              C.byref(rep)), "compute")
    torch.cuda.synchronize()
    return c_rp, c_ci[:nnz], c_va[:nnz], int(rs.flops)


def rows_block(A, r0, r1):
    s, e = int(A.row_ptr[r0]), int(A.row_ptr[r1])
    return ob.Mat(r1 - r0, A.cols, A.row_ptr[r0:r1 + 1] - s, A.col[s:e], A.val[s:e])


def test_k4_whole_on_one_gpu(k4):
    A, torch = k4["A"], k4["torch"]
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
    try:
        c_rp, c_ci, c_va, flops = block_product(k4, plan, 0, A.rows)
    finally:
        ias.lib.ias_plan_destroy(plan)
    try:
        assert flops == REC["flops"]
        rp = c_rp.cpu().numpy()
        assert int(rp[-1]) == REC["nnz_c"], (int(rp[-1]), REC["nnz_c"])
        assert hashlib.sha256(rp.tobytes()).hexdigest() == REC["c_row_ptr_sha256"], "row pointer differs"
        assert digest_torch(c_rp, c_ci, c_va) == REC["c_digest"], "C differs from the oracle (digest)"
        Bm = ob.Mat.of(A)
        for r0, r1 in ((0, 32), (A.rows - 2048, A.rows)):
            ref = ob.csr_mul_csr(rows_block(A, r0, r1), Bm)
            s, e = int(rp[r0]), int(rp[r1])
            np.testing.assert_array_equal(rp[r0:r1 + 1] - s, ref.row_ptr, err_msg=f"rows {r0}:{r1} row_ptr")
            np.testing.assert_array_equal(c_ci[s:e].cpu().numpy(), ref.col, err_msg=f"rows {r0}:{r1} col")
            np.testing.assert_array_equal(c_va[s:e].cpu().numpy().view(np.int64), ref.val.view(np.int64),
                                          err_msg=f"rows {r0}:{r1} values")
    finally:
        del c_rp, c_ci, c_va
        torch.cuda.empty_cache()


def test_k4_eight_shards(k4):
    A, torch = k4["A"], k4["torch"]
    bounds = (C.c_int64 * (NPARTS + 1))()
    sa = A.struct()
    ias.check(ias.lib.ias_partition_rows(C.byref(sa), C.byref(sa), NPARTS, bounds), "partition")
    b = list(bounds)
    assert b[0] == 0 and b[-1] == A.rows and all(x < y for x, y in zip(b[:-1], b[1:]))
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), 0, None), "plan")
    digest, off, flops, pieces = 0, 0, 0, [np.zeros(1, np.int64)]
    try:
        for r0, r1 in zip(b[:-1], b[1:]):
            c_rp, c_ci, c_va, f = block_product(k4, plan, r0, r1)
            try:
                rp = c_rp.cpu().numpy()
                assert rp[0] == 0
                pieces.append(rp[1:] + off)
                digest += digest_torch(c_rp, c_ci, c_va, row0=r0)
                off += int(rp[-1])
                flops += f
            finally:
                del c_rp, c_ci, c_va
                torch.cuda.empty_cache()
    finally:
        ias.lib.ias_plan_destroy(plan)
    rp_all = np.concatenate(pieces)
    assert flops == REC["flops"]
    assert off == REC["nnz_c"], (off, REC["nnz_c"])
    assert hashlib.sha256(rp_all.tobytes()).hexdigest() == REC["c_row_ptr_sha256"], "concatenated row pointer"
    assert digest % (1 << 64) == REC["c_digest"], "the shards' C differs from the oracle (digest)"
