"""Device memory the library keeps between calls (include/ias.h:
ias_device_release / ias_device_cached_bytes): the per-device default plan's
workspace (calls made without a plan) and the block cache of freed outputs.

  * after a plan-less call the kept bytes are reported and released on request;
  * out-of-memory relief: with the device nearly full, an allocation that only
    fits once the idle default plan's workspace is given back succeeds (the
    library's hipMalloc retry releases it), as does a later plan-less call.
"""
import ctypes as C

import numpy as np
import pytest

import ias

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if ias.device_count() < 1 or not t.cuda.is_available():
        pytest.fail("no HIP device visible: the gpu tests must run on an MI355X box")
    return t


def _cached():
    b = C.c_int64(0)
    ias.check(ias.lib.ias_device_cached_bytes(0, C.byref(b)), "cached_bytes")
    return int(b.value)


def _planless_call(A):
    """ias_csr_mul_csr with no plan and device output (default plan), C freed."""
    c, rep = ias.Csr(), ias.Report()
    o = ias.opts(output_memory=ias.MEMORY_DEVICE, device=0)
    s = A.struct()
    ias.check(ias.lib.ias_csr_mul_csr(C.byref(s), C.byref(s), C.byref(c), C.byref(o), C.byref(rep)), "planless")
    nnz = int(c.nnz)
    ias.lib.ias_csr_free(C.byref(c))
    return nnz


def test_release_reports_and_frees(torch):
    A = ias.gen_rmat(17, 16, seed=4)
    _planless_call(A)
    before = _cached()
    assert before > 0
    freed = C.c_int64(0)
    ias.check(ias.lib.ias_device_release(0, C.byref(freed)), "release")
    assert freed.value > 0
    assert _cached() == 0
    # the next plan-less call grows the workspace again and is still correct
    got, _ = ias.spgemm(A, device=0)
    assert got.nnz > 0


def test_out_of_memory_relief(torch):
    A = ias.gen_rmat(19, 16, seed=6)
    nnz = _planless_call(A)            # default plan workspace grown for this product
    W = _cached()
    assert W > (64 << 20), W
    free0, _ = torch.cuda.mem_get_info(0)
    # left free: room for the closing plan-less call's C and staged A (its
    # workspace comes back by the release) + 256 MiB
    keep = 12 * nnz + 12 * A.nnz + 16 * (A.rows + 1) + (256 << 20)
    hog = torch.empty(max(free0 - keep - W // 4, 0), dtype=torch.uint8, device="cuda:0")
    try:
        torch.cuda.synchronize()
        free1, _ = torch.cuda.mem_get_info(0)
        # 12 B per entry (int32 col + f64 val): more than is free, less than
        # free + the kept workspace
        want = free1 + W // 2
        n = want // 12
        m = ias.Csr()
        st = ias.lib.ias_csr_alloc(C.byref(m), 1, 1, n, ias.MEMORY_DEVICE, 0)
        assert st == 0, f"allocation of {want} B with {free1} B free and {W} B kept failed: " \
                        f"{ias.lib.ias_last_error().decode()}"
        ias.lib.ias_csr_free(C.byref(m))
        ias.check(ias.lib.ias_device_release(0, None), "release")
        # a plan-less call still runs next to the hog (its workspace is back)
        assert _planless_call(A) == nnz
    finally:
        del hog
        torch.cuda.empty_cache()
