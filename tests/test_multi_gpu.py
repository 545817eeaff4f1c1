"""Multi-GPU entry points of the C-ABI on one MI355X:
ias_csr_mul_csr_multi with a device repeated (one host thread + plan per
entry, the row split and the row-order concatenation exercised on one GPU),
the RCCL path (ias_dist_*) with a one-rank communicator (unique id, comm,
partition, allgatherv assembly), the same entry points over the loopback
transport with 2 / 4 / 8 ranks on one GPU, and
`spgemm-gpu --devices`.  Every result is
compared bit for bit with the single-device engine and the oracle."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import ias
import oracle_bind as ob

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.int64)


def host_of(m):
    h = ias.Csr()
    ias.check(ias.lib.ias_csr_copy(C.byref(m), C.byref(h), ias.MEMORY_HOST, 0), "copy")
    return ias.csr_to_numpy(h)


@pytest.fixture(scope="module")
def rmat():
    A = ias.gen_rmat(14, 12, seed=17, value_mode=0)
    return A, ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))


@pytest.mark.parametrize("devs", [[0], [0, 0], [0, 0, 0, 0, 0]])
@pytest.mark.parametrize("order", [ias.ORDER_REFERENCE, ias.ORDER_SORTED])
def test_multi_devices_match_oracle(rmat, devs, order):
    A, ref = rmat
    s = A.struct()
    out = ias.Csr()
    o = ias.opts(order=order, output_memory=ias.MEMORY_HOST)
    d = (C.c_int32 * len(devs))(*devs)
    rep = ias.Report()
    ias.check(ias.lib.ias_csr_mul_csr_multi(C.byref(s), C.byref(s), C.byref(out), len(devs), d, C.byref(o),
                                            C.byref(rep)), "multi")
    got = ias.csr_to_numpy(out)
    assert rep.flops == ob.flops(ob.Mat.of(A), ob.Mat.of(A)) and rep.nnz_c == ref.nnz
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
    if order == ias.ORDER_REFERENCE:
        np.testing.assert_array_equal(got.col, ref.col)
        np.testing.assert_array_equal(bits(got.val), bits(ref.val))
    else:
        single, _ = ias.spgemm(A, order=ias.ORDER_SORTED)
        np.testing.assert_array_equal(got.col, single.col)
        np.testing.assert_array_equal(bits(got.val), bits(single.val))


def test_multi_device_operands_device_output(rmat):
    A, ref = rmat
    s = A.struct()
    dA = ias.Csr()
    ias.check(ias.lib.ias_csr_copy(C.byref(s), C.byref(dA), ias.MEMORY_DEVICE, 0), "upload")
    out = ias.Csr()
    o = ias.opts(output_memory=ias.MEMORY_DEVICE)
    d = (C.c_int32 * 3)(0, 0, 0)
    ias.check(ias.lib.ias_csr_mul_csr_multi(C.byref(dA), C.byref(dA), C.byref(out), 3, d, C.byref(o), None),
              "multi")
    assert out.memory == ias.MEMORY_DEVICE
    got = host_of(out)
    ias.lib.ias_csr_free(C.byref(out))
    ias.lib.ias_csr_free(C.byref(dA))
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
    np.testing.assert_array_equal(got.col, ref.col)
    np.testing.assert_array_equal(bits(got.val), bits(ref.val))


@pytest.fixture(scope="module")
def dist1():
    uid = C.create_string_buffer(128)
    st = ias.lib.ias_dist_unique_id(uid, 128)
    if st != 0:
        pytest.fail("RCCL unavailable: " + ias.lib.ias_last_error().decode())
    d = C.c_void_p()
    ias.check(ias.lib.ias_dist_create(C.byref(d), uid, 1, 0, 0), "dist_create")
    yield d
    ias.lib.ias_dist_destroy(d)


@pytest.mark.parametrize("gather", [0, 1])
def test_dist_one_rank(rmat, dist1, gather):
    A, ref = rmat
    s = A.struct()
    out = ias.Csr()
    ias.check(ias.lib.ias_dist_csr_mul_csr(dist1, C.byref(s), C.byref(s), C.byref(out), gather,
                                           ias.ORDER_REFERENCE, None), "dist_csr_mul_csr")
    assert out.memory == ias.MEMORY_DEVICE
    got = host_of(out)
    ias.lib.ias_csr_free(C.byref(out))
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
    np.testing.assert_array_equal(got.col, ref.col)
    np.testing.assert_array_equal(bits(got.val), bits(ref.val))


def test_dist_allgatherv_row_view_block(rmat, dist1):
    """allgatherv of a block whose row pointer does not start at 0 (a row
    view of C): the output's row pointer is rebased to 0."""
    A, ref = rmat
    s = A.struct()
    full = ias.Csr()
    o = ias.opts(output_memory=ias.MEMORY_DEVICE)
    ias.check(ias.lib.ias_csr_mul_csr(C.byref(s), C.byref(s), C.byref(full), C.byref(o), None), "spgemm")
    r0, r1 = 100, 9000
    v = ias.Csr()
    ias.check(ias.lib.ias_csr_row_view(C.byref(full), r0, r1, C.byref(v)), "view")
    # a row view addresses col / val absolutely (row_ptr[0] = its first entry)
    base = int(ref.row_ptr[r0])
    n = int(ref.row_ptr[r1]) - base
    assert v.nnz == n
    out = ias.Csr()
    ias.check(ias.lib.ias_dist_allgatherv_csr(dist1, C.byref(v), C.byref(out), None), "allgatherv")
    got = host_of(out)
    ias.lib.ias_csr_free(C.byref(out))
    ias.lib.ias_csr_free(C.byref(full))
    np.testing.assert_array_equal(got.row_ptr, ref.row_ptr[r0:r1 + 1] - base)
    np.testing.assert_array_equal(got.col, ref.col[base:base + n])
    np.testing.assert_array_equal(bits(got.val), bits(ref.val[base:base + n]))


def _ranks(P, fn):
    """Run fn(rank) on P host threads (one loopback rank each; ctypes releases
    the GIL inside the library); re-raise the first failure."""
    import threading
    errs, res = [None] * P, [None] * P

    def run(r):
        try:
            res[r] = fn(r)
        except BaseException as e:  # noqa: BLE001 - reported below
            errs[r] = e

    th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a loopback rank hung"
    for e in errs:
        if e is not None:
            raise e
    return res


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("gather", [0, 1])
def test_dist_loopback_ranks(rmat, P, gather):
    """P loopback ranks on one GPU run the sharded path —
    ias_partition_rows, every rank's block through the engine, and (gather=1)
    the allgatherv with its per-root offsets and k_shift_ends fix-up; the
    concatenated C equals the oracle's bit for bit on every rank."""
    A, ref = rmat
    s = A.struct()
    group = f"test-{P}-{gather}".encode()
    bounds = (C.c_int64 * (P + 1))()
    ias.check(ias.lib.ias_partition_rows(C.byref(s), C.byref(s), P, bounds), "partition")

    def rank(r):
        d = C.c_void_p()
        ias.check(ias.lib.ias_dist_create_loopback(C.byref(d), group, P, r, 0), "create_loopback")
        try:
            out = ias.Csr()
            ias.check(ias.lib.ias_dist_csr_mul_csr(d, C.byref(s), C.byref(s), C.byref(out), gather,
                                                   ias.ORDER_REFERENCE, None), "dist_csr_mul_csr")
            got = host_of(out)
            ias.lib.ias_csr_free(C.byref(out))
            return got
        finally:
            ias.lib.ias_dist_destroy(d)

    outs = _ranks(P, rank)
    for r, got in enumerate(outs):
        if gather:
            np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
            np.testing.assert_array_equal(got.col, ref.col)
            np.testing.assert_array_equal(bits(got.val), bits(ref.val))
        else:
            r0, r1 = bounds[r], bounds[r + 1]
            lo, hi = int(ref.row_ptr[r0]), int(ref.row_ptr[r1])
            np.testing.assert_array_equal(got.row_ptr, ref.row_ptr[r0:r1 + 1] - lo)
            np.testing.assert_array_equal(got.col, ref.col[lo:hi])
            np.testing.assert_array_equal(bits(got.val), bits(ref.val[lo:hi]))


def test_dist_loopback_allgatherv_of_row_views(rmat):
    """Four loopback ranks each hand in a row view of one full C (row_ptr not
    starting at 0, col / val addressed absolutely): the gathered C is the full
    C, rebased."""
    A, ref = rmat
    s = A.struct()
    full = ias.Csr()
    o = ias.opts(output_memory=ias.MEMORY_DEVICE)
    ias.check(ias.lib.ias_csr_mul_csr(C.byref(s), C.byref(s), C.byref(full), C.byref(o), None), "spgemm")
    P = 4
    cuts = [0, 1, 2000, 9000, A.rows]   # one near-empty block

    def rank(r):
        d = C.c_void_p()
        ias.check(ias.lib.ias_dist_create_loopback(C.byref(d), b"views-4", P, r, 0), "create_loopback")
        try:
            v = ias.Csr()
            ias.check(ias.lib.ias_csr_row_view(C.byref(full), cuts[r], cuts[r + 1], C.byref(v)), "view")
            out = ias.Csr()
            ias.check(ias.lib.ias_dist_allgatherv_csr(d, C.byref(v), C.byref(out), None), "allgatherv")
            got = host_of(out)
            ias.lib.ias_csr_free(C.byref(out))
            return got
        finally:
            ias.lib.ias_dist_destroy(d)

    outs = _ranks(P, rank)
    ias.lib.ias_csr_free(C.byref(full))
    for got in outs:
        np.testing.assert_array_equal(got.row_ptr, ref.row_ptr)
        np.testing.assert_array_equal(got.col, ref.col)
        np.testing.assert_array_equal(bits(got.val), bits(ref.val))


def test_cli_gpu_devices(inputs_dir):
    exe = os.path.join(ROOT, "ia-spgemm_amd", "bin", "spgemm-gpu")
    path = os.path.join(inputs_dir, "Ragusa18.mtx")
    one = subprocess.run([exe, path], capture_output=True, text=True, timeout=120)
    two = subprocess.run([exe, path, "--devices", "0,0,0"], capture_output=True, text=True, timeout=120)
    assert one.returncode == 0 and two.returncode == 0, two.stdout + two.stderr
    assert "row blocks over 3 devices" in two.stdout
    sums = lambda out: [l for l in out.splitlines() if l.startswith("verified_sum")]
    assert sums(one.stdout) == sums(two.stdout) and sums(one.stdout)
