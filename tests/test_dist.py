"""World-size-2 (and 3) gloo runs of the multi-GPU logic on CPU: flops-balanced
row sharding + the allgatherv assembly of C (ias/dist.py).  Each rank
computes its block with the oracle (CPU); the assembled C must be identical to
the single-process oracle result, byte for byte."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, q):
    sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    import ias
    import oracle_bind as ob
    from ias import dist as idist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        A = ias.gen_rmat(11, 12, seed=21, value_mode=0)
        s = A.struct()
        b = (C.c_int64 * (world + 1))()
        ias.check(ias.lib.ias_partition_rows(C.byref(s), C.byref(s), world, b), "partition")
        r0, r1 = b[rank], b[rank + 1]
        blk = ob.Mat(r1 - r0, A.cols, A.row_ptr[r0:r1 + 1] - A.row_ptr[r0],
                     A.col[A.row_ptr[r0]:A.row_ptr[r1]], A.val[A.row_ptr[r0]:A.row_ptr[r1]])
        part = ob.csr_mul_csr(blk, ob.Mat.of(A))
        out = idist.gather_csr(torch.from_numpy(part.row_ptr), torch.from_numpy(part.col),
                               torch.from_numpy(part.val), mode=mode)
        if out is not None:
            full = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
            rp, c, v = (t.numpy() for t in out)
            ok = (np.array_equal(rp, full.row_ptr) and np.array_equal(c, full.col)
                  and np.array_equal(v.view(np.int64), full.val.view(np.int64)))
            q.put((rank, bool(ok)))
        else:
            q.put((rank, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "all"), (2, "root"), (3, "all")])
def test_sharded_assembly_matches_single(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if mode == "all":
        assert all(res[r] is True for r in range(world))
    else:
        assert res[0] is True and all(res[r] is None for r in range(1, world))


def _gather_bench_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    import bench
    import ias
    import oracle_bind as ob
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        A = ias.gen_rmat(10, 8, seed=5, value_mode=0)
        s = A.struct()
        b = (C.c_int64 * (world + 1))()
        ias.check(ias.lib.ias_partition_rows(C.byref(s), C.byref(s), world, b), "partition")
        r0, r1 = b[rank], b[rank + 1]
        blk = ob.Mat(r1 - r0, A.cols, A.row_ptr[r0:r1 + 1] - A.row_ptr[r0],
                     A.col[A.row_ptr[r0]:A.row_ptr[r1]], A.val[A.row_ptr[r0]:A.row_ptr[r1]])
        part = ob.csr_mul_csr(blk, ob.Mat.of(A))
        calls = []
        res = bench.measure_allgatherv(lambda: calls.append(1), torch.from_numpy(part.row_ptr),
                                       torch.from_numpy(part.col), torch.from_numpy(part.val), reps=2)
        full = ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A))
        q.put((rank, res, len(calls), int(full.row_ptr[-1]), int(part.row_ptr[-1]), int(A.rows)))
    finally:
        dist.destroy_process_group()


def test_allgatherv_measurement_gloo():
    """bench.measure_allgatherv (compute-only vs compute +
    allgatherv, max over ranks) on two gloo ranks with CPU tensors."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((x[0], x[1:]) for x in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nnz_local = {r: res[r][3] for r in res}
    for r, (m, ncalls, nnz_full, _, rows) in res.items():
        assert ncalls == 4   # 2 reps x (compute-only + compute with gather)
        assert m["c_nnz_total"] == nnz_full
        assert m["ms_compute_allgatherv"] >= 0 and m["ms_compute"] >= 0
        # the rank that receives the most: the other rank's entries and rows
        assert m["bytes_received_per_rank_max"] >= 12 * min(nnz_local.values())
