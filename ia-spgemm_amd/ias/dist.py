"""Multi-GPU exchange step of the row-sharded SpGEMM.

One process per GPU.  Rows of A are split into contiguous blocks of equal
products (ias_partition_rows); every rank holds all of B and computes its
block of C with the single-GPU engine — no collective on that path.  The only
exchange is assembling C when the caller wants it whole: per-rank (rows, nnz)
counts by all_gather, then an allgatherv of col/val/row_ptr.  RCCL has no
v-variant, so the allgatherv is one broadcast per root into that root's slice
of the output (every peer receives each slice over its own xGMI link); the
row pointers are shifted by the rank's global nnz offset before the gather.
`mode="root"` gathers to rank 0 only (point-to-point recv of each slice).

Works with the "nccl" (RCCL) backend on device tensors and with "gloo" on
CPU tensors (tests/test_dist.py).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def _counts(local_rows: int, local_nnz: int, device) -> Tuple[List[int], List[int]]:
    world = dist.get_world_size()
    mine = torch.tensor([local_rows, local_nnz], dtype=torch.int64, device=device)
    allc = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(allc, mine)
    rows = [int(t[0]) for t in allc]
    nnz = [int(t[1]) for t in allc]
    return rows, nnz


def allgatherv(local: torch.Tensor, counts: List[int], root_only: bool = False) -> Optional[torch.Tensor]:
    """Concatenate 1-D tensors of per-rank lengths `counts` on every rank
    (or on rank 0 only when root_only)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    assert local.numel() == counts[rank]
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    if root_only:
        if rank == 0:
            out = torch.empty(offs[-1], dtype=local.dtype, device=local.device)
            out[offs[0]:offs[1]].copy_(local)
            for r in range(1, world):
                if counts[r]:
                    dist.recv(out[offs[r]:offs[r + 1]], src=r)
            return out
        if counts[rank]:
            dist.send(local.contiguous(), dst=0)
        return None
    out = torch.empty(offs[-1], dtype=local.dtype, device=local.device)
    for r in range(world):
        if counts[r] == 0:
            continue
        sl = out[offs[r]:offs[r + 1]]
        if r == rank:
            sl.copy_(local)
        dist.broadcast(sl, src=r)
    return out


def gather_csr(row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, mode: str = "all"):
    """Assemble the row-sharded C.  row_ptr is this rank's local pointer
    (rows_local + 1 entries, starting at 0).  Returns (row_ptr, col, val) of
    the whole C (mode "all": on every rank; "root": on rank 0, None elsewhere)."""
    assert mode in ("all", "root")
    rank = dist.get_rank()
    rows_local = row_ptr.numel() - 1
    nnz_local = int(col.numel())
    rows, nnz = _counts(rows_local, nnz_local, row_ptr.device)
    base = sum(nnz[:rank])
    shifted = row_ptr[1:] + base                     # global offsets of this block's row ends
    root_only = mode == "root"
    rp = allgatherv(shifted, rows, root_only)
    c = allgatherv(col, nnz, root_only)
    v = allgatherv(val, nnz, root_only)
    if rp is None:
        return None
    rp = torch.cat([torch.zeros(1, dtype=rp.dtype, device=rp.device), rp])
    return rp, c, v
