"""Order-sensitive digest of a CSR product C, for full-size parity pins.

digest = sum over entries e of mix(row(e), position of e in its row, col[e],
bits of val[e]) mod 2^64 — the same function oracle/ias_oracle.c
(ora_csr_mul_csr_digest) folds CSR_MUL_CSR's rows into, so a C too large to
store on the host (K3: 2.28e9 entries) is still compared entry for entry in
the reference's order: column order, position and value bits all enter.
TEST INFRASTRUCTURE (tests/ only).
"""
from __future__ import annotations

import numpy as np

M_COL = 0x9E3779B97F4A7C15
M_POS = 0xC2B2AE3D27D4EB4F
M_ROW = 0x165667B19E3779F9
M_MUL = 0xD6E8FEB86659FD93
MASK64 = (1 << 64) - 1


def _s64(x: int) -> int:
    """a 64-bit constant as a signed int64 (torch has no uint64 arithmetic)"""
    return x - (1 << 64) if x >= (1 << 63) else x


def digest_numpy(row_ptr: np.ndarray, col: np.ndarray, val: np.ndarray) -> int:
    rows = row_ptr.shape[0] - 1
    rp = row_ptr.astype(np.int64) - int(row_ptr[0])
    lens = np.diff(rp)
    r = np.repeat(np.arange(rows, dtype=np.uint64), lens)
    pos = (np.arange(int(rp[-1]), dtype=np.int64) - np.repeat(rp[:-1], lens)).astype(np.uint64)
    with np.errstate(over="ignore"):
        x = (np.ascontiguousarray(val, np.float64).view(np.uint64)
             ^ (col.astype(np.uint32).astype(np.uint64) * np.uint64(M_COL))
             ^ (pos * np.uint64(M_POS)) ^ (r * np.uint64(M_ROW)))
        x = x * np.uint64(M_MUL)
        x ^= x >> np.uint64(32)
        return int(x.sum(dtype=np.uint64)) & MASK64


def digest_torch(row_ptr, col, val, chunk: int = 1 << 27, row0: int = 0) -> int:
    """The same digest of a device-resident C (torch tensors: int64 row_ptr,
    int32 col, float64 val), in chunks of entries.  row0: the global index of
    C's first row, for a row block of a larger C — the digest is a sum over
    entries, so the blocks' digests add up (mod 2^64) to the whole C's."""
    import torch
    dev = col.device
    rp = row_ptr.to(torch.int64) - row_ptr[0].to(torch.int64)
    nnz = int(rp[-1].item())
    vb = val.view(torch.int64)
    total = torch.zeros((), dtype=torch.int64, device=dev)
    c_col, c_pos, c_row, c_mul = (torch.tensor(_s64(c), dtype=torch.int64, device=dev)
                                  for c in (M_COL, M_POS, M_ROW, M_MUL))
    lo32 = torch.tensor(0xFFFFFFFF, dtype=torch.int64, device=dev)
    for e0 in range(0, nnz, chunk):
        e1 = min(nnz, e0 + chunk)
        e = torch.arange(e0, e1, dtype=torch.int64, device=dev)
        r = torch.searchsorted(rp, e, right=True) - 1
        pos = e - rp[r]
        x = vb[e0:e1] ^ (col[e0:e1].to(torch.int64) * c_col) ^ (pos * c_pos) ^ ((r + row0) * c_row)
        x = x * c_mul
        x = x ^ ((x >> 32) & lo32)
        total += x.sum()
        del e, r, pos, x
    return int(total.item()) & MASK64
