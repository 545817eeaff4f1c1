#!/usr/bin/env python3
"""Run C = A*A with a timing build of libias (tools/timing.sh) and print the
mean per-row microseconds of each phase of the row kernels.

Phases (spgemm_kernels.hpp, Timer marks):
  symbolic (k_symbolic_st): 0 table clear, 1 wait for column loads, 2 inserts,
    3 step/segment syncs, 4 duplicate scan, 5 slot scan+bits, 6 bitmap
    write, 7 duplicate flush
  numeric (k_numeric_st): 0 setup, 1 segment load, 2 gather+write,
    3 segment sync, 4 fix-up barrier, 5 duplicate fix-up
  sym-cbm (k_sym_cbm): 0 pass 1, 1 multi bitmap, 2 ranks + minima init,
    3 pass 2, 4 pass 3, 5 word prefixes, 6 placement
  sym4 / sym5 (k_sym4, k_sym5): 0 staging, 1 filter, 2 classify, 3 exact,
    4 finish, 5 filter clear
  sort (k_sort_bucket, --sorted): 0 loads + range, 1 coarse bins, 2 fine
    buckets, 3 bucket scan, 4 ranks, 5 staging, 6 stores issued;
    k_sort_bitmap16: 0 loads + clear, 1 bitmap, 2 prefix, 3 ranks, 4 staging + stores;
    k_sort_bitmap: 0 row + clear, 1 bitmap, 2 prefix, 3 ranks + workspace, 4 copy back
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))
import torch  # noqa: E402,F401  (one HIP runtime: torch's)
import ias  # noqa: E402

SLOTS, PH = 32, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--ef", type=float, default=20)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--sorted", action="store_true", help="IAS_ORDER_SORTED (row sort kernels timed)")
    a = ap.parse_args()
    order = ias.ORDER_SORTED if a.sorted else ias.ORDER_REFERENCE
    A = ias.gen_rmat(a.scale, a.ef, seed=a.seed)
    f = ias.lib.ias_debug_timing
    f.restype = C.c_int
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * (SLOTS * (PH + 1)))()
    ias.spgemm(A, device=0, order=order)          # warm-up
    f(buf, len(buf))                               # reset
    _, rep = ias.spgemm(A, device=0, order=order)
    n = f(buf, len(buf))
    if n <= 0:
        print("not a timing build"); return
    print("report ms: symbolic %.3f numeric %.3f total %.3f" % (rep.ms_symbolic, rep.ms_numeric, rep.ms_total))
    for slot in range(SLOTS):
        row = buf[slot * (PH + 1):(slot + 1) * (PH + 1)]
        cnt = row[PH]
        if not cnt:
            continue
        kind = "symbolic" if slot < 16 else "numeric"
        team = 1 << (slot % 16)
        if 24 <= slot <= 26:
            kind, team = "sym3 K=%d" % (8, 12, 16)[slot - 24], 64
        elif slot >= 30:
            kind, team = ("sym5 U=16384" if slot == 31 else "sym5 U=8192"), 64 * (4 if slot == 31 else 2)
        elif slot == 27:
            kind, team = "sym4", 64
        elif slot == 29:
            kind, team = "sym-part", 1024
        elif slot == 28:
            kind, team = "sym-cbm", 1024
        elif slot == 17:
            kind, team = "sortbm16", 1024
        elif slot == 18:
            kind, team = "sortbm", 1024
        elif 11 <= slot <= 16:
            kind, team = "sort", (64 if slot <= 12 else 1 << (slot - 6))
        us = [row[i] / cnt / 100.0 for i in range(PH)]   # wall clock: 100 MHz
        print("%-8s TEAM %4d rows %8d  per-row us: %s  sum %.2f" % (
            kind, team, cnt, " ".join("%6.2f" % u for u in us), sum(us)))


if __name__ == "__main__":
    main()
