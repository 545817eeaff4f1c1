#!/usr/bin/env python3
"""Call one GPU parity test function N times in one process (flakiness
check; prints pass/fail per repetition).  usage: rerun_gpu_case.py N module func [args...]"""
import importlib
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ia-spgemm_amd"), os.path.join(ROOT, "tests")]
n, mod, fn, *args = sys.argv[1:]
if os.environ.get("DIRTY_GB"):
    # fill device memory with garbage and hand it back to the driver, so the
    # library's fresh allocations start dirty (as after other tests in a suite)
    import torch
    t = torch.full((int(float(os.environ["DIRTY_GB"]) * 2**30),), 0xAB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    del t
    torch.cuda.empty_cache()
m = importlib.import_module(mod)
f = getattr(m, fn)
bad = 0
for i in range(int(n)):
    try:
        f(*args)
        print(f"rep {i}: ok", flush=True)
    except Exception as e:  # noqa: BLE001
        bad += 1
        print(f"rep {i}: FAIL {type(e).__name__}: {str(e)[:300]}", flush=True)
print(f"{bad} of {n} failed")
sys.exit(1 if bad else 0)
