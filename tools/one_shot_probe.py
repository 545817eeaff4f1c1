#!/usr/bin/env python3
"""First-call probe: K3' on the device, then two ias_csr_mul_csr calls with no
plan (the per-device default plan) and a library-allocated device C, as
bench.py's one_shot leg.  Run under `rocprofv3 --hip-trace --kernel-trace` to
see where the first call's wall time goes (tools/hip_api_summary.py).
usage: python tools/one_shot_probe.py [--config k3p] [--warm-plan]"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="k3p")
    p.add_argument("--calls", type=int, default=3)
    a = p.parse_args()
    import torch
    import ias
    import bench
    kind, prm, _ = bench.workload(a.config, 1)
    A = bench.generate(kind, prm)
    dev = torch.device("cuda", 0)
    rp = torch.from_numpy(A.row_ptr).to(dev)
    ci = torch.from_numpy(A.col).to(dev)
    va = torch.from_numpy(A.val).to(dev)
    torch.cuda.synchronize()
    Am = ias.Csr(A.rows, A.cols, A.nnz, C.cast(C.c_void_p(rp.data_ptr()), ias.i64p),
                 C.cast(C.c_void_p(ci.data_ptr()), ias.i32p), C.cast(C.c_void_p(va.data_ptr()), ias.f64p),
                 ias.MEMORY_DEVICE, 0)
    for i in range(a.calls):
        c, rep = ias.Csr(), ias.Report()
        o = ias.opts(output_memory=ias.MEMORY_DEVICE, device=0)
        t = time.perf_counter()
        ias.check(ias.lib.ias_csr_mul_csr(C.byref(Am), C.byref(Am), C.byref(c), C.byref(o), C.byref(rep)), "one-shot")
        wall = 1e3 * (time.perf_counter() - t)
        t = time.perf_counter()
        ias.lib.ias_csr_free(C.byref(c))
        fr = 1e3 * (time.perf_counter() - t)
        print(f"call {i}: wall {wall:.2f} ms device {rep.ms_total:.2f} ms (analysis {rep.ms_analysis:.2f} "
              f"symbolic {rep.ms_symbolic:.2f} numeric {rep.ms_numeric:.2f}) free {fr:.2f} ms nnz {c.nnz}",
              flush=True)


if __name__ == "__main__":
    main()
