#!/usr/bin/env python3
"""bench.py — SpGEMM GFLOP/s (2*flops(A*A)/t) + output nnz/s, fp64, on N MI355X.

Contract:
  python bench.py --gpus N --steps K --warmup W
One step = one full C = A*A of this rank's row block through the C-ABI,
inputs resident in HBM, C written into preallocated device arrays.  Default
`--engine twophase`: ias_csr_mul_csr_nnz + ias_csr_mul_csr_compute, as
cuSPARSE's csrgemmNnz + csrgemm (row analysis, binning, symbolic, scan, host
read of nnz, numeric + write C).  `--engine into`: one ias_csr_mul_csr_into
call per step into C of capacity flops(A*A) >= nnz(C).

Workload (default `--config auto`): R-MAT power-law, a,b,c = .45,.15,.15.
N=1: the north-star headline matrix K3' (2^20 rows, edge factor 20, seed 2;
SURVEY.md §8).  N>1: the K4 family, 2^(20+log2 N) rows, edge factor 24,
seed 3 — N=8 is BASELINE's K4 (8M x 8M, avg 24 nnz/row).  Rows are sharded by
estimated device cost (ias_partition_rows) across ranks with B replicated
(broadcast once over RCCL before timing); per-rank work grows with the
matrix, hence "scaling": "weak".  The line names its series
(config.family / config.series, series()); the N=1 line also times the K4
family's own N=1 point (R-MAT 2^20, ef 24, seed 3) as `weak_anchor`, after
its own loop.  A named --config is the same matrix for every N: "strong".  No collective inside the timed region (C
stays sharded).  For N>1 the exchange step is measured after the timed loop
(`allgatherv` in the line): one step compute-only and one step
compute + the RCCL allgatherv that concatenates C on every rank
(ias/dist.py gather_csr), max over ranks; `--no-gather` skips it,
tools/gather_bench.py runs it alone with more repetitions.
"""
import argparse
import ctypes as C
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ia-spgemm_amd"))

import numpy as np  # noqa: E402

METRIC = "SpGEMM GFLOP/s (2·flops(A·A)/t) + output nnz/s, fp64, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)

CONFIGS = {
    # name: (kind, params, description)
    "k1": ("band", dict(n=1 << 18, h=3, seed=7), "banded 256k x 256k, 7 diagonals"),
    "k1w": ("band", dict(n=1 << 18, h=32, seed=7), "banded 256k x 256k, 65 diagonals (wide band: DIA MFMA A/B)"),
    "k2": ("ell", dict(n=1 << 20, k=16, seed=7), "ELL-shaped 1M x 1M, 16 nnz/row (CSR path)"),
    "k3": ("rmat", dict(scale=20, ef=32, seed=1), "R-MAT 2^20, avg 32 nnz/row"),
    "k3p": ("rmat", dict(scale=20, ef=20, seed=2), "R-MAT 2^20, ~20 nnz/row (north-star headline)"),
    "k4": ("rmat", dict(scale=23, ef=24, seed=3), "R-MAT 2^23, avg 24 nnz/row"),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="auto", help="auto | " + " | ".join(CONFIGS))
    p.add_argument("--order", default="reference", choices=["reference", "sorted"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-full", action="store_true",
                   help="CPU baseline on the full matrix (ILP64 MKL when nnz(C) > 2^31) instead of a row "
                        "sample for products beyond 1.2e9 flops")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--json-out", default=None)
    p.add_argument("--engine", default="twophase", choices=["twophase", "into"],
                   help="twophase: ias_csr_mul_csr_nnz + ias_csr_mul_csr_compute; into: one "
                        "ias_csr_mul_csr_into call per step")
    p.add_argument("--no-host-e2e", action="store_true",
                   help="skip the one PCIe-inclusive call with host operands (N=1 only)")
    p.add_argument("--as-rank", default=None,
                   help="single process: run only rank R's shard of the --gpus N workload "
                        "(rehearses one rank of the multi-GPU run on one GPU; reports per-rank numbers); "
                        "'R1,R2,...' or 'all' run several shards one after the other, one line each")
    p.add_argument("--format", default="csr", choices=["csr", "dia"],
                   help="dia: C = A*A through the DIA kernel (ias_dia_mul_dia_into) on device-resident DIA "
                        "operands (banded configs, N=1)")
    p.add_argument("--no-gather", action="store_true", help="N>1: skip the allgatherv measurement")
    p.add_argument("--gather-reps", type=int, default=1, help="N>1: repetitions of the allgatherv measurement")
    p.add_argument("--no-anchor", action="store_true",
                   help="N>1: skip timing the whole matrix on rank 0's GPU alone after the distributed loop")
    p.add_argument("--no-weak-anchor", action="store_true",
                   help="N=1 auto: skip timing the K4 family's N=1 point (R-MAT 2^20, ef 24, seed 3)")
    p.add_argument("--no-one-shot", action="store_true",
                   help="N=1: skip the library-allocated one-shot calls (ias_csr_mul_csr, device C)")
    return p.parse_args(argv)


def workload(cfg: str, world: int):
    if cfg == "auto":
        if world <= 1:
            return "rmat", dict(scale=20, ef=20, seed=2), (
                "R-MAT 2^20, edge factor 20, seed 2, (a,b,c)=(.45,.15,.15): north-star K3'")
        scale = 20 + int(round(math.log2(world)))
        return "rmat", dict(scale=scale, ef=24, seed=3), (
            f"R-MAT 2^{scale}, edge factor 24, seed 3, (a,b,c)=(.45,.15,.15): K4 family (N=8: BASELINE K4)")
    kind, prm, desc = CONFIGS[cfg]
    return kind, dict(prm), desc


def series(cfg: str, world: int) -> dict:
    """How this line belongs to a scaling series (config.family / scaling /
    series): `auto` is the north-star K3' at N = 1 and the K4 family (R-MAT
    2^(20+log2 N), edge factor 24, seed 3, ~2^20 rows per GPU) for N > 1 — a
    weak-scaling series whose own N = 1 point (R-MAT 2^20, ef 24, seed 3) the
    N = 1 line carries as `weak_anchor`; a named --config is the same matrix
    for every N, a strong-scaling series."""
    if cfg == "auto":
        if world <= 1:
            return {"family": "K3'", "scaling": "weak",
                    "series": "N=1 headline: K3' (north-star). The N>1 lines are the K4-family weak-scaling "
                              "series (R-MAT 2^(20+log2 N), ef 24, seed 3); its N=1 point is this line's "
                              "weak_anchor"}
        return {"family": "K4", "scaling": "weak",
                "series": f"K4-family weak scaling: R-MAT 2^{20 + int(round(math.log2(world)))} on {world} GPUs "
                          f"(~2^20 rows per GPU); its N=1 point is the N=1 line's weak_anchor, not its value (K3')"}
    name = cfg.upper().replace("P", "'")
    return {"family": name, "scaling": "strong",
            "series": f"{name} strong scaling: the same matrix for every N, rows sharded by estimated cost"}


def generate(kind, prm):
    import ias
    if kind == "rmat":
        return ias.gen_rmat(prm["scale"], prm["ef"], 0.45, 0.15, 0.15, prm["seed"], 0)
    if kind == "band":
        return ias.gen_band(prm["n"], prm["h"], prm["seed"], 0)
    if kind == "ell":
        return ias.gen_ell(prm["n"], prm["k"], prm["seed"], 0)
    raise ValueError(kind)


def as_rank_list(spec, n):
    if spec is None:
        return None
    if spec == "all":
        return list(range(n))
    rs = [int(x) for x in str(spec).split(",") if x != ""]
    for r in rs:
        if not 0 <= r < n:
            raise SystemExit(f"--as-rank {r} outside 0..{n - 1}")
    return rs


def main(argv=None):
    args = parse(argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world == 1:
        world_req = args.gpus
    else:
        world_req = world
    import torch
    import torch.distributed as dist
    import ias

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    as_ranks = as_rank_list(args.as_rank, world_req) if not dist_on else None

    kind, prm, desc = workload(args.config, world_req)
    ser = series(args.config, world_req)
    # ---------------- inputs: rank 0 generates, B replicated by broadcast
    t_gen = time.time()
    meta = torch.zeros(4, dtype=torch.int64)
    nparts = world_req if (as_ranks is not None) else world
    if rank == 0:
        A = generate(kind, prm)
        meta[:] = torch.tensor([A.rows, A.cols, A.nnz, ias.flops(A, A)])
        bounds = (C.c_int64 * (nparts + 1))()
        sa = A.struct()
        ias.check(ias.lib.ias_partition_rows(C.byref(sa), C.byref(sa), nparts, bounds), "partition")
        bnd = torch.tensor(list(bounds), dtype=torch.int64)
    else:
        A = None
        bnd = torch.zeros(world + 1, dtype=torch.int64)
    if dist_on:
        meta_d, bnd_d = meta.to(dev), bnd.to(dev)
        dist.broadcast(meta_d, 0)
        dist.broadcast(bnd_d, 0)
        meta, bnd = meta_d.cpu(), bnd_d.cpu()
    rows, cols, nnz_a, flops_total = [int(x) for x in meta]
    if rank == 0:
        rp = torch.from_numpy(A.row_ptr).to(dev)
        ci = torch.from_numpy(A.col).to(dev)
        va = torch.from_numpy(A.val).to(dev)
    else:
        rp = torch.empty(rows + 1, dtype=torch.int64, device=dev)
        ci = torch.empty(nnz_a, dtype=torch.int32, device=dev)
        va = torch.empty(nnz_a, dtype=torch.float64, device=dev)
    if dist_on:
        for t in (rp, ci, va):
            dist.broadcast(t, 0)
    torch.cuda.synchronize()
    t_gen = time.time() - t_gen

    def dcsr(r0, r1, rp_t, nnz):
        return ias.Csr(r1 - r0, cols, nnz,
                       C.cast(C.c_void_p(rp_t.data_ptr() + 8 * r0), ias.i64p),
                       C.cast(C.c_void_p(ci.data_ptr()), ias.i32p),
                       C.cast(C.c_void_p(va.data_ptr()), ias.f64p), ias.MEMORY_DEVICE, local)

    if args.format == "dia":
        if dist_on or as_ranks is not None:
            raise SystemExit("--format dia runs on one GPU")
        run_dia(args, A, kind, prm, desc, flops_total, local, t_gen)
        return

    Bm = dcsr(0, rows, rp, nnz_a)
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), local, None), "plan")
    order = ias.ORDER_SORTED if args.order == "sorted" else ias.ORDER_REFERENCE

    def run_shard(shard):
        """Warm-up + the timed loop over this process's shard `shard` of A;
        returns the JSON line (rank 0's view) and the shard's C tensors."""
        r0, r1 = int(bnd[shard]), int(bnd[shard + 1])
        rp_host = rp[r0:r1 + 1].cpu()
        Am = dcsr(r0, r1, rp, int(rp_host[-1] - rp_host[0]))
        if args.engine == "twophase":
            nnz_c = C.c_int64(0)
            ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Am), C.byref(Bm), C.byref(nnz_c), None, None),
                      "nnz")
            cap = int(nnz_c.value)
        else:
            # capacity = flops of this shard, an upper bound of nnz(C) known from
            # A and B alone (here read off a symbolic pass's report)
            nnz_c, probe = C.c_int64(0), ias.Report()
            ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Am), C.byref(Bm), C.byref(nnz_c), None,
                                                  C.byref(probe)), "nnz (capacity probe)")
            cap = int(probe.flops)
        c_rp = torch.empty(r1 - r0 + 1, dtype=torch.int64, device=dev)
        c_ci = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        c_va = torch.empty(max(cap, 1), dtype=torch.float64, device=dev)
        Cm = ias.Csr(r1 - r0, cols, cap, C.cast(C.c_void_p(c_rp.data_ptr()), ias.i64p),
                     C.cast(C.c_void_p(c_ci.data_ptr()), ias.i32p),
                     C.cast(C.c_void_p(c_va.data_ptr()), ias.f64p), ias.MEMORY_DEVICE, local)
        rep = ias.Report()
        rep_s = ias.Report()

        def step_into():
            Cm.nnz = cap
            ias.check(ias.lib.ias_csr_mul_csr_into(plan, C.byref(Am), C.byref(Bm), C.byref(Cm), order,
                                                   C.byref(rep)), "into")
            return rep

        def step_twophase():
            n = C.c_int64(0)
            ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Am), C.byref(Bm), C.byref(n), None,
                                                  C.byref(rep_s)), "nnz")
            Cm.nnz = cap
            ias.check(ias.lib.ias_csr_mul_csr_compute(plan, C.byref(Am), C.byref(Bm), C.byref(Cm), order,
                                                      C.byref(rep)), "compute")
            rep.ms_analysis, rep.ms_symbolic = rep_s.ms_analysis, rep_s.ms_symbolic
            return rep

        step = step_into if args.engine == "into" else step_twophase

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = []
        for _ in range(args.steps):
            r = step()
            reps.append((r.ms_total, r.ms_analysis, r.ms_symbolic, r.ms_numeric, r.ms_stream))
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        local_nnz = int(Cm.nnz) if args.engine == "into" else cap
        t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        nnz_tot = torch.tensor([float(local_nnz)], dtype=torch.float64, device=dev)
        num_ms = torch.tensor([statistics.mean(x[3] for x in reps)], dtype=torch.float64, device=dev)
        if dist_on:
            dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
            dist.all_reduce(nnz_tot, op=dist.ReduceOp.SUM)
            dist.all_reduce(num_ms, op=dist.ReduceOp.MAX)
        elapsed = float(t_max.item())
        ms_step = 1000.0 * elapsed / args.steps
        gflops = 2.0 * flops_total / (ms_step * 1e6)
        nnz_c_total = int(nnz_tot.item())

        # Roofline (HBM-bound).  Dominant launch: the streaming
        # numeric pass (k_num2), event-timed on
        # its own stream inside the library.  Its algorithmic bytes per launch
        # follow §8(d3)'s B_alg: the C entries it writes (12 B each) plus one
        # read of A and of B (bytes(X) = 8·(rows+1) + 12·nnz(X)); the B-row
        # re-reads (12 B per product, mostly served by L2 / the Infinity Cache)
        # are reported separately as gather_bytes, never in `achieved`.
        rows_local = r1 - r0
        bytes_a = 8 * (rows_local + 1) + 12 * int(Am.nnz)
        bytes_b = 8 * (rows + 1) + 12 * nnz_a
        bytes_c = 8 * (rows_local + 1) + 12 * local_nnz
        alg_bytes = bytes_a + bytes_b + bytes_c
        ms_flat = statistics.mean(x[4] for x in reps)
        flat_bytes = 12 * int(rep.stream_nnz) + bytes_a + bytes_b
        gather_bytes = 12 * int(rep.stream_products)
        kname = "k_num2"
        units = {"products": int(rep.stream_products), "c_entries": int(rep.stream_nnz)}
        # the pass is 1 to 3 launches (rows by duplicate class; each class's
        # fix-ups overlap the rest): ms_stream sums the launches' own durations
        # (events around each launch), so per launch = the pass's bytes and time
        # / launches, which is what rocprofv3's average launch duration shows
        launches = max(1, int(getattr(rep, "stream_launches", 1) or 1))
        if int(rep.stream_nnz) < local_nnz // 2:
            # most of C comes from the short-row / table kernels (K1, K2): the
            # dominant unit is then the whole numeric phase (event-timed), its
            # bytes the C entries it writes plus one read of A and B
            kname = "numeric phase (k_short_num / table kernels)"
            ms_flat = statistics.mean(x[3] for x in reps)
            flat_bytes = 12 * local_nnz + bytes_a + bytes_b
            gather_bytes = 12 * int(rep_s.flops)
            units = {"products": int(rep_s.flops), "c_entries": local_nnz}
            launches = 1
        achieved = flat_bytes / (ms_flat * 1e-3) / 1e9 if ms_flat > 0 else 0.0
        traffic, lds_conf = None, None
        pmc_file = os.path.join(ROOT, "profiles", f"pmc_{args.config}_n{world_req}.json")
        if os.path.exists(pmc_file):
            try:
                prof = json.load(open(pmc_file))
                traffic = prof.get(kname, {}).get("hbm_bytes_per_launch")
                lds_conf = prof.get("lds_bank_conflict_ratio")
            except Exception:
                traffic, lds_conf = None, None

        out = {
            "metric": METRIC,
            "value": round(gflops, 3),
            "unit": "GFLOP/s",
            "n_gpus": world_req,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": ser["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (deterministic R-MAT/band/ELL generator, ia-spgemm_amd/csrc/gen.cpp)",
            "config": {
                "workload": desc,
                "family": ser["family"],
                "series": ser["series"],
                "kind": kind, **prm,
                "rows": rows, "nnz_a": nnz_a, "flops": flops_total, "nnz_c": nnz_c_total,
                "order": args.order,
                "engine": args.engine,
                "parallelism": f"row-block x{world_req}, B replicated",
            },
            "nnz_per_s": round(nnz_c_total / (ms_step * 1e-3), 1),
            "phases_ms_rank0": {
                "total_device": round(statistics.mean(x[0] for x in reps), 4),
                "analysis": round(statistics.mean(x[1] for x in reps), 4),
                "symbolic": round(statistics.mean(x[2] for x in reps), 4),
                "numeric": round(statistics.mean(x[3] for x in reps), 4),
            },
            "roofline": {
                "kernel": kname,
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "alg_bytes_per_launch": flat_bytes // launches,
                "launches_per_pass": launches,
                "ms_per_pass": round(ms_flat, 4),
                "alg_bytes_formula": "12*c_entries + bytes(A) + bytes(B), bytes(X) = 8*(rows+1) + 12*nnz(X)",
                "gather_bytes": gather_bytes,
                "lds_bank_conflict_ratio": lds_conf,
                "ms_per_launch": round(ms_flat / launches, 4),
                "units_per_pass": units,
            },
            "roofline_step": {
                "what": "whole step: B_alg = bytes(A) + bytes(B) + bytes(C) (SURVEY 8 d3) / step time",
                "alg_bytes": alg_bytes,
                "achieved": round(alg_bytes / (ms_step * 1e-3) / 1e9, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(alg_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            },
            "setup_s": round(t_gen, 2),
        }
        if as_ranks is not None:
            out["as_rank"] = {"rank": shard, "of": world_req, "rows": [r0, r1],
                              "note": "one rank's shard only: value / nnz_per_s are per-rank figures"}
            shard_flops = int(rep_s.flops) if args.engine == "twophase" else int(rep.flops)
            out["as_rank"]["flops"] = shard_flops
            out["as_rank"]["nnz_c"] = local_nnz
            out["value"] = round(2.0 * shard_flops / (ms_step * 1e6), 3)
            out["nnz_per_s"] = round(local_nnz / (ms_step * 1e-3), 1)
            out["n_gpus"] = 1
        return out, step, (c_rp, c_ci[:local_nnz], c_va[:local_nnz])

    shards = as_ranks if as_ranks is not None else [rank]
    for shard in shards:
        out, step, cbufs = run_shard(shard)
        out["value_per_gpu"] = round(out["value"] / max(1, out["n_gpus"]), 3)
        if dist_on and not args.no_gather:
            out["allgatherv"] = measure_allgatherv(step, *cbufs, args.gather_reps)
        if dist_on and not args.no_anchor:
            # the same matrix on one GPU (rank 0's, the others idle at a
            # barrier), after the distributed loop: the scaling anchor
            del cbufs, step
            step = cbufs = None
            torch.cuda.empty_cache()
            anchor = same_matrix_1gpu(plan, dcsr(0, rows, rp, nnz_a), Bm, rows, cols, local, dev, rank,
                                      out["ms_per_step"], flops_total)
            if rank == 0:
                out["same_matrix_1gpu"] = anchor
        if rank == 0 and world == 1 and as_ranks is None and args.config == "auto" and not args.no_weak_anchor:
            # the K4 family's N = 1 point (the weak-scaling series' anchor)
            del cbufs, step
            step = cbufs = None
            torch.cuda.empty_cache()
            out["weak_anchor"] = weak_anchor(local, dev, args.steps, args.warmup)
        if rank == 0 and world == 1 and as_ranks is None and not args.no_one_shot:
            # C's buffers go back to torch's cache, not to the driver: the
            # one-shot call then allocates fresh memory beside them, as a caller
            # holding its own tensors would
            del cbufs, step
            step = cbufs = None
            out["one_shot"] = one_shot(dcsr(0, rows, rp, nnz_a), local, out["ms_per_step"], nnz_c_step=out["config"]["nnz_c"])
        if rank == 0 and world == 1 and as_ranks is None and not args.no_cpu_baseline and \
                kind in ("rmat", "band", "ell"):
            out["cpu_baseline"] = cpu_baseline(A, flops_total, args.cpu_threads, args.cpu_full)
            if out["cpu_baseline"] and out["cpu_baseline"].get("value"):
                out["speedup_vs_cpu_baseline"] = round(out["value"] / out["cpu_baseline"]["value"], 2)
            out["cpu_baseline_alg2"] = cpu_baseline_alg2(A, flops_total, args.cpu_threads)

        if rank == 0 and world == 1 and as_ranks is None and not args.no_host_e2e:
            # the end-to-end rate with host operands (A, B uploaded, C
            # downloaded over PCIe inside the call), one call after the timed
            # region; never `value`.
            del cbufs, step
            torch.cuda.empty_cache()
            step = cbufs = None
            t_e = time.perf_counter()
            _, rh = ias.spgemm(A, order=order, device=local)
            wall = (time.perf_counter() - t_e) * 1e3
            out["host_e2e"] = {
                "what": "one ias_csr_mul_csr call with host A, B and host C (upload + compute + download); "
                        "ms_wall also holds the call's workspace allocation and the numpy copy of C",
                "ms_wall": round(wall, 2), "ms_upload": round(rh.ms_upload, 3),
                "ms_device": round(rh.ms_total, 3), "ms_download": round(rh.ms_download, 3),
                "gflops_pcie_inclusive": round(2.0 * flops_total / (wall * 1e6), 3),
            }
        if rank == 0:
            line = json.dumps(out)
            print(line, flush=True)
            if args.json_out:
                with open(args.json_out, "a" if len(shards) > 1 else "w") as f:
                    f.write(line + "\n")
        del cbufs, step
        torch.cuda.empty_cache()

    ias.lib.ias_plan_destroy(plan)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


def weak_anchor(local, dev, steps, warmup):
    """The K4 family at N = 1 (R-MAT 2^20, edge factor 24, seed 3) on this GPU,
    the same two-phase step as the line's own: the point the driver's
    1/2/4/8-GPU curve (whose N > 1 lines are this family) scales from."""
    import torch
    import ias
    kind, prm, _ = workload("auto", 2)
    prm = dict(prm, scale=20)
    A = generate(kind, prm)
    flops = ias.flops(A, A)
    rp = torch.from_numpy(A.row_ptr).to(dev)
    ci = torch.from_numpy(A.col).to(dev)
    va = torch.from_numpy(A.val).to(dev)

    def csr(r, c, v, rows, nnz):
        return ias.Csr(rows, A.cols, nnz, C.cast(C.c_void_p(r.data_ptr()), ias.i64p),
                       C.cast(C.c_void_p(c.data_ptr()), ias.i32p),
                       C.cast(C.c_void_p(v.data_ptr()), ias.f64p), ias.MEMORY_DEVICE, local)

    Am = csr(rp, ci, va, A.rows, A.nnz)
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), local, None), "plan")
    try:
        n = C.c_int64(0)
        ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Am), C.byref(Am), C.byref(n), None, None), "nnz")
        nnz = int(n.value)
        c_rp = torch.empty(A.rows + 1, dtype=torch.int64, device=dev)
        c_ci = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
        c_va = torch.empty(max(nnz, 1), dtype=torch.float64, device=dev)
        Cm = csr(c_rp, c_ci, c_va, A.rows, nnz)

        def step():
            m = C.c_int64(0)
            ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Am), C.byref(Am), C.byref(m), None, None), "nnz")
            ias.check(ias.lib.ias_csr_mul_csr_compute(plan, C.byref(Am), C.byref(Am), C.byref(Cm), 0, None),
                      "compute")
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / steps
    finally:
        ias.lib.ias_plan_destroy(plan)
    return {"what": "the K4 family's N=1 point: R-MAT 2^20, edge factor 24, seed 3, (a,b,c)=(.45,.15,.15) on "
                    "this GPU, the same two-phase step",
            "scale": 20, "ef": prm["ef"], "seed": prm["seed"], "flops": flops, "nnz_c": nnz,
            "ms_per_step": round(ms, 4), "value": round(2.0 * flops / (ms * 1e6), 3), "steps": steps}


def same_matrix_1gpu(plan, Afull, Bm, rows, cols, local, dev, rank, ms_dist, flops_total, steps=2):
    """Rank 0 computes the WHOLE C = A*A alone on its GPU (2 timed steps after
    a warm-up, the same two-phase calls as a bench step) while the other ranks
    wait at a barrier: the same-problem anchor of the N-GPU line
    (speedup_vs_1gpu_same_matrix = t_1gpu / t_step).  Skipped when the whole
    C does not fit next to what rank 0 holds."""
    import torch
    import torch.distributed as dist
    import ias
    res = None
    dist.barrier()
    if rank == 0:
        nnz_c = C.c_int64(0)
        ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Afull), C.byref(Bm), C.byref(nnz_c), None, None), "nnz")
        need = 12 * int(nnz_c.value) + 8 * (rows + 1)
        free = torch.cuda.mem_get_info(dev)[0]
        if need > 0.85 * free:
            res = {"what": "skipped: the whole C does not fit on one GPU next to the workspace",
                   "c_bytes": need, "free_bytes": free}
        else:
            c_rp = torch.empty(rows + 1, dtype=torch.int64, device=dev)
            c_ci = torch.empty(max(int(nnz_c.value), 1), dtype=torch.int32, device=dev)
            c_va = torch.empty(max(int(nnz_c.value), 1), dtype=torch.float64, device=dev)
            Cm = ias.Csr(rows, cols, int(nnz_c.value), C.cast(C.c_void_p(c_rp.data_ptr()), ias.i64p),
                         C.cast(C.c_void_p(c_ci.data_ptr()), ias.i32p),
                         C.cast(C.c_void_p(c_va.data_ptr()), ias.f64p), ias.MEMORY_DEVICE, local)

            def step():
                n = C.c_int64(0)
                ias.check(ias.lib.ias_csr_mul_csr_nnz(plan, C.byref(Afull), C.byref(Bm), C.byref(n), None, None),
                          "nnz")
                ias.check(ias.lib.ias_csr_mul_csr_compute(plan, C.byref(Afull), C.byref(Bm), C.byref(Cm), 0, None),
                          "compute")
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            ms1 = 1e3 * (time.perf_counter() - t0) / steps
            del c_rp, c_ci, c_va
            torch.cuda.empty_cache()
            res = {"what": "the whole matrix C = A*A on rank 0's GPU alone (same two-phase calls), after the "
                           "distributed loop", "ms_per_step": round(ms1, 3),
                   "gflops": round(2.0 * flops_total / (ms1 * 1e6), 3), "steps": steps,
                   "speedup_vs_1gpu_same_matrix": round(ms1 / ms_dist, 3)}
    dist.barrier()
    return res


def one_shot(Am, local, ms_step, nnz_c_step=0):
    """Two ias_csr_mul_csr calls with device-resident A = B and a device C the
    library allocates (no plan, no stream passed: the per-device default plan),
    as the reference's cuSPARSE timed region includes C's allocation
    (GPU/detail/cusparse/common_cusparse.h:74-93): wall and device ms of the
    first call (workspace allocation included) and of the second.  Before them,
    `alloc_probe_ms`: one hipMalloc + hipFree of C's size (through
    ias_csr_alloc, blocks this large bypass the block cache) — what fresh
    device memory costs on this box, the part of the first call no kernel
    change can remove."""
    import ias
    res = {}
    if nnz_c_step > 0:
        m = ias.Csr()
        t = time.perf_counter()
        ias.check(ias.lib.ias_csr_alloc(C.byref(m), Am.rows, Am.cols, nnz_c_step, ias.MEMORY_DEVICE, local),
                  "alloc probe")
        ta = time.perf_counter()
        ias.lib.ias_csr_free(C.byref(m))
        tf = time.perf_counter()
        res["alloc_probe_ms"] = {"bytes": 12 * nnz_c_step + 8 * (Am.rows + 1),
                                 "alloc": round(1e3 * (ta - t), 3), "free": round(1e3 * (tf - ta), 3)}
    for tag in ("first", "second"):
        c, rep = ias.Csr(), ias.Report()
        o = ias.opts(output_memory=ias.MEMORY_DEVICE, device=local)
        t = time.perf_counter()
        ias.check(ias.lib.ias_csr_mul_csr(C.byref(Am), C.byref(Am), C.byref(c), C.byref(o), C.byref(rep)),
                  "one-shot")
        res[f"ms_wall_{tag}"] = round(1e3 * (time.perf_counter() - t), 3)
        res[f"ms_device_{tag}"] = round(rep.ms_total, 3)
        ias.lib.ias_csr_free(C.byref(c))
    res["what"] = ("ias_csr_mul_csr, device A = B, library-allocated device C (C's allocation inside the call, "
                   "as cuSPARSE's timed region), default plan; wall includes the call's host work")
    res["first_vs_warm_step"] = round(res["ms_wall_first"] / ms_step, 3)
    return res


def run_dia(args, A, kind, prm, desc, flops_total, local, t_gen):
    """One step = ias_dia_mul_dia_into(A, A, C) on device-resident DIA operands
    into a device C allocated once before the loop (the reference's GPU DIA
    path writes into C arrays allocated before its kernels,
    GPU/detail/dia_dev/common_dia_dev.h:85-122); the kernel time is the call's
    event-timed ms_total.  The library-allocating ias_dia_mul_dia (C allocated
    and freed every call) is timed after the loop as `alloc_call`."""
    import torch
    import ias
    s = A.struct()
    ha, da = ias.Dia(), ias.Dia()
    ias.check(ias.lib.ias_csr_to_dia(C.byref(s), C.byref(ha), 0.0), "to_dia")
    ias.check(ias.lib.ias_dia_copy(C.byref(ha), C.byref(da), ias.MEMORY_DEVICE, local), "dia upload")
    nda = int(ha.num_diagonals)
    ias.lib.ias_dia_free(C.byref(ha))
    plan = C.c_void_p()
    ias.check(ias.lib.ias_plan_create(C.byref(plan), local, None), "plan")
    o = ias.opts(output_memory=ias.MEMORY_DEVICE, device=local, plan=plan)
    rep = ias.Report()
    nd = C.c_int32(0)
    ias.check(ias.lib.ias_dia_mul_dia_ndiag(C.byref(da), C.byref(da), C.byref(nd)), "ndiag")
    ndc = [int(nd.value)]
    rows_a, cols_b = int(da.rows), int(da.cols)
    dev = torch.device("cuda", local)
    c_off = torch.empty(max(ndc[0], 1), dtype=torch.int32, device=dev)
    c_ind = torch.empty(max(rows_a + cols_b - 1, 1), dtype=torch.int32, device=dev)
    c_val = torch.empty(max(rows_a * ndc[0], 1), dtype=torch.float64, device=dev)

    def cdia():
        return ias.Dia(rows=rows_a, cols=cols_b, num_diagonals=ndc[0], choice=1,
                       diagonal_offsets=C.cast(C.c_void_p(c_off.data_ptr()), ias.i32p),
                       diagonal_ind=C.cast(C.c_void_p(c_ind.data_ptr()), ias.i32p),
                       val=C.cast(C.c_void_p(c_val.data_ptr()), ias.f64p), memory=ias.MEMORY_DEVICE, device=local)
    Cd = cdia()

    def step():
        Cd.num_diagonals = ndc[0]
        ias.check(ias.lib.ias_dia_mul_dia_into(C.byref(da), C.byref(da), C.byref(Cd), C.byref(o), C.byref(rep)),
                  "dia into")

    def step_alloc():
        dc = ias.Dia()
        ias.check(ias.lib.ias_dia_mul_dia(C.byref(da), C.byref(da), C.byref(dc), C.byref(o), C.byref(rep)), "dia")
        ias.lib.ias_dia_free(C.byref(dc))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        step()
        kms.append(rep.ms_total)
    torch.cuda.synchronize()
    ms_step = 1e3 * (time.perf_counter() - t0) / args.steps
    ms_k = statistics.mean(kms)
    step_alloc()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step_alloc()
    torch.cuda.synchronize()
    ms_alloc = 1e3 * (time.perf_counter() - t1) / args.steps
    rows = int(A.rows)
    alg = 8 * rows * (2 * nda + ndc[0]) + 4 * (2 * nda + ndc[0])   # A, B (= A) read, C written
    kname = {1: "k_dia_tile", 2: "k_dia_mfma", 3: "k_dia_mul"}.get(int(rep.kernel), "?")   # the library's choice
    out = {
        "metric": METRIC,
        "value": round(2.0 * flops_total / (ms_step * 1e6), 3),
        "unit": "GFLOP/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (deterministic band generator, ia-spgemm_amd/csrc/gen.cpp)",
        "config": {"workload": desc + " (DIA format)", "kind": kind, **prm, "rows": rows,
                   "diagonals_a": nda, "diagonals_c": ndc[0], "flops": flops_total, "format": "dia",
                   "parallelism": "single GPU"},
        "roofline": {
            "kernel": kname,
            "bound": "hbm", "achieved": round(alg / (ms_k * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(alg / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
            "alg_bytes_per_launch": alg,
            "alg_bytes_formula": "8*rows*(nd_A + nd_B + nd_C) + 4*(nd_A + nd_B + nd_C)",
            "ms_per_launch": round(ms_k, 4),
        },
        "alloc_call": {"what": "ias_dia_mul_dia (library-allocated device C, freed every call), same loop",
                       "ms_per_step": round(ms_alloc, 4)},
        "setup_s": round(t_gen, 2),
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(A, flops_total, args.cpu_threads, args.cpu_full)
    ias.lib.ias_dia_free(C.byref(da))
    ias.lib.ias_plan_destroy(plan)
    line = json.dumps(out)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")


def measure_allgatherv(step, c_rp, c_ci, c_va, reps=1):
    """SURVEY §8 e1's exchange step, after the timed loop: `reps` times one
    step compute-only and one step compute + the allgatherv that concatenates
    the row-sharded C on every rank (ias/dist.py gather_csr: per-rank counts,
    then one RCCL broadcast per root into that root's slice), each bracketed by
    barriers, max over ranks.  Returns ms figures and the bytes each rank
    receives."""
    import torch
    import torch.distributed as dist
    from ias.dist import gather_csr
    dev = c_ci.device
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)

    def timed(fn):
        sync()
        dist.barrier()
        sync()
        t = time.perf_counter()
        res = fn()
        sync()
        dist.barrier()
        sync()
        el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return 1e3 * float(el.item()), res

    def compute_and_gather():
        step()
        return gather_csr(c_rp, c_ci, c_va, mode="all")

    # the gathered C must fit next to everything this rank holds
    tot = torch.tensor([int(c_ci.numel()), int(c_rp.numel()) - 1], dtype=torch.int64, device=dev)
    dist.all_reduce(tot)
    need = 12 * int(tot[0]) + 8 * (int(tot[1]) + 1)
    if dev.type == "cuda":
        free = torch.tensor([torch.cuda.mem_get_info(dev)[0]], dtype=torch.int64, device=dev)
        dist.all_reduce(free, op=dist.ReduceOp.MIN)
        if need > 0.8 * int(free.item()):
            return {"what": "skipped: the gathered C would not fit", "c_bytes": need,
                    "free_bytes_min": int(free.item())}
    mc, mcg = [], []
    full_nnz = full_rows = 0
    for _ in range(max(1, reps)):
        ms, _ = timed(step)
        mc.append(ms)
        ms, full = timed(compute_and_gather)
        mcg.append(ms)
        full_rows, full_nnz = int(full[0].numel()) - 1, int(full[1].numel())
        del full
    rows_local, nnz_local = int(c_rp.numel()) - 1, int(c_ci.numel())
    rv = torch.tensor([12 * (full_nnz - nnz_local) + 8 * (full_rows - rows_local)], dtype=torch.int64, device=dev)
    dist.all_reduce(rv, op=dist.ReduceOp.MAX)
    recv = int(rv.item())
    ms_c, ms_cg = min(mc), min(mcg)
    ms_g = max(ms_cg - ms_c, 1e-6)
    return {"what": "one step compute-only vs compute + RCCL allgatherv of C on every rank "
                    "(ias/dist.py gather_csr), max over ranks, best of reps",
            "reps": max(1, reps), "ms_compute": round(ms_c, 3), "ms_compute_allgatherv": round(ms_cg, 3),
            "ms_allgatherv": round(ms_g, 3), "c_nnz_total": full_nnz,
            "bytes_received_per_rank_max": recv,
            "gbps_received_per_rank": round(recv / (ms_g * 1e-3) / 1e9, 1)}


def row_sample(A, every):
    """Every `every`-th block of 4096 rows of A (spread over the matrix, hub rows
    included), as one CSR: the bounded sample the CPU baselines run when the
    full product is beyond the budget (or beyond MKL LP64's 2^31 entries)."""
    import ias
    if every <= 1:
        return A
    blocks = [(r, min(r + 4096, A.rows)) for r in range(0, A.rows, 4096 * every)]
    rp = [np.zeros(1, np.int64)]
    cols, vals, base = [], [], 0
    for r0, r1 in blocks:
        s, e = int(A.row_ptr[r0]), int(A.row_ptr[r1])
        rp.append(A.row_ptr[r0 + 1:r1 + 1] - s + base)
        cols.append(A.col[s:e])
        vals.append(A.val[s:e])
        base += e - s
    return ias.HostCsr(sum(r1 - r0 for r0, r1 in blocks), A.cols, np.concatenate(rp),
                       np.concatenate(cols), np.concatenate(vals))


def cpu_baseline(A, flops_total, threads, full=False):
    """The reference's Algorithm 1 (MKL mkl_sparse_sp2m, create+multiply+export
    as main.cpp:746-748) on the host cores: 1 warm-up + median of 3 runs.  The
    full matrix when its product is small enough for a bounded run (or with
    full=True: --cpu-full, ILP64 indices since K3's nnz(C) exceeds 2^31, as the
    reference's own build needs there); otherwise a row sample (row_sample)
    times B = A, reported per its own flops."""
    import ias
    if full:
        os.environ["IAS_MKL_ILP64"] = "1"   # read when MKL is first loaded (mkl_baseline.cpp)
    ok, ver = ias.mkl_available()
    if not ok:
        return {"value": None, "unit": "GFLOP/s", "cores": 0, "kind": "reference",
                "sample": "MKL runtime not present on this host"}
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    every = 1 if (full or flops_total <= 1_200_000_000) else int(math.ceil(flops_total / 3e8))
    As = row_sample(A, every)
    f_s = ias.flops(As, A)
    times = []
    sa, sb = As.struct(), A.struct()
    for i in range(4):
        cm, ms = ias.Csr(), C.c_double(0)
        ias.check(ias.lib.ias_mkl_sp2m(C.byref(sa), C.byref(sb), C.byref(cm), threads, C.byref(ms)),
                  "ias_mkl_sp2m")
        ias.lib.ias_csr_free(C.byref(cm))
        if i:
            times.append(ms.value)
    med = statistics.median(times)
    what = "full matrix" if every == 1 else \
        f"row sample: every {every}th block of 4096 rows ({As.rows} rows, {f_s} of {flops_total} flops) x full B"
    return {"value": round(2.0 * f_s / (med * 1e6), 4), "unit": "GFLOP/s", "cores": threads,
            "kind": "reference",
            "sample": f"{what}, MKL mkl_sparse_sp2m FULL_MULT (reference Algorithm 1, "
                      f"csr/common_csr.h:18-47), {ver.split(' Product')[0]}, "
                      f"{'ILP64' if os.environ.get('IAS_MKL_ILP64') == '1' else 'LP64'}, GNU threading, "
                      f"median of 3 after 1 warm-up: {med:.1f} ms",
            "ms": round(med, 2)}


def cpu_baseline_alg2(A, flops_total, threads):
    """The reference's Algorithm 2 (CSR_MUL_CSR, csr/common_csr.h:85-193: per-
    thread dense SPA, two passes, OpenMP over rows) as restated by the oracle
    (oracle/ias_oracle.c, the test-infrastructure CPU port; used here only as
    the timed CPU baseline), on `threads` host threads: 1 warm-up + median of 3."""
    os.environ["OMP_NUM_THREADS"] = str(threads)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    try:
        import oracle_bind as ob
    except Exception as e:  # oracle not built on this host
        return {"value": None, "unit": "GFLOP/s", "cores": 0, "kind": "port", "sample": f"unavailable: {e}"}
    every = 1 if flops_total <= 1_000_000_000 else int(math.ceil(flops_total / 2.5e8))
    As = row_sample(A, every)
    import ias
    f_s = ias.flops(As, A)
    Ma, Mb = ob.Mat.of(As), ob.Mat.of(A)
    times = []
    for i in range(4):
        t = time.perf_counter()
        c = ob.csr_mul_csr(Ma, Mb)
        times.append((time.perf_counter() - t) * 1e3)
        del c
    med = statistics.median(times[1:])
    what = "full matrix" if every == 1 else \
        f"row sample: every {every}th block of 4096 rows ({f_s} of {flops_total} flops) x full B"
    return {"value": round(2.0 * f_s / (med * 1e6), 4), "unit": "GFLOP/s", "cores": threads, "kind": "port",
            "sample": f"{what}; reference Algorithm 2 CSR_MUL_CSR semantics (OpenMP restatement, "
                      f"oracle/ias_oracle.c ora_csr_mul_csr, incl. copy-out to numpy), median of 3 after "
                      f"1 warm-up: {med:.1f} ms",
            "ms": round(med, 2)}


if __name__ == "__main__":
    main()
