#!/usr/bin/env python3
"""SURVEY §8 e1's exchange step on its own: the row-sharded C = A·A of
bench.py's workload, then per repetition one step compute-only and one step
compute + the RCCL allgatherv that concatenates C on every rank
(ias/dist.py gather_csr), max over ranks.  One process per GPU:

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port 29511 tools/gather_bench.py --gpus 8

Prints bench.py's JSON line (its `allgatherv` object holds the figures);
extra arguments go to bench.py (e.g. --config k4, --gather-reps 5)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

if __name__ == "__main__":
    argv = sys.argv[1:]
    defaults = ["--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-host-e2e"]
    if "--gather-reps" not in argv:
        defaults += ["--gather-reps", "3"]
    if int(os.environ.get("WORLD_SIZE", "1")) < 2:
        sys.exit("gather_bench.py needs one process per GPU (WORLD_SIZE >= 2, torch.distributed.run)")
    bench.main(defaults + argv)
