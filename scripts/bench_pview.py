#!/usr/bin/env python3
"""BASELINE config 5 (partial view) alone: the `pview` line item of bench.py.

    python scripts/bench_pview.py [--nodes 1048576] [--steps K] [--warmup W] [--no-cpu-baseline]
                                  [--inbox 0]
    python -m torch.distributed.run --nproc-per-node N scripts/bench_pview.py ...   (row shards)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import PV_NODES, run_pview  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=PV_NODES)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inbox", type=int, default=None, help="0: drain all (default: bench.PV_KW's 7)")
    ap.add_argument("--group", type=int, default=1,
                    help="G row shards inside this process on one GPU (exchange by device copies)")
    args = ap.parse_args()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    out = run_pview(args.nodes, args.steps, args.warmup, world, local, dist,
                    not args.no_cpu_baseline, group=args.group, inbox=args.inbox)
    if out is not None:
        print(json.dumps(dict(out, n_gpus=world, steps=args.steps, warmup=args.warmup)), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
