#!/usr/bin/env python3
"""Strong-scaling probe on ONE GPU: config 3 as G in-process column shards (the kernels and
exchange of the G-GPU run, shards launched back to back on one device).  Per-shard kernel
time ~ what each of G GPUs would spend per tick; the exchange here is device copies, not RCCL.

    python scripts/scaling_probe.py [--nodes 65536] [--groups 1 2 4 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=65536)
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--layout", default="columns")
    args = ap.parse_args()
    import torch
    from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine
    for g in args.groups:
        with ScaleEngine(args.nodes, fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000,
                         seed=0x5EED, max_ticks=20, group=g, layout=args.layout) as eng:
            eng.step(5)
            eng.sync()
            p0 = eng.perf()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.step(10)
            eng.sync()
            el = time.perf_counter() - t0
            p1 = eng.perf()
            launches = max(p1["merge_launches"] - p0["merge_launches"], 1)
            merge = (p1["merge_ms"] - p0["merge_ms"]) / launches
            csr = (p1["csr_ms"] - p0["csr_ms"]) / launches
            print(json.dumps({"group": g, "layout": args.layout, "ms_per_tick": el * 100.0,
                              "kernels_ms_per_tick": merge, "per_shard_kernel_ms": merge / g,
                              "csr_ms": csr}), flush=True)


if __name__ == "__main__":
    main()
