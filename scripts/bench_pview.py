#!/usr/bin/env python3
"""BASELINE config 5 (partial view) on one GPU: node-rounds/s and the tick kernel's roofline.

    python scripts/bench_pview.py [--nodes 1048576] [--steps K] [--warmup W]

1,048,576 nodes, V = 256 entries per view (8 B each), fanout 3, inbox 7, 10% drops, a 5%
contiguous crash at t = 10.  Algorithmic bytes per node-round: own view read + write
(2 * V * 8) + one sender view per merged message (V * 8) + 4 B per CSR entry.
The CPU baseline is oracle/pview_oracle.c (1 thread) on n = 5000 with the same V, fanout,
inbox and drop rate: per-node work does not depend on n in a bounded view.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0
KW = dict(view=256, fanout=3, inbox=7, drop_pct=10, fail_mode=2, fail_tick=10, fail_ppm=50000,
          seed=0x5EED)


def cpu_baseline(budget_s=10.0):
    from tests.oracle_binding import PviewOracle
    o = PviewOracle(5000, **KW)
    t0 = time.perf_counter()
    ticks = rounds = 0
    while time.perf_counter() - t0 < budget_s and ticks < 40:
        rounds += o.step()["node_rounds"]
        ticks += 1
    el = time.perf_counter() - t0
    o.close()
    return {"value": rounds / el, "unit": "node-rounds/s", "cores": 1, "kind": "port",
            "sample": "oracle/pview_oracle.c, n=5000, V=256, %d ticks in %.1f s" % (ticks, el)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import torch
    from gossip_protocol_amd.pview import PviewEngine
    eng = PviewEngine(args.nodes, max_ticks=args.warmup + args.steps, **KW)
    eng.step(args.warmup)
    eng.sync()
    p0 = eng.perf()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step(args.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eng.sync()
    p1 = eng.perf()
    rounds = delivered = merges = csr = 0
    for t in range(args.warmup + 1, args.warmup + args.steps + 1):
        d = eng.digest(t)
        rounds += d["node_rounds"]
        delivered += d["delivered"]
        merges += d["merges"]
        csr += d["delivered"] + d["overflow"]
    V = KW["view"]
    launches = p1["merge_launches"] - p0["merge_launches"]
    kern_ms = (p1["merge_ms"] - p0["merge_ms"]) / max(launches, 1)
    bytes_per_launch = ((2.0 * rounds + delivered) * V * 8.0 + csr * 4.0) / args.steps
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    out = {
        "metric": "gossip node-rounds/sec (partial view)", "value": rounds / el,
        "unit": "node-rounds/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u64 entries (id:32 | hb:11 | ts5)",
        "data": "synthetic (ring-initialised bounded views, Philox peers/drops/failures)",
        "config": {"workload": "config5: %d nodes, partial view V=256, fanout 3, inbox 7, "
                               "10%% drop, 5%% contiguous crash at t=10" % args.nodes},
        "merges_per_s": merges / el,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": None, "kernel": "pview_tick_kernel",
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": bytes_per_launch},
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
