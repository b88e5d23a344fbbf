#!/usr/bin/env python3
"""In-degree skew of the partial view at config 5, per eviction order.

For each evict_order (0: (age, -hb, id), the default; 1: ties by the rotated id), runs BASELINE
config 5 (1,048,576 nodes, V = 256, fanout 3, inbox 7, 10 % drop, 5 % block crash at t = 10)
for --ticks ticks on one GPU and, at the sampled ticks, reads the message list of that tick
(sent at t, merged at t + 1) to report the in-degree of the alive receivers (max, p99, p99.9),
the k-bucket mix the tick kernel will see (k = min(in-degree, inbox); k = 7 holds every inbox
overflow), and the mean tick-kernel and CSR + receipt times of each window between samples
(HIP events, gsp_pview_perf_get).

    python scripts/pview_skew.py [--ticks 100] [--sample 25,50,75,100] [--orders 0,1] [--nodes N]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1 << 20)
    ap.add_argument("--ticks", type=int, default=100)
    ap.add_argument("--sample", default="25,50,75,100")
    ap.add_argument("--orders", default="0,1")
    ap.add_argument("--out", default="")
    ap.add_argument("--inbox", type=int, default=7, help="0: drain all")
    args = ap.parse_args()
    from gossip_protocol_amd import _lib
    from gossip_protocol_amd.pview import PviewEngine
    n = args.nodes
    fail = _lib.fail_schedule(n, 0x5EED, 2, 10, 50000)
    samples = [int(x) for x in args.sample.split(",")]
    out = {"nodes": n, "ticks": args.ticks, "orders": {}}
    for order in [int(x) for x in args.orders.split(",")]:
        rows = []
        with PviewEngine(n, view=256, fanout=3, inbox=args.inbox, drop_pct=10, fail_mode=2, fail_tick=10,
                         fail_ppm=50000, seed=0x5EED, max_ticks=args.ticks, evict_order=order) as eng:
            done, last = 0, eng.perf()
            for s in samples:
                eng.step(s - done)
                done = s
                p = eng.perf()
                ms = (p["merge_ms"] - last["merge_ms"]) / max(1, p["merge_launches"] - last["merge_launches"])
                csr = (p["csr_ms"] - last["csr_ms"]) / max(1, p["merge_launches"] - last["merge_launches"])
                last = p
                m = eng.messages()
                live = m[m >= 0]
                deg = np.bincount(live, minlength=n)
                d = deg[fail >= s + 1]                      # the receivers alive at s + 1
                k = np.minimum(d, 7)
                mix = np.bincount(k, minlength=8) / len(k)
                dg = eng.digest(s)
                lg = d[d > 7]
                rows.append({"tick": s, "long_rows": int(len(lg)), "long_msgs": int(lg.sum()),
                             "long_k_p50": float(np.percentile(lg, 50)) if len(lg) else 0.0,
                             "long_k_p99": float(np.percentile(lg, 99)) if len(lg) else 0.0,
                             "deg_max": int(d.max()), "deg_p99": float(np.percentile(d, 99)),
                             "deg_p999": float(np.percentile(d, 99.9)), "k_mix": [round(x, 4) for x in mix],
                             "overflow_frac": float(np.maximum(d - 7, 0).sum() / max(1, d.sum())),
                             "tick_kernel_ms": ms, "csr_receipt_ms": csr, "evicts": dg["evicts"],
                             "window": [(samples[samples.index(s) - 1] if samples.index(s) else 0) + 1, s]})
                print(json.dumps({"order": order, **rows[-1]}), flush=True)
        out["orders"][order] = rows
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
