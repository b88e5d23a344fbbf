#!/usr/bin/env python3
"""Kernel-time cost of the device event stream (gsp_*_params.events) on one box.

Each measurement runs in its own child process (fresh allocations), interleaved and repeated
`--reps` times; the line per variant reports every run and the median.  Config 3 (full view,
65,536 nodes, 1 % crash at t = 10; ticks 6-45, the removals of the crash happen at t >= 30):
events off / every kind.  Config 5 (partial view, 1,048,576 nodes; ticks 11-14): off / every
kind / removes only, with the per-tick event volume from the digests.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys
sys.path.insert(0, %r)
item, events = sys.argv[1], int(sys.argv[2])
if item == "config3":
    from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine as E
    n, warm, ticks = 65536, 5, 45
    kw = dict(fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000, seed=0x5EED)
else:
    from gossip_protocol_amd.pview import PviewEngine as E
    n, warm, ticks = 1 << 20, 10, 14
    kw = dict(view=256, fanout=3, inbox=7, drop_pct=10, fail_mode=2, fail_tick=10, fail_ppm=50000,
              seed=0x5EED)
if events:
    kw.update(events=events, event_cap=1 << 28)
with E(n, max_ticks=ticks, **kw) as e:
    e.step(warm); e.sync()
    if events:
        e.drain_events()
    p0 = e.perf(); e.step(ticks - warm); e.sync(); p1 = e.perf()
    d = [e.digest(t) for t in range(warm + 1, ticks + 1)]
    out = {"item": item, "events": events,
           "kernel_ms": (p1["merge_ms"] - p0["merge_ms"]) / (p1["merge_launches"] - p0["merge_launches"]),
           "events_per_tick": sum(x["joins"] + x["removes"] + x.get("evicts", 0) for x in d) / len(d)}
    if events:
        rec, lost = e.drain_events()
        out.update(records=int(len(rec)), lost=int(lost))
print(json.dumps(out))
''' % ROOT


def run(item, events):
    r = subprocess.run([sys.executable, "-c", CHILD, item, str(events)], capture_output=True,
                       text=True, timeout=150)
    if r.returncode:
        raise RuntimeError(r.stderr[-800:])
    return json.loads(r.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("items", nargs="*", default=["config3", "config5"])
    args = ap.parse_args()
    variants = {"config3": [0, 1], "config5": [0, 1, 4]}
    for item in args.items:
        res = {v: [] for v in variants[item]}
        for _ in range(args.reps):
            for v in variants[item]:
                res[v].append(run(item, v))
                print(json.dumps(res[v][-1]), flush=True)
        base = statistics.median(r["kernel_ms"] for r in res[0])
        for v, rs in res.items():
            med = statistics.median(r["kernel_ms"] for r in rs)
            print(json.dumps({"item": item, "events": v, "median_kernel_ms": med,
                              "overhead_vs_off": med / base - 1.0,
                              "runs_ms": [round(r["kernel_ms"], 4) for r in rs]}), flush=True)
