#!/usr/bin/env python3
"""Kernel-time cost of the device event stream (gsp_*_params.events) on one box.

Config 3 (full view, 65,536 nodes) with events off / on interleaved, each run ticks 1..T with
the mean tick-kernel time over ticks W+1..T (HIP events, gsp_scale_perf); then config 5's
per-tick event volume (digest joins / removes / evicts) and its tick-kernel time with events
on.  Prints one JSON line per measurement.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def full(events, ticks=45, warm=5):
    from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine
    kw = dict(fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000, seed=0x5EED,
              max_ticks=ticks)
    if events:
        kw.update(events=True, event_cap=1 << 27)
    with ScaleEngine(65536, **kw) as e:
        e.step(warm)
        e.sync()
        p0 = e.perf()
        e.step(ticks - warm)
        e.sync()
        p1 = e.perf()
        out = {"item": "config3", "events": events,
               "kernel_ms": (p1["merge_ms"] - p0["merge_ms"]) / (p1["merge_launches"] - p0["merge_launches"])}
        if events:
            rec, lost = e.drain_events()
            out.update(records=len(rec), lost=lost)
        return out


def pview(events, ticks=14, warm=10):
    """events: False, True (every kind) or a kind mask (gsp_pview_params.events)."""
    from gossip_protocol_amd.pview import PviewEngine
    kw = dict(view=256, fanout=3, inbox=7, drop_pct=10, fail_mode=2, fail_tick=10, fail_ppm=50000,
              seed=0x5EED, max_ticks=ticks)
    if events:
        kw.update(events=True, event_cap=1 << 28)
    with PviewEngine(1 << 20, **kw) as e:
        e.step(warm)
        e.sync()
        if events:
            e.drain_events()
        p0 = e.perf()
        e.step(ticks - warm)
        e.sync()
        p1 = e.perf()
        d = [e.digest(t) for t in range(warm + 1, ticks + 1)]
        out = {"item": "config5", "events": events,
               "kernel_ms": (p1["merge_ms"] - p0["merge_ms"]) / (p1["merge_launches"] - p0["merge_launches"]),
               "joins_per_tick": sum(x["joins"] for x in d) / len(d),
               "removes_per_tick": sum(x["removes"] for x in d) / len(d),
               "evicts_per_tick": sum(x["evicts"] for x in d) / len(d)}
        if events:
            rec, lost = e.drain_events()
            out.update(records=len(rec), lost=lost)
        return out


if __name__ == "__main__":
    which = sys.argv[1:] or ["full", "pview"]
    if "full" in which:
        for ev in (False, True, False, True):
            print(json.dumps(full(ev)), flush=True)
    if "pview" in which:
        for ev in (False, True, 4, False, True, 4):
            print(json.dumps(pview(ev)), flush=True)
