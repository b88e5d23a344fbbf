#!/usr/bin/env python3
"""Config 5 drained, one engine in this process (safe under rocprofv3): PV_SWIM / PV_TFAIL /
PV_EVENTS from the environment, ticks 1-25; prints the tick-kernel ms per tick over 6-25.
    PV_SWIM=2 PV_TFAIL=5 PV_EVENTS=4 python3 scripts/pv_variant_trace.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from gossip_protocol_amd.pview import PviewEngine  # noqa: E402

kw = dict(bench.PV_KW, max_ticks=26, swim=int(os.environ.get("PV_SWIM", 0)),
          tfail=int(os.environ.get("PV_TFAIL", 0)))
ev = int(os.environ.get("PV_EVENTS", 0))
if ev:
    kw.update(events=ev, event_cap=bench.EVENT_CAP)
with PviewEngine(bench.PV_NODES, **kw) as e:
    e.step(5)
    e.sync()
    if ev:
        e.drain_events()
    p0 = e.perf()
    for _ in range(4):
        e.step(5)
        e.sync()
        if ev:
            e.drain_events()
    p1 = e.perf()
    st = e.drain_stats()
ms = (p1["merge_ms"] - p0["merge_ms"]) / 20
print(json.dumps({"kernel_ms_per_tick": ms, "drain_ms": [x / 25 for x in st["ms"]]}), flush=True)
