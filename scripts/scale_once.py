#!/usr/bin/env python3
"""One full-view engine run in this process (no child: safe under rocprofv3 --pmc), as
scripts/ab_scale_tiles.py's child: AB_N nodes as AB_G in-process column tiles, AB_W warm-up then
AB_S timed ticks; prints the tick kernels' ms per launch / per tick and the tick's event hash.
    AB_N=262144 AB_G=32 AB_W=2 AB_S=8 python3 scripts/scale_once.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine  # noqa: E402

N, G = int(os.environ.get("AB_N", 65536)), int(os.environ.get("AB_G", 8))
W, S = int(os.environ.get("AB_W", 5)), int(os.environ.get("AB_S", 20))
with ScaleEngine(N, fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000,
                 seed=0x5EED, max_ticks=W + S + 2, group=G) as e:
    e.step(W)
    e.sync()
    p0 = e.perf()
    e.step(S)
    e.sync()
    p1 = e.perf()
    d = e.digest(W + S)
launches = p1["merge_launches"] - p0["merge_launches"]
ms = p1["merge_ms"] - p0["merge_ms"]
print(json.dumps({"ms_per_launch": ms / launches, "kernel_ms_per_tick": ms / S,
                  "hash": d["event_hash"] if isinstance(d, dict) else None}), flush=True)
