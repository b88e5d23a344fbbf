#!/usr/bin/env python3
"""Config 3 (65,536 full view) as G in-process column tiles for a few ticks: the program a
rocprofv3 PMC pass wraps to compare tile widths (G = 1 is the fused row kernel).

    python scripts/tile_run.py <G> [--nodes N] [--ticks T] [--warmup W]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("group", type=int)
    ap.add_argument("--nodes", type=int, default=65536)
    ap.add_argument("--ticks", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=4)
    a = ap.parse_args()
    from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine
    with ScaleEngine(a.nodes, fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000,
                     seed=0x5EED, max_ticks=a.warmup + a.ticks, group=a.group) as e:
        e.step(a.warmup)
        e.sync()
        p0 = e.perf()
        e.step(a.ticks)
        e.sync()
        p1 = e.perf()
        print(json.dumps({"group": a.group, "nodes": a.nodes, "layout": e.layout(),
                          "kernel_ms_per_tick": (p1["merge_ms"] - p0["merge_ms"]) / a.ticks}))


if __name__ == "__main__":
    main()
