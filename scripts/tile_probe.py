#!/usr/bin/env python3
"""Where does the column-sliced tick kernel gain over the fused one (config 3, one GPU)?
fused (G = 1), sliced G = 1 (the RCCL rank path with a world of one: slice kernel + resolve),
and in-process column groups G = 2, 4, 8; tick-kernel ms (summed over shards) and wall ms per
tick, interleaved twice."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(kind, g):
    import torch
    from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine, nccl_unique_id
    kw = dict(fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000, seed=0x5EED, max_ticks=25)
    if kind == "sliced1":
        kw.update(rank=0, world=1, nccl_id=nccl_unique_id())
    else:
        kw.update(group=g)
    with ScaleEngine(65536, **kw) as e:
        e.step(5); e.sync(); p0 = e.perf()
        torch.cuda.synchronize(); t0 = time.perf_counter()
        e.step(20); e.sync()
        el = time.perf_counter() - t0
        p1 = e.perf()
        n = p1["merge_launches"] - p0["merge_launches"]
        return {"kind": kind, "group": g, "wall_ms": el * 50.0,
                "kernel_ms_per_tick": (p1["merge_ms"] - p0["merge_ms"]) / 20.0, "launches": n}


if __name__ == "__main__":
    for rep in range(2):
        for kind, g in (("fused", 1), ("sliced1", 1), ("group", 2), ("group", 4), ("group", 8)):
            print(json.dumps(run(kind, g)), flush=True)
