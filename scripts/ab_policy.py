#!/usr/bin/env python3
"""A/B variants of the fused tick kernel at BASELINE config 3 (65,536 full view).

Variants = (merge form, cache policy).  They are interleaved tick-pair by tick-pair on one
engine (same tables, same protocol phase); prints the mean fused-kernel time and achieved
algorithmic GB/s per variant.
    python scripts/ab_policy.py [n] [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine  # noqa: E402

VARIANTS = [("scalar", 0, 0), ("scalar", 0, 1), ("packed", 1, 0), ("packed", 1, 1),
            ("packed", 1, 3), ("packed", 1, 5)]     # policy bit 2: pipelined chunk loads


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    res = {v: [0.0, 0.0, 0] for v in VARIANTS}
    with ScaleEngine(n, fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000,
                     seed=0x5EED, max_ticks=6 + reps * len(VARIANTS) * 2) as eng:
        stride = eng.layout()[2]
        eng.step(6)
        eng.sync()
        for _ in range(reps):
            for v in VARIANTS:
                eng.set_merge(v[1])
                eng.set_cache_policy(v[2])
                before = eng.perf()
                t0 = eng.tick
                eng.step(2)
                eng.sync()
                after = eng.perf()
                byts = 0.0
                for t in range(t0 + 1, t0 + 3):
                    d = eng.digest(t)
                    byts += (2.0 * d["node_rounds"] + d["delivered"]) * stride * 2 + d["delivered"] * 4
                res[v][0] += after["merge_ms"] - before["merge_ms"]
                res[v][1] += byts
                res[v][2] += after["merge_launches"] - before["merge_launches"]
    out = {}
    for v, (ms, byts, launches) in res.items():
        out["%s/policy%d" % (v[0], v[2])] = {"ms_per_launch": ms / launches,
                                             "GBps": byts / (ms * 1e-3) / 1e9}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
