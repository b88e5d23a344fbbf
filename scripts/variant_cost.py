#!/usr/bin/env python3
"""Cost of the protocol-variant flags of the fused tick kernel at BASELINE config 3.

One engine per variant (65,536 full view, fanout 3, 1% random crash at t=10), warm-up ticks
1-5, then the mean fused-kernel time over ticks 6-25 (HIP events on the engine stream,
gsp_scale_perf_get) and the algorithmic GB/s of the plain per-message model.
    python scripts/variant_cost.py [n] [ticks]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine  # noqa: E402

VARIANTS = {"plain": {}, "tfail5": {"tfail": 5}, "swim2": {"swim": 2},
            "tfail5_swim2": {"tfail": 5, "swim": 2}}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    out = {}
    for name, kw in VARIANTS.items():
        with ScaleEngine(n, fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000,
                         seed=0x5EED, max_ticks=5 + ticks, **kw) as eng:
            stride = eng.layout()[2]
            eng.step(5)
            eng.sync()
            before = eng.perf()
            eng.step(ticks)
            eng.sync()
            after = eng.perf()
            ms = after["merge_ms"] - before["merge_ms"]
            launches = after["merge_launches"] - before["merge_launches"]
            byts, removes = 0.0, 0
            for t in range(6, 6 + ticks):
                d = eng.digest(t)
                byts += (2.0 * d["node_rounds"] + d["delivered"]) * stride * 2 + d["delivered"] * 4
                removes += d["removes"]
            out[name] = {"ms_per_launch": ms / launches, "GBps": byts / (ms * 1e-3) / 1e9,
                         "removes": removes}
        print(name, json.dumps(out[name]), flush=True)
    print(json.dumps({"n": n, "ticks": ticks, "variants": out}))


if __name__ == "__main__":
    main()
