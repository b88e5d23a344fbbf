#!/usr/bin/env python3
"""Config-3 tick-kernel time vs extra dynamic LDS per workgroup (GSP_TEST_SCALE_LDS_PAD), events
off, interleaved on one box: does fewer resident workgroups per CU change the HBM rate?
usage: python scripts/ab_scale_pad.py 0 8192 16384 ... (each run in a child process)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys
sys.path.insert(0, %r)
from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine
with ScaleEngine(65536, fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000,
                 seed=0x5EED, max_ticks=30) as e:
    e.step(5); e.sync(); p0 = e.perf(); e.step(25); e.sync(); p1 = e.perf()
print(json.dumps({"pad": int(os.environ.get("GSP_TEST_SCALE_LDS_PAD", "0")),
                  "kernel_ms": (p1["merge_ms"] - p0["merge_ms"]) / (p1["merge_launches"] - p0["merge_launches"])}))
''' % ROOT

if __name__ == "__main__":
    for rep in range(2):
        for pad in sys.argv[1:]:
            env = dict(os.environ, GSP_TEST_SCALE_LDS_PAD=pad)
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                               timeout=120)
            print(r.stdout.strip() or r.stderr[-500:], flush=True)
