#!/usr/bin/env python3
"""Config-3 tick-kernel time under environment variants (GSP_LIB_VARIANT=<tag> of a
`make lib-variant` library, GSP_TEST_SCALE_POLICY, ...), each in its own child process, interleaved:
    python scripts/ab_scale_env.py base: nosend:GSP_LIB_VARIANT=nosend pol1:GSP_TEST_SCALE_POLICY=1
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys
sys.path.insert(0, %r)
from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine
with ScaleEngine(65536, fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000,
                 seed=0x5EED, max_ticks=25) as e:
    e.step(5); e.sync(); p0 = e.perf(); e.step(20); e.sync(); p1 = e.perf()
print(json.dumps({"kernel_ms": (p1["merge_ms"] - p0["merge_ms"]) / (p1["merge_launches"] - p0["merge_launches"])}))
''' % ROOT

if __name__ == "__main__":
    for rep in range(2):
        for spec in sys.argv[1:]:
            name, _, envs = spec.partition(":")
            env = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                               timeout=150)
            out = r.stdout.strip().splitlines()
            print(name, out[-1] if out else r.stderr[-400:], flush=True)
