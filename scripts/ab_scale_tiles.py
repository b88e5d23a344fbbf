#!/usr/bin/env python3
"""Config-3 headline form (8 in-process column tiles, as bench.py runs it) under library /
environment variants, each in its own child process, interleaved; per variant and run: the
tick kernels' ms per launch and per tick, and the CSR (+ segment order) ms per tick, over the
driver's window (ticks 6-25).
    python scripts/ab_scale_tiles.py [reps] base: nopre:GSP_LIB_VARIANT=nopresort
AB_N / AB_G / AB_W / AB_S (environment) change the nodes, tiles, warm-up and timed ticks
(config 4 as bench.py runs it: AB_N=262144 AB_G=32 AB_W=2 AB_S=8).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys
sys.path.insert(0, %r)
from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine
import os
N, G = int(os.environ.get("AB_N", 65536)), int(os.environ.get("AB_G", 8))
W, S = int(os.environ.get("AB_W", 5)), int(os.environ.get("AB_S", 20))
with ScaleEngine(N, fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000,
                 seed=0x5EED, max_ticks=W + S + 2, group=G) as e:
    e.step(W); e.sync(); p0 = e.perf(); e.step(S); e.sync(); p1 = e.perf()
    d = e.digest(W + S)
launches = p1["merge_launches"] - p0["merge_launches"]
ms = p1["merge_ms"] - p0["merge_ms"]
print(json.dumps({"ms_per_launch": ms / launches, "kernel_ms_per_tick": ms / S,
                  "csr_ms_per_tick": (p1["csr_ms"] - p0["csr_ms"]) / S,
                  "hash": d["event_hash"] if isinstance(d, dict) else None}))
''' % ROOT

if __name__ == "__main__":
    args = sys.argv[1:]
    reps = int(args.pop(0)) if args and args[0].isdigit() else 2
    for rep in range(reps):
        for spec in args:
            name, _, envs = spec.partition(":")
            env = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                               timeout=int(os.environ.get("AB_TIMEOUT", 240)))
            out = r.stdout.strip().splitlines()
            print(name, out[-1] if out else r.stderr[-600:], flush=True)
