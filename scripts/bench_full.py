#!/usr/bin/env python3
"""One full-view line item of bench.py alone (BASELINE config 3 or 4), e.g. for a rocprofv3
kernel trace per config (each frac in BENCH recomputes from one CSV line).

    python scripts/bench_full.py [--nodes 262144] [--steps 8] [--warmup 2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import run_full, summarize_full  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    r = run_full(a.nodes, a.steps, a.warmup, 1, 0, None)
    print(json.dumps(dict(summarize_full(r, a.nodes, a.steps, 1, a.warmup), steps=a.steps, warmup=a.warmup)),
          flush=True)


if __name__ == "__main__":
    main()
