#!/usr/bin/env python3
"""profiles/pmc_traffic.json from the two passes of scripts/pmc_c3.sh: config 3's HBM bytes per
tick = FETCH_SIZE x 2 + WRITE_SIZE (the gfx950 correction for 16-B/lane streaming reads,
MI355X_MICROARCH.md HBM section), summed over the 8 column-tile launches of
scale_tick_kernel<false ...> in each of ticks 6-25 (tile_scan_kernel opens a tick).

    python scripts/pmc_c3_json.py gpurun_out/<tag> [--out profiles]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ANCHOR = "tile_scan_kernel"
KERNEL = "scale_tick_kernel<false"
TICKS = (6, 25)


def per_tick(path, counter):
    rows = []
    for p in glob.glob(os.path.join(path, "*counter_collection.csv")):
        rows += [r for r in csv.DictReader(open(p)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    tick, tot, n = 0, 0.0, defaultdict(int)
    for r in rows:
        if ANCHOR in r["Kernel_Name"]:
            tick += 1
        if TICKS[0] <= tick <= TICKS[1] and KERNEL in r["Kernel_Name"]:
            tot += float(r["Counter_Value"])
            n[tick] += 1
    return tot / (TICKS[1] - TICKS[0] + 1), (max(n.values()) if n else 0)


def main():
    src = sys.argv[1]
    dst = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(src, "json")
    os.makedirs(dst, exist_ok=True)
    fetch, launches = per_tick(os.path.join(src, "pmc_c3_FETCH_SIZE"), "FETCH_SIZE")
    write, _ = per_tick(os.path.join(src, "pmc_c3_WRITE_SIZE"), "WRITE_SIZE")
    rd, wr = fetch * 1024 * 2, write * 1024
    tag = os.path.basename(os.path.normpath(src))
    json.dump({"kernel": "scale_tick_kernel (8 column-tile launches per tick, config 3)",
               "window_ticks": list(TICKS), "launches_per_tick": launches,
               "fetch_size_kib_per_tick_raw": fetch, "write_size_kib_per_tick": write,
               "read_bytes_per_tick": rd, "write_bytes_per_tick": wr, "bytes_per_tick": rd + wr,
               "bytes_per_launch": (rd + wr) / max(1, launches),
               "correction": "FETCH_SIZE x2 (gfx950 counts half of 16-B/lane streaming reads)",
               "source": "profiles/r06/%s (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one pass each, "
                         "scripts/pmc_c3.sh)" % tag},
              open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    print("launches/tick %d bytes/tick %.4g" % (launches, rd + wr))


if __name__ == "__main__":
    main()
