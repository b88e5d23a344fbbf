#!/usr/bin/env python3
"""profiles/pmc_sq_pview.json and profiles/pmc_traffic_pview.json (--inbox 0, drain all: the
split kernels and the drain kernels) or pmc_*_pview_inbox7.json (--inbox 7: the split kernels)
from the three passes of scripts/pmc_pview.sh (ticks 6-25 of scripts/bench_pview.py --steps 20
--warmup 5: the driver's window): SQ issue counters per tick, and HBM bytes per tick =
FETCH_SIZE x 2 + WRITE_SIZE (the gfx950 correction for wide streaming reads, MI355X_MICROARCH.md
HBM section), summed over the partial-view tick kernels of each tick (the receipt kernel opens
a tick).

    python scripts/pmc_pview_json.py gpurun_out/<tag> [--out profiles] [--inbox 7]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ANCHOR = "pview_receipt_kernel"
KERNELS = ("pview_tick", "pview_drain")
TICKS = (6, 25)


def per_tick(path):
    rows = defaultdict(list)
    for p in glob.glob(os.path.join(path, "*counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            rows[r["Counter_Name"]].append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    out = {}
    for c, lst in rows.items():
        lst.sort()
        tick, tot = 0, 0.0
        for _, name, v in lst:
            if ANCHOR in name:
                tick += 1
            if TICKS[0] <= tick <= TICKS[1] and any(k in name for k in KERNELS):
                tot += v
        out[c] = tot / (TICKS[1] - TICKS[0] + 1)
    return out


def main():
    src = sys.argv[1]
    dst = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(src, "json")
    inbox = int(sys.argv[sys.argv.index("--inbox") + 1]) if "--inbox" in sys.argv else 0
    suffix = "" if inbox == 0 else "_inbox%d" % inbox
    what = ("the four split kernels and the drain kernels (inbox 0)" if inbox == 0 else
            "the four split kernels (inbox %d)" % inbox)
    os.makedirs(dst, exist_ok=True)
    sq = per_tick(os.path.join(src, "pmc_sq"))
    tag = os.path.basename(os.path.normpath(src))
    counters = {c: {"per_launch": v, "per_tick": v, "ticks": list(TICKS)} for c, v in sorted(sq.items())}
    json.dump({"kernel": "pview tick kernels (%s), per tick" % what, "window_ticks": list(TICKS),
               "source": "profiles/r06/%s (rocprofv3 --pmc, scripts/pmc_pview.sh + pmc_pview_json.py)" % tag,
               "counters": counters}, open(os.path.join(dst, "pmc_sq_pview%s.json" % suffix), "w"), indent=1)
    fetch = per_tick(os.path.join(src, "pmc_fetch"))["FETCH_SIZE"]
    write = per_tick(os.path.join(src, "pmc_write"))["WRITE_SIZE"]
    rd, wr = fetch * 1024 * 2, write * 1024
    json.dump({"kernel": "pview tick kernels (%s, per tick, config 5)" % what,
               "window_ticks": list(TICKS), "launches_per_tick": 1,
               "fetch_size_kib_per_tick_raw": fetch, "write_size_kib_per_tick": write,
               "read_bytes_per_tick": rd, "write_bytes_per_tick": wr, "bytes_per_tick": rd + wr,
               "bytes_per_launch": rd + wr,
               "correction": "FETCH_SIZE x2 (the gfx950 16-B/lane rule applied to this kernel's 8-B/lane view "
                             "loads: uncalibrated for that width, MI355X_MICROARCH.md HBM section)",
               "source": "profiles/r06/%s (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one pass each)" % tag},
              open(os.path.join(dst, "pmc_traffic_pview%s.json" % suffix), "w"), indent=1)
    print("VALU/tick %.4g SALU/tick %.4g bytes/tick %.4g" % (sq["SQ_INSTS_VALU"], sq["SQ_INSTS_SALU"], rd + wr))


if __name__ == "__main__":
    main()
