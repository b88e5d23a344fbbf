#!/usr/bin/env python3
"""HBM traffic per launch of the fused tick kernel from rocprofv3 PMC passes.

    python scripts/pmc_traffic.py <pmc_fetch.csv> <pmc_write.csv> [out.json] [--pview] [--tiles T]

--pview: the partial-view tick kernels (8-B/lane view loads and stores; per tick the
256-lane and the 128-lane split kernel, summed) instead of the full-view fused tick kernel.  --tiles T: the full view ran as T column tiles (T launches per
tick); bytes_per_tick = T x the per-launch average.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts half of
the bytes of a wide (16 B/lane) coalesced streaming read, which is every load of this
kernel, so it is doubled (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for
16-B-per-lane stores.
"""
import csv
import json
import sys

KERNEL = "scale_tick_kernel<false"
NOTE = "FETCH_SIZE x2 (gfx950 counts half of 16-B/lane streaming reads)"


ANCHOR = None   # --pview: one dispatch of this kernel per tick; the tick's kernels are summed


def per_launch(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    vals = [float(r["Counter_Value"]) for r in rows if KERNEL in r["Kernel_Name"]]
    if ANCHOR is None:
        return sum(vals) / len(vals), len(vals)
    ticks = sum(1 for r in rows if ANCHOR in r["Kernel_Name"])
    return sum(vals) / ticks, ticks


def main():
    global KERNEL, NOTE, ANCHOR
    name = "scale_tick_kernel (fused merge/ops/send)"
    if "--pview" in sys.argv:
        sys.argv.remove("--pview")
        KERNEL = "pview_tick_split_kernel<0, "
        ANCHOR = "pview_tick_split_kernel<0, 128, 0, 3,"
        name = ("pview_tick_split_kernel (partial-view union/fold/evict; per tick: the 256-lane and "
                "the 128-lane kernel summed)")
        NOTE = ("FETCH_SIZE x2 (the gfx950 16-B/lane rule applied to this kernel's 8-B/lane view "
                "loads: uncalibrated for that width, MI355X_MICROARCH.md HBM section)")
    tiles = 1
    if "--tiles" in sys.argv:
        i = sys.argv.index("--tiles")
        tiles = int(sys.argv[i + 1])
        del sys.argv[i:i + 2]
    fetch, n1 = per_launch(sys.argv[1], "FETCH_SIZE")
    write, n2 = per_launch(sys.argv[2], "WRITE_SIZE")
    out = {
        "kernel": name,
        "launches": min(n1, n2),
        "fetch_size_kib_raw": fetch,
        "write_size_kib": write,
        "read_bytes_per_launch": fetch * 1024 * 2,
        "write_bytes_per_launch": write * 1024,
        "bytes_per_launch": fetch * 1024 * 2 + write * 1024,
        "launches_per_tick": tiles,
        "bytes_per_tick": (fetch * 1024 * 2 + write * 1024) * tiles,
        "correction": NOTE,
    }
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
