#!/usr/bin/env python3
"""Per-launch averages of every PMC counter of one kernel from rocprofv3 counter CSVs.

    python scripts/pmc_summary.py <kernel-substring> <run_counter_collection.csv>... [--json out]
                                  [--per-tick <anchor-substring>]

--per-tick: every kernel matching the substring is summed and divided by the dispatches of the
anchor kernel (one per tick): the partial view's two split tick kernels as one per-tick figure.
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    out = None
    if "--json" in args:
        i = args.index("--json")
        out = args[i + 1]
        del args[i:i + 2]
    anchor = None
    if "--per-tick" in args:        # sum every matching kernel, per dispatch of the anchor kernel
        i = args.index("--per-tick")
        anchor = args[i + 1]
        del args[i:i + 2]
    kern, paths = args[0], args[1:]
    vals = defaultdict(list)
    ticks = defaultdict(int)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if kern in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if anchor is not None and anchor in r["Kernel_Name"]:
                ticks[r["Counter_Name"]] += 1
    if anchor is None:
        res = {c: {"per_launch": sum(v) / len(v), "launches": len(v)} for c, v in sorted(vals.items())}
    else:
        res = {c: {"per_launch": sum(v) / ticks[c], "launches": ticks[c]}
               for c, v in sorted(vals.items()) if ticks[c]}
    for c, d in res.items():
        print("%-26s %18.1f  (%d launches)" % (c, d["per_launch"], d["launches"]))
    if out:
        open(out, "w").write(json.dumps({"kernel": kern, "counters": res}, indent=1) + "\n")


if __name__ == "__main__":
    main()
