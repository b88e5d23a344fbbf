#!/usr/bin/env python3
"""PMC counters of a tick window from rocprofv3 counter CSVs (every
derived number labelled with its window, and taken over that window only).

    python scripts/pmc_window.py <counter_collection.csv>... --anchor <substr> --ticks A B
                                 --kernels <substr>[,<substr>...] [--json out]

Dispatches are taken in Dispatch_Id order per counter; the i-th dispatch of the anchor kernel
(one per tick, e.g. the CSR scan or the receipt kernel) opens tick i, so a dispatch belongs to
the tick of the last anchor before it.  Counters of the dispatches whose kernel name matches
any --kernels substring are summed over ticks A..B and divided by the number of ticks.
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]

    def opt(name, n=1):
        i = args.index(name)
        v = args[i + 1:i + 1 + n]
        del args[i:i + 1 + n]
        return v
    out = opt("--json")[0] if "--json" in args else None
    anchor = opt("--anchor")[0]
    a, b = (int(x) for x in opt("--ticks", 2))
    kerns = opt("--kernels")[0].split(",")
    rows = defaultdict(list)               # counter -> [(dispatch, kernel, value, start, end)]
    for p in args:
        for r in csv.DictReader(open(p)):
            rows[r["Counter_Name"]].append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                                            float(r["Counter_Value"]), int(r["Start_Timestamp"]),
                                            int(r["End_Timestamp"])))
    res = {}
    for c, lst in sorted(rows.items()):
        lst.sort()
        tick, tot, n, ns = 0, 0.0, 0, 0
        for _, name, v, s, e in lst:
            if anchor in name:
                tick += 1
            if a <= tick <= b and any(k in name for k in kerns):
                tot += v
                n += 1
                ns += e - s
        res[c] = {"per_tick": tot / (b - a + 1), "dispatches": n, "ticks": [a, b],
                  "dispatch_ms_per_tick_under_pmc": ns / 1e6 / (b - a + 1)}
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump({"anchor": anchor, "kernels": kerns, "window_ticks": [a, b], "counters": res}, f,
                      indent=1)


if __name__ == "__main__":
    main()
