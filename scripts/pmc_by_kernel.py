#!/usr/bin/env python3
"""Per-launch averages of every PMC counter, per kernel INSTANCE (full template name), from
rocprofv3 counter CSVs; kernels whose name contains any of the given substrings.

    python scripts/pmc_by_kernel.py <substring>[,<substring>...] <counter_collection.csv>... [--json out]

Also prints, per instance, the derived ratios used in DESIGN.md: LDS bank-conflict cycles per
LDS-active cycle, waits for LDS per wave cycle, SALU and branch instructions per VALU one.
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
    subs, paths = args[0].split(","), args[1:]
    vals = defaultdict(lambda: defaultdict(list))     # kernel -> counter -> per-dispatch values
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            if any(s in name for s in subs):
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k in sorted(vals):
        c = {n: {"per_launch": sum(v) / len(v), "launches": len(v)} for n, v in sorted(vals[k].items())}
        g = lambda n: c.get(n, {}).get("per_launch")
        ratios = {}
        for name, a, b in (("lds_conflict_per_lds_active", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
                           ("wait_lds_per_wave_cycle", "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES"),
                           ("salu_per_valu", "SQ_INSTS_SALU", "SQ_INSTS_VALU"),
                           ("branch_per_valu", "SQ_INSTS_BRANCH", "SQ_INSTS_VALU"),
                           ("l2_hit_rate", "TCC_HIT_sum", None)):
            if b is None:
                h, m = g("TCC_HIT_sum"), g("TCC_MISS_sum")
                if h is not None and m is not None and h + m > 0:
                    ratios[name] = h / (h + m)
            elif g(a) is not None and g(b):
                ratios[name] = g(a) / g(b)
        res[k] = {"counters": c, "ratios": ratios}
        print(k)
        for n, d in c.items():
            print("   %-26s %18.1f  (%d launches)" % (n, d["per_launch"], d["launches"]))
        for n, v in ratios.items():
            print("   %-26s %18.4f" % (n, v))
    if out:
        open(out, "w").write(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
