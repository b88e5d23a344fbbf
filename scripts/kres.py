#!/usr/bin/env python3
"""Per-kernel resource usage of one HIP source (VGPRs, SGPRs, spills, occupancy, LDS), from
hipcc's -Rpass-analysis=kernel-resource-usage remarks -- a quick check that a change to a hot
kernel did not cost registers or occupancy.

    python scripts/kres.py gossip_protocol_amd/csrc/scale_kernels.hip [filter] [-D...]
"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    filt = next((a for a in sys.argv[2:] if not a.startswith("-")), "")
    extra = [a for a in sys.argv[2:] if a.startswith("-")]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude",
           "-Igossip_protocol_amd/csrc", "-c", src, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: +([A-Za-z /\[\]]+?): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    for r in rows:
        if filt in r["name"]:
            print("%-4s vgpr %3s sgpr %3s spillv %3s spills %3s occ %s lds %6s  %s" % (
                "", r.get("VGPRs"), r.get("TotalSGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
                r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]"), r["name"][:110]))


if __name__ == "__main__":
    main()
