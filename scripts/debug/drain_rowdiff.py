"""Debug: step GPU and oracle in lock-step and report the rows whose views differ (with the
row's in-degree at that tick)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gossip_protocol_amd.pview import PviewEngine, unpack_view
from tests.oracle_binding import PviewOracle

n, V, f = 2000, 32, 8
kw = dict(view=V, fanout=f, inbox=0, drop_pct=10, fail_mode=1, fail_tick=6, fail_ppm=30000, seed=41,
          tfail=int(os.environ.get("TF", "5")), swim=int(os.environ.get("SW", "0")))
ticks = int(os.environ.get("TICKS", "16"))
orc = PviewOracle(n, **kw)
with PviewEngine(n, max_ticks=ticks, **kw) as eng:
    for t in range(1, ticks + 1):
        src, dst = orc.messages()
        deg = np.bincount(dst, minlength=n)
        want = orc.step(); eng.step(1); got = eng.digest(t)
        bad = []
        for r in range(n):
            io, ho, to = orc.row(r)
            buf, ln = eng.row(r)
            i, h, s5 = unpack_view(buf, ln)
            if ln != len(io) or not (np.array_equal(i, io) and np.array_equal(h, ho) and np.array_equal(s5, to & 31)):
                bad.append(r)
        print("tick", t, "digest_ok", got == want, "bad rows", len(bad), flush=True)
        for r in bad[:6]:
            io, ho, to = orc.row(r); buf, ln = eng.row(r); i, h, s5 = unpack_view(buf, ln)
            so = set(io.tolist()); sg = set(i.tolist())
            print("  row", r, "deg", deg[r], "len gpu/orc", ln, len(io), "only gpu", sorted(sg - so)[:8],
                  "only orc", sorted(so - sg)[:8], flush=True)
            common = sorted(so & sg)
            for x in common:
                a = np.where(io == x)[0][0]; b = np.where(i == x)[0][0]
                if ho[a] != h[b] or (to[a] & 31) != s5[b]:
                    print("    id", x, "orc hb/ts", ho[a], to[a] & 31, "gpu", h[b], s5[b])
                    break
        if bad:
            break
