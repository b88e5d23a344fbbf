import numpy as np, collections
from gossip_protocol_amd import _lib
from gossip_protocol_amd.pview import PviewEngine
from gossip_protocol_amd.scale import make_policy
from tests.oracle_binding import PviewOracle
from tests.oracle_binding import make_policy as oracle_policy
POL = dict(drop_window=(3, 20), step_rate=0.02, intro_list=4, fail_events=[(10, 3, 0), (14, 2, 50000)])
n, V, f, K, drop = 1500, 48, 3, 5, 20
kw = dict(view=V, fanout=f, inbox=K, drop_pct=drop, fail_mode=1, fail_tick=6, fail_ppm=30000, seed=23, tremove=12)
orc = PviewOracle(n, policy=oracle_policy(**POL), **kw)
with PviewEngine(n, max_ticks=6, events=True, policy=make_policy(**POL), **kw) as eng:
    print("create", len(eng.drain_events()[0]))
    for t in range(1, 5):
        d = orc.step(); eng.step(1)
        print(t, "digest", eng.digest(t) == d, d)
        rec, lost = eng.drain_events()
        k, tk, r, x = _lib.split_events(rec)
        ok, orr, ox = orc.events()
        g = collections.Counter(r.tolist()); w = collections.Counter(orr.tolist())
        bad = sorted(set(g) ^ set(w) | {q for q in g if g[q] != w.get(q)})
        print(t, len(rec), len(ok), "rows differing", bad[:40])
        for q in bad[:3]:
            print("  row", q, "got", sorted(zip(k[r==q].tolist(), x[r==q].tolist())), "want", sorted(zip(ok[orr==q].tolist(), ox[orr==q].tolist())), "start", orc.start_tick(q))
