import sys
sys.path.insert(0, '.')
from gossip_protocol_amd.scale import ScaleEngine, make_policy, nccl_unique_id, FAIL_RANDOM
from tests.oracle_binding import ScaleOracle
from tests.oracle_binding import make_policy as oracle_policy
cases = {"joins": dict(step_rate=0.002, intro_list=4), "joins_b0": dict(step_rate=0.002),
         "window": dict(drop_window=(2, 9)), "failev": dict(fail_events=[(8, 3, 0)])}
for name, pol in cases.items():
    for comm in (False, True):
        n, ticks = 8192, 14
        kw = dict(fanout=3, drop_pct=10, fail_mode=FAIL_RANDOM, fail_tick=5, fail_ppm=20000, seed=6)
        orc = ScaleOracle(n, policy=oracle_policy(**pol), **kw)
        ekw = dict(rank=0, world=1, nccl_id=nccl_unique_id()) if comm else dict(group=2)
        try:
            with ScaleEngine(n, max_ticks=ticks, policy=make_policy(**pol), **ekw, **kw) as eng:
                bad = None
                for t in range(1, ticks + 1):
                    want = orc.step(); eng.step(1)
                    d = eng.digest(t)
                    if d != want and bad is None:
                        bad = (t, {k: (d[k], want[k]) for k in d if d[k] != want[k]})
                print(name, "comm" if comm else "group2", "OK" if bad is None else bad, flush=True)
        except Exception as e:
            print(name, "comm" if comm else "group2", "ERR", str(e)[:150], flush=True)
