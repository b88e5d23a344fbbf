import sys, traceback
sys.path.insert(0, '.')
from gossip_protocol_amd.scale import ScaleEngine, make_policy, nccl_unique_id, FAIL_RANDOM
from tests.oracle_binding import ScaleOracle
from tests.oracle_binding import make_policy as oracle_policy
for tiles in (1, 2):
    for pol_on, ev in ((True, False), (False, True), (True, True)):
        n, ticks = 8192, 14
        kw = dict(fanout=3, drop_pct=10, fail_mode=FAIL_RANDOM, fail_tick=5, fail_ppm=20000, seed=6)
        pol = dict(drop_window=(2, 9), step_rate=0.002, intro_list=4, fail_events=[(8, 3, 0)]) if pol_on else None
        orc = ScaleOracle(n, policy=oracle_policy(**pol) if pol else None, **kw)
        try:
            with ScaleEngine(n, max_ticks=ticks, rank=0, world=1, nccl_id=nccl_unique_id(), tiles=tiles,
                             policy=make_policy(**pol) if pol else None, events=ev, **kw) as eng:
                bad = None
                for t in range(1, ticks + 1):
                    want = orc.step(); eng.step(1)
                    if eng.digest(t) != want and bad is None:
                        bad = (t, eng.digest(t), want)
                print(tiles, pol_on, ev, "OK" if bad is None else bad, flush=True)
        except Exception as e:
            print(tiles, pol_on, ev, "ERR", e, flush=True)
