"""Driver policies of the scale protocols on the CPU restatements (oracle/schedule.c,
scale_oracle.c, pview_oracle.c): the reference's hard-coded driver (Application.cpp:143 join
schedule, :177/:198 drop window, :180-196 crash injection) as data, plus the bounded
introducer list (MP1Node.cpp:221-230 sends the whole list; its receiver ignores it).

These are build-defined protocol extensions: the tests pin their semantics by invariants
(parity of the GPU against these restatements: tests/test_policy_gpu.py).
"""
import numpy as np

from tests.oracle_binding import PviewOracle, ScaleOracle, make_policy

SINGLE, HALF, RANDOM, BLOCK = 3, 4, 1, 2


def test_zero_policy_is_the_single_event_protocol():
    kw = dict(fanout=3, drop_pct=10, fail_mode=RANDOM, fail_tick=6, fail_ppm=40000, seed=5)
    a, b = ScaleOracle(120, **kw), ScaleOracle(120, policy=make_policy(), **kw)
    assert [a.step() for _ in range(20)] == [b.step() for _ in range(20)]


def test_drop_window():
    o = ScaleOracle(200, fanout=3, drop_pct=30, seed=3, policy=make_policy(drop_window=(4, 9)))
    for t in range(1, 14):
        d = o.step()
        assert (d["dropped"] > 0) == (4 <= t < 9), t


def test_failure_events_compose():
    n = 300
    pol = make_policy(fail_events=[(8, SINGLE, 0), (12, HALF, 0), (15, BLOCK, 100000)])
    o = ScaleOracle(n, fanout=3, fail_mode=RANDOM, fail_tick=5, fail_ppm=20000, seed=9, policy=pol)
    f = np.array([o.fail_tick(r) for r in range(n)])
    at = {t: np.nonzero(f == t)[0] for t in (5, 8, 12, 15)}
    assert 0 < len(at[5]) < 20 and len(at[8]) <= 1
    half = np.nonzero(f <= 12)[0]
    first = (f == 12).nonzero()[0]
    assert len(first) > 0 and len(half) >= n // 2 - len(at[5]) - len(at[8])
    # the HALF event is n/2 contiguous nodes (Application.cpp:189-195)
    crashed_by_12 = f <= 12
    runs = np.diff(np.concatenate([[0], crashed_by_12.astype(int), [0]]))
    assert (np.nonzero(runs == -1)[0] - np.nonzero(runs == 1)[0]).max() >= n // 2
    assert (f <= 15).sum() >= (f <= 12).sum()          # the BLOCK event may overlap the HALF
    d = [o.step() for _ in range(16)]
    alive = [int(((f >= t)).sum()) for t in range(1, 17)]
    assert [x["node_rounds"] for x in d] == alive


def _joins(Oracle, **kw):
    n, rate, B = 240, 0.05, 4
    o = Oracle(n, fanout=3, seed=13, policy=make_policy(step_rate=rate, intro_list=B), **kw)
    start = np.array([o.start_tick(r) for r in range(n)])
    assert (start == (rate * np.arange(n)).astype(int)).all()
    for t in range(1, 25):
        jr = set(o.joinreps().tolist())                 # sent at t - 1, merged at t
        assert jr == set(np.nonzero(start == t)[0].tolist())
        d = o.step()
        assert d["node_rounds"] == int((start <= t).sum())
        for j in jr:
            row = o.row(j)
            ids = np.nonzero(row[0])[0] if Oracle is ScaleOracle else row[0]
            assert 0 in ids and 1 <= len(ids) <= B + 1  # the introducer + the bounded list
    # by now the early joiners are known to others
    j = int(np.nonzero(start == 2)[0][0])
    known = sum(1 for r in range(n) if r != j and (
        o.row(r)[0][j] if Oracle is ScaleOracle else j in o.row(r)[0]))
    assert known > 0
    return o


def test_join_schedule_and_bounded_introducer_list_full_view():
    _joins(ScaleOracle)


def test_join_schedule_and_bounded_introducer_list_partial_view():
    _joins(PviewOracle, view=32, inbox=4)


def test_pview_tfail_and_swim_change_the_run():
    kw = dict(view=32, fanout=3, inbox=5, drop_pct=10, fail_mode=RANDOM, fail_tick=4,
              fail_ppm=50000, seed=17)
    base = PviewOracle(400, **kw)
    db = [base.step() for _ in range(30)]
    for extra in (dict(tfail=5), dict(swim=2), dict(tfail=5, swim=2)):
        o = PviewOracle(400, **kw, **extra)
        d = [o.step() for _ in range(30)]
        assert d != db, extra
        if "swim" in extra:
            # unanswered probes of crashed members remove them before TREMOVE (20 ticks after
            # the crash at t = 4) could
            first = next(t for t, x in enumerate(d, 1) if x["removes"] > 0)
            assert first < 4 + 20


def test_events_match_digest_counts():
    o = PviewOracle(300, view=24, fanout=3, inbox=4, drop_pct=5, fail_mode=BLOCK, fail_tick=3,
                    fail_ppm=100000, seed=2)
    s = ScaleOracle(200, fanout=3, fail_mode=RANDOM, fail_tick=3, fail_ppm=50000, seed=2)
    for _ in range(28):
        d = o.step()
        k, r, x = o.events()
        assert (int((k == 1).sum()), int((k == 2).sum()), int((k == 3).sum())) == (
            d["joins"], d["removes"], d["evicts"])
        e = s.step()
        k, r, x = s.events()
        assert (int((k == 1).sum()), int((k == 2).sum())) == (e["joins"], e["removes"])
