"""Driver policies at scale on the GPU against the CPU restatements.

The join schedule with JOINREPs carrying a bounded introducer list, the drop window and
multi-event crash schedules (gsp_policy, include/gossip/gossip.h) -- the reference's
Application.cpp:143, 177-200 and MP1Node.cpp:221-230 as data -- in every layout of both scale
engines, and TFAIL / SWIM in the partial view: every tick's digest, the message lists and
the membership state must equal oracle/scale_oracle.c / oracle/pview_oracle.c.
"""
import numpy as np
import pytest

from gossip_protocol_amd.pview import PviewEngine, unpack_view
from gossip_protocol_amd.scale import ScaleEngine, make_policy, unpack
from tests.oracle_binding import PviewOracle, ScaleOracle
from tests.oracle_binding import make_policy as oracle_policy

pytestmark = pytest.mark.gpu
RANDOM, BLOCK, SINGLE, HALF = 1, 2, 3, 4

POLICIES = {
    # name: dict(drop_window, step_rate, intro_list, fail_events) -- both bindings build it
    "joins_b4_window_events": dict(drop_window=(3, 20), step_rate=0.02, intro_list=4,
                                   fail_events=[(10, SINGLE, 0), (14, BLOCK, 50000)]),
    "joins_b16_half": dict(step_rate=0.006, intro_list=16, fail_events=[(9, HALF, 0)]),
    "joins_b0": dict(step_rate=0.03, intro_list=0, drop_window=(0, 8)),
}


def _pol(name, oracle=False):
    return (oracle_policy if oracle else make_policy)(**POLICIES[name])


FULL_CASES = [
    # (n, fanout, drop, policy, shards, layout, tfail, swim, ticks)
    (600, 3, 20, "joins_b4_window_events", 1, "columns", 0, 0, 26),
    (2100, 3, 10, "joins_b16_half", 1, "columns", 0, 0, 22),
    (600, 4, 20, "joins_b4_window_events", 2, "columns", 0, 0, 22),
    (2100, 3, 10, "joins_b16_half", 3, "columns", 5, 0, 20),
    (600, 3, 20, "joins_b4_window_events", 3, "rows", 0, 0, 22),
    (900, 3, 30, "joins_b0", 2, "rows", 0, 2, 22),
    (900, 3, 30, "joins_b0", 1, "columns", 5, 2, 24),
]


@pytest.mark.parametrize("case", FULL_CASES, ids=lambda c: "n%d_%s_%s%d_tf%d_sw%d" % (
    c[0], c[3], c[5], c[4], c[6], c[7]))
def test_full_view_policies_match_oracle(case):
    n, f, drop, pol, shards, layout, tfail, swim, ticks = case
    kw = dict(fanout=f, drop_pct=drop, fail_mode=RANDOM, fail_tick=6, fail_ppm=20000, seed=31,
              tfail=tfail, swim=swim)
    orc = ScaleOracle(n, policy=_pol(pol, True), **kw)
    joined = 0
    with ScaleEngine(n, max_ticks=ticks, group=shards, layout=layout, policy=_pol(pol),
                     **kw) as eng:
        for t in range(1, ticks + 1):
            joined += len(orc.joinreps())
            want = orc.step()
            eng.step(1)
            assert eng.digest(t) == want, "tick %d\n got %s\nwant %s" % (t, eng.digest(t), want)
            if t % 5 == 0 or t == ticks:
                src, dst = orc.messages()
                m = eng.messages()
                assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                    sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
        for r in range(0, n, 7):
            pres_o, hb_o, ts_o = orc.row(r)
            pres_d, hb_d, ts5_d = unpack(eng.row(r))
            assert np.array_equal(pres_d, pres_o.astype(bool)), "presence row %d" % r
            assert np.array_equal(hb_d[pres_d], hb_o[pres_d]), "hb row %d" % r
            assert np.array_equal(ts5_d[pres_d], ts_o[pres_d] & 31), "ts row %d" % r
            if orc.fail_tick(r) >= ticks and orc.start_tick(r) <= ticks:
                assert eng.own_hb(r) == orc.own_hb(r), "own hb row %d" % r
    assert joined > 10                              # the case exercises the join schedule


PV_CASES = [
    # (n, view, fanout, inbox, drop, policy, shards, tfail, swim, ticks)
    (1500, 48, 3, 5, 20, "joins_b4_window_events", 1, 0, 0, 24),
    (3000, 64, 3, 7, 10, "joins_b16_half", 1, 0, 0, 22),
    (1500, 48, 3, 5, 20, "joins_b4_window_events", 3, 0, 0, 20),
    (2000, 32, 4, 4, 10, "joins_b0", 1, 5, 0, 26),
    (2000, 32, 4, 4, 10, "joins_b0", 1, 0, 2, 26),
    (2000, 48, 3, 5, 30, "joins_b4_window_events", 2, 5, 2, 24),
]


@pytest.mark.parametrize("case", PV_CASES, ids=lambda c: "n%d_v%d_%s_g%d_tf%d_sw%d" % (
    c[0], c[1], c[5], c[6], c[7], c[8]))
def test_partial_view_policies_match_oracle(case):
    n, V, f, K, drop, pol, shards, tfail, swim, ticks = case
    kw = dict(view=V, fanout=f, inbox=K, drop_pct=drop, fail_mode=RANDOM, fail_tick=6,
              fail_ppm=30000, seed=41, tfail=tfail, swim=swim)
    orc = PviewOracle(n, policy=_pol(pol, True), **kw)
    with PviewEngine(n, max_ticks=ticks, group=shards, policy=_pol(pol), **kw) as eng:
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            got = eng.digest(t)
            assert got == want, "tick %d\n got %s\nwant %s" % (t, got, want)
            if t % 6 == 0 or t == ticks:
                src, dst = orc.messages()
                m = eng.messages()
                assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                    sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
        for r in range(0, n, 5):
            ids_o, hb_o, ts_o = orc.row(r)
            buf, ln = eng.row(r)
            ids, hb, ts5 = unpack_view(buf, ln)
            assert ln == len(ids_o) and np.array_equal(ids, ids_o), "ids row %d" % r
            assert np.array_equal(hb, hb_o) and np.array_equal(ts5, ts_o & 31), "row %d" % r
            if orc.fail_tick(r) >= ticks and orc.start_tick(r) <= ticks:
                assert eng.own_hb(r) == orc.own_hb(r), "own hb row %d" % r


def test_partial_view_join_burst_past_1024_messages():
    """A join burst: 2,000 nodes start in one tick knowing only the introducer (no introducer
    list, B = 0) and all gossip to it, so node 0 is sent up to ~2,450 messages per tick (oracle,
    ticks 2-8) -- past round 2's 1,024-message segment bound, which
    made the job stop with a capacity error. The receipt kernel keeps the K smallest senders of
    any number (include/gossip/gossip.h: the bound is now the digest's 16-bit overflow field):
    every tick's digest, the message lists and the views equal oracle/pview_oracle.c, which has
    no bound."""
    n, ticks = 5000, 8
    kw = dict(view=64, fanout=3, inbox=7, drop_pct=10, fail_mode=RANDOM, fail_tick=6,
              fail_ppm=20000, seed=43)
    pol = dict(step_rate=0.0005, intro_list=0)
    orc = PviewOracle(n, policy=oracle_policy(**pol), **kw)
    burst = 0
    with PviewEngine(n, max_ticks=ticks, policy=make_policy(**pol), **kw) as eng:
        for t in range(1, ticks + 1):
            src, dst = orc.messages()          # sent at t - 1, received at t
            burst = max(burst, int(np.bincount(dst, minlength=n).max()))
            want = orc.step()
            eng.step(1)
            got = eng.digest(t)
            assert got == want, "tick %d\n got %s\nwant %s" % (t, got, want)
            m = eng.messages()
            src, dst = orc.messages()
            assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
        for r in list(range(0, 40)) + list(range(40, n, 37)):
            ids_o, hb_o, ts_o = orc.row(r)
            buf, ln = eng.row(r)
            ids, hb, ts5 = unpack_view(buf, ln)
            assert ln == len(ids_o) and np.array_equal(ids, ids_o), "ids row %d" % r
            assert np.array_equal(hb, hb_o) and np.array_equal(ts5, ts_o & 31), "row %d" % r
    assert burst > 1024, "the case must send one receiver more than 1,024 messages (got %d)" % burst


@pytest.mark.parametrize("layout,shards,tfail,swim,events", [
    ("columns", 1, 0, 0, False), ("columns", 3, 0, 0, True), ("rows", 2, 0, 0, True),
    ("columns", 1, 5, 2, True)], ids=["fused", "columns3_events", "rows2_events", "tfail_swim_events"])
def test_full_view_join_burst_past_1024_messages(layout, shards, tfail, swim, events):
    """The full view's join burst: 2,000 nodes start in one tick knowing
    only the introducer (B = 0) and all gossip to it, so node 0 is sent ~2,000 messages a tick --
    past the tick kernel's LDS sort of 1,024 senders, which round 3 turned into a capacity
    error.  The reference drains a queue of any length (MP1Node.cpp:200-212); the kernel now
    sorts such a segment in HBM and merges its first k - 1,024 messages in a premerge pass
    (scale_kernels.hip).  Every tick's digest, the message lists, every row of the hub and of
    sampled nodes, and (events on) every tick's join / remove records equal
    oracle/scale_oracle.c, which has no bound -- in the fused, column-group and row layouts,
    with TFAIL and SWIM."""
    from gossip_protocol_amd import _lib
    n, ticks = 5000, 8
    kw = dict(fanout=3, drop_pct=10, fail_mode=RANDOM, fail_tick=6, fail_ppm=20000, seed=43,
              tfail=tfail, swim=swim)
    pol = dict(step_rate=0.0005, intro_list=0)
    orc = ScaleOracle(n, policy=oracle_policy(**pol), **kw)
    burst = 0
    with ScaleEngine(n, max_ticks=ticks, group=shards, layout=layout, policy=make_policy(**pol),
                     events=events, **kw) as eng:
        if events:
            eng.drain_events()
        for t in range(1, ticks + 1):
            src, dst = orc.messages()          # sent at t - 1, received at t
            burst = max(burst, int(np.bincount(dst, minlength=n).max()))
            want = orc.step()
            eng.step(1)
            got = eng.digest(t)
            assert got == want, "tick %d\n got %s\nwant %s" % (t, got, want)
            if events:
                rec, lost = eng.drain_events()
                assert lost == 0
                k, tk, r, x = _lib.split_events(rec)
                ok, orr, ox = orc.events()
                assert sorted(zip(k.tolist(), r.tolist(), x.tolist())) == \
                    sorted(zip(ok.tolist(), orr.tolist(), ox.tolist())), "events tick %d" % t
            m = eng.messages()
            src, dst = orc.messages()
            assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
        for r in list(range(0, 8)) + list(range(8, n, 41)):
            pres_o, hb_o, ts_o = orc.row(r)
            pres_d, hb_d, ts5_d = unpack(eng.row(r))
            assert np.array_equal(pres_d, pres_o.astype(bool)), "presence row %d" % r
            assert np.array_equal(hb_d[pres_d], hb_o[pres_d]), "hb row %d" % r
            assert np.array_equal(ts5_d[pres_d], ts_o[pres_d] & 31), "ts row %d" % r
    assert burst > 1024, "the case must send one receiver more than 1,024 messages (got %d)" % burst


@pytest.mark.parametrize("engine", ["pview_inbox7", "pview_drain", "full_rows"])
def test_row_exchange_posted_sizes_cover_join_bursts(monkeypatch, engine):
    """The sizes a communicator posts to RCCL come from earlier ticks' counts plus margins
    (rowx_host.cpp); the growth the host knows of -- a join burst's new senders, a drop window
    that ends -- is added to them.  GSP_TEST_ROWX_POSTED=1 makes an in-process
    group of 3 post and check exactly those sizes (a count past them stops the job with
    GSP_ERR_CAPACITY), so a burst of thousands of joiners with the drop rate falling from 30 %
    to 0 must run to the end and equal the oracle."""
    monkeypatch.setenv("GSP_TEST_ROWX_POSTED", "1")
    ticks = 12
    if engine == "full_rows":
        n, pol = 2100, dict(step_rate=0.002, intro_list=4, drop_window=(0, 5))
        kw = dict(fanout=3, drop_pct=30, fail_mode=RANDOM, fail_tick=6, fail_ppm=20000, seed=53)
        orc = ScaleOracle(n, policy=oracle_policy(**pol), **kw)
        eng = ScaleEngine(n, max_ticks=ticks, group=3, layout="rows", policy=make_policy(**pol), **kw)
    else:
        n, pol = 6000, dict(step_rate=0.0005, intro_list=0, drop_window=(0, 5))
        kw = dict(view=64, fanout=3, inbox=7 if engine == "pview_inbox7" else 0, drop_pct=30,
                  fail_mode=RANDOM, fail_tick=6, fail_ppm=20000, seed=53)
        orc = PviewOracle(n, policy=oracle_policy(**pol), **kw)
        eng = PviewEngine(n, max_ticks=ticks, group=3, policy=make_policy(**pol), **kw)
    with eng:
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            assert eng.digest(t) == want, "tick %d" % t
        src, dst = orc.messages()
        m = eng.messages()
        assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
            sorted(zip(src.tolist(), dst.tolist()))
