"""The device event stream against the CPU restatements.

With events on, the tick kernels append one 64-bit record per join / remove (/ evict, partial
view) -- the reference's logNodeAdd / logNodeRemove calls (MP1Node.cpp:276, 297, 343) -- to a
ring drained by gsp_scale_drain_events / gsp_pview_drain_events.  Every tick's drained list
must equal, as a multiset of (kind, r, x) with the record's tick = t, the event list the
oracle builds for that tick (oracle/scale_oracle.c, oracle/pview_oracle.c), in every layout,
with the driver policies, TFAIL and SWIM on.  The lines gsp_events_write_log makes of the
stream are checked against the reference's own dbg.log in tests/test_events_cpu.py.
"""
import numpy as np
import pytest

from gossip_protocol_amd import _lib
from gossip_protocol_amd.pview import PviewEngine
from gossip_protocol_amd.scale import ScaleEngine, make_policy
from tests.oracle_binding import PviewOracle, ScaleOracle
from tests.oracle_binding import make_policy as oracle_policy

pytestmark = pytest.mark.gpu
RANDOM, BLOCK, SINGLE = 1, 2, 3
POL = dict(drop_window=(3, 20), step_rate=0.02, intro_list=4,
           fail_events=[(10, SINGLE, 0), (14, BLOCK, 50000)])


def _multiset(kind, r, x):
    return sorted(zip(np.asarray(kind).tolist(), np.asarray(r).tolist(), np.asarray(x).tolist()))


def _check_tick(eng, orc, t, kinds=(1, 2, 3)):
    rec, lost = eng.drain_events()
    assert lost == 0
    k, tk, r, x = _lib.split_events(rec)
    assert np.all(tk == t), "tick field"
    ok, orr, ox = orc.events()
    keep = np.isin(ok, kinds)
    want = _multiset(ok[keep], orr[keep], ox[keep])
    got = _multiset(k, r, x)
    assert got == want, "tick %d: %d events vs %d; first diff %s" % (
        t, len(got), len(want), next(((a, b) for a, b in zip(got, want) if a != b), None))
    return len(want)


FULL = [
    # (n, fanout, drop, shards, layout, tfail, swim, policy)
    (700, 3, 20, 1, "columns", 0, 0, False),
    (700, 3, 20, 1, "columns", 0, 0, True),
    (900, 4, 10, 3, "columns", 5, 0, True),
    (900, 3, 30, 2, "rows", 0, 2, True),
    (600, 3, 10, 3, "rows", 5, 2, False),
]


@pytest.mark.parametrize("case", FULL, ids=lambda c: "n%d_%s%d_tf%d_sw%d_pol%d" % (
    c[0], c[4], c[3], c[5], c[6], c[7]))
def test_full_view_event_stream_matches_oracle(case):
    n, f, drop, shards, layout, tfail, swim, pol = case
    ticks = 32
    kw = dict(fanout=f, drop_pct=drop, fail_mode=RANDOM, fail_tick=6, fail_ppm=30000, seed=17,
              tfail=tfail, swim=swim, tremove=12)
    orc = ScaleOracle(n, policy=oracle_policy(**POL) if pol else None, **kw)
    total = 0
    with ScaleEngine(n, max_ticks=ticks, group=shards, layout=layout, events=True,
                     policy=make_policy(**POL) if pol else None, **kw) as eng:
        eng.drain_events()                              # anything recorded at create
        for t in range(1, ticks + 1):
            orc.step()
            eng.step(1)
            total += _check_tick(eng, orc, t)
    assert total > n                                    # joins and removes both happen


PV = [
    # (n, view, fanout, inbox, drop, shards, tfail, swim, policy)
    (1500, 48, 3, 5, 20, 1, 0, 0, False),
    (1500, 48, 3, 5, 20, 1, 0, 0, True),
    (2000, 32, 4, 4, 10, 3, 5, 2, True),
    (1200, 64, 3, 7, 30, 2, 0, 2, False),
]


@pytest.mark.parametrize("case", PV, ids=lambda c: "n%d_v%d_g%d_tf%d_sw%d_pol%d" % (
    c[0], c[1], c[5], c[6], c[7], c[8]))
def test_partial_view_event_stream_matches_oracle(case):
    n, V, f, K, drop, shards, tfail, swim, pol = case
    ticks = 30
    kw = dict(view=V, fanout=f, inbox=K, drop_pct=drop, fail_mode=RANDOM, fail_tick=6,
              fail_ppm=30000, seed=23, tfail=tfail, swim=swim, tremove=12)
    orc = PviewOracle(n, policy=oracle_policy(**POL) if pol else None, **kw)
    kinds = set()
    with PviewEngine(n, max_ticks=ticks, group=shards, events=True,
                     policy=make_policy(**POL) if pol else None, **kw) as eng:
        eng.drain_events()
        for t in range(1, ticks + 1):
            orc.step()
            eng.step(1)
            _check_tick(eng, orc, t)
            kinds |= set(orc.events()[0].tolist())
    assert kinds == {1, 2, 3}                           # joins, removes and evictions


@pytest.mark.parametrize("kinds", [_lib.EVENTS_REMOVE, _lib.EVENTS_JOIN,
                                   _lib.EVENTS_REMOVE | _lib.EVENTS_EVICT])
def test_event_kind_mask(kinds):
    """params.events as a kind mask: only the selected kinds are recorded, all of them."""
    sel = tuple(k for k in (1, 2, 3) if kinds >> k & 1)
    n, ticks = 1200, 24
    kw = dict(fanout=3, drop_pct=10, fail_mode=RANDOM, fail_tick=6, fail_ppm=30000, seed=29,
              tremove=10)
    orc = ScaleOracle(n, **kw)
    with ScaleEngine(n, max_ticks=ticks, events=kinds, **kw) as eng:
        for t in range(1, ticks + 1):
            orc.step()
            eng.step(1)
            _check_tick(eng, orc, t, sel)
    pkw = dict(view=48, fanout=3, inbox=5, drop_pct=10, fail_mode=RANDOM, fail_tick=6,
               fail_ppm=30000, seed=29, tremove=10)
    orc = PviewOracle(n, **pkw)
    with PviewEngine(n, max_ticks=ticks, events=kinds, **pkw) as eng:
        for t in range(1, ticks + 1):
            orc.step()
            eng.step(1)
            _check_tick(eng, orc, t, sel)


def test_event_ring_overflow_counts_lost():
    """A ring too small for the run: its 256 stripes (row % 256) keep event_cap / 256 records
    each (rounded up), and every record beyond is counted as lost -- held + lost = all."""
    n, ticks = 400, 8                                   # ~40 crashes at t = 2, tremove 3
    with ScaleEngine(n, max_ticks=ticks, fanout=3, seed=5, fail_mode=RANDOM, fail_tick=2,
                     fail_ppm=100000, tremove=3, events=True, event_cap=100) as eng:
        eng.drain_events()
        eng.step(ticks)
        total = sum(eng.digest(t)["joins"] + eng.digest(t)["removes"] for t in range(1, ticks + 1))
        rec, lost = eng.drain_events()
        assert 0 < len(rec) <= 256 and lost > 0 and len(rec) + lost == total
        rec, lost = eng.drain_events()                  # the drain emptied the ring
        assert len(rec) == 0 and lost == 0


def test_events_off_refuses_drain():
    with ScaleEngine(64, max_ticks=2, fanout=3, seed=5) as eng:
        with pytest.raises(Exception, match="records no events"):
            eng.drain_events()


def test_drain_with_small_buffer_counts_the_rest_as_lost():
    """gsp_scale_drain_events with cap below the records held: *n = the records copied (cap),
    the rest count as lost, and the ring is emptied (gossip.h)."""
    import ctypes
    n, ticks = 400, 8
    with ScaleEngine(n, max_ticks=ticks, fanout=3, seed=5, fail_mode=RANDOM, fail_tick=2,
                     fail_ppm=100000, tremove=3, events=True) as eng:
        eng.drain_events()
        eng.step(ticks)
        fn = _lib.lib().gsp_scale_drain_events
        held, lost = ctypes.c_int64(), ctypes.c_int64()
        assert fn(eng._h, None, 0, ctypes.byref(held), ctypes.byref(lost)) == 0
        assert held.value > 10 and lost.value == 0
        cap = held.value // 3
        buf = np.zeros(held.value, np.uint64)
        got, lost = ctypes.c_int64(), ctypes.c_int64()
        assert fn(eng._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cap,
                  ctypes.byref(got), ctypes.byref(lost)) == 0
        assert got.value == cap and lost.value == held.value - cap
        assert np.all(buf[cap:] == 0) and np.all(buf[:cap] != 0)
        rec, lost2 = eng.drain_events()
        assert len(rec) == 0 and lost2 == 0
