"""Drain-all partial view (gsp_pview_params.inbox = 0) on the GPU against oracle/pview_oracle.c.

The reference drains every queued message (checkMessages, MP1Node.cpp:200-212); with inbox = 0
so does the partial view: rows sent at most 7 messages run in the tick kernels, rows sent more
run in gossip_protocol_amd/csrc/pview_drain.hip -- the LDS classes (the row's update tuples
sorted and folded in one LDS buffer) or the hub kernel (the same in HBM buffers) -- which merge
them all in ascending sender order.  Every tick's digest (no overflow), the message lists and the views must
equal the oracle's, which folds every message of every row the same way.  The cases make most
rows long (fan-out 8 and 16 against small views), make hubs past 1,000 senders (a join burst
of 2,000 nodes knowing only the introducer), force every row class in turn (GSP_TEST_PV_DRAIN_WIDE
moves the rows of the smaller LDS classes up, GSP_TEST_PV_DRAIN_LDS sends every long row to the
hub kernel, whose hubs also take their messages in several chunks, the list carried between
them), and run the protocol extensions (TFAIL, SWIM, the JOINREP's introducer list) drained.
"""
import numpy as np
import pytest

from gossip_protocol_amd.pview import PviewEngine, unpack_view
from tests.oracle_binding import PviewOracle, make_policy as oracle_policy
from gossip_protocol_amd._lib import make_policy

pytestmark = pytest.mark.gpu


def _cmp_rows(eng, orc, rows, t):
    for r in rows:
        ids_o, hb_o, ts_o = orc.row(r)
        buf, ln = eng.row(r)
        ids, hb, ts5 = unpack_view(buf, ln)
        assert ln == len(ids_o), "tick %d len row %d: %d vs %d" % (t, r, ln, len(ids_o))
        assert np.array_equal(ids, ids_o), "tick %d ids row %d" % (t, r)
        assert np.array_equal(hb, hb_o), "tick %d hb row %d" % (t, r)
        assert np.array_equal(ts5, ts_o & 31), "tick %d ts row %d" % (t, r)
        assert np.all(buf[ln:] == np.uint64(0xFFFFFFFFFFFFFFFF))
        if orc.fail_tick(r) >= t:
            assert eng.own_hb(r) == orc.own_hb(r), "own hb row %d" % r


def _run(n, ticks, kw, policy=None, events=False, rows_run=False, group=1, every=1, check=None):
    from gossip_protocol_amd import _lib
    orc = PviewOracle(n, policy=oracle_policy(**policy) if policy else None, **kw)
    ekw = dict(kw)
    if policy:
        ekw["policy"] = make_policy(**policy)
    longest = 0
    rng = np.random.default_rng(kw.get("seed", 1))
    with PviewEngine(n, max_ticks=ticks, events=events, group=group, **ekw) as eng:
        if events:
            eng.drain_events()
        for t in range(1, ticks + 1):
            src, dst = orc.messages()                    # sent at t - 1, merged at t
            if len(dst):
                longest = max(longest, int(np.bincount(dst, minlength=n).max()))
            want = orc.step()
            eng.step(1)
            got = eng.digest(t)
            assert got == want, "tick %d\n got %s\nwant %s" % (t, got, want)
            assert got["overflow"] == 0
            if rows_run:
                assert eng.rows_run(t) == n, "tick %d: %d rows run" % (t, eng.rows_run(t))
            if events:
                rec, lost = eng.drain_events()
                assert lost == 0
                k, tk, r, x = _lib.split_events(rec)
                ok, orr, ox = orc.events()
                assert sorted(zip(k.tolist(), r.tolist(), x.tolist())) == \
                    sorted(zip(ok.tolist(), orr.tolist(), ox.tolist())), "events tick %d" % t
            if t % every == 0 or t == ticks:
                m = eng.messages()
                src, dst = orc.messages()
                assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                    sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
                rows = sorted(set(rng.integers(0, n, 60).tolist()) | set(check or ()))
                _cmp_rows(eng, orc, rows, t)
    return longest


CASES = [
    # n, view, fanout, drop, fail_mode, fail_tick, ppm, seed, ticks
    (3000, 32, 8, 0, 1, 5, 20000, 3, 24),        # most rows sent > 7 messages
    (2000, 64, 3, 10, 2, 8, 50000, 7, 30),       # config-5 rules: a few long rows
    (4096, 16, 16, 10, 1, 6, 10000, 5, 16),      # full fan-out to a 16-entry view: k ~ 14
    (3000, 256, 8, 10, 2, 5, 50000, 11, 10),     # config 5's view: 256 slots, more than 192 lanes
]


# the drain kernels' row classes (pv_drain_class): "c0" as sized (class 0: <= 3,072 tuples,
# 192 lanes), "c1" .. "c3" (GSP_TEST_PV_DRAIN_WIDE=1..3: the rows of the smaller classes run in
# class w -- 256, 512 or 1024 lanes), "hub" (GSP_TEST_PV_DRAIN_LDS=300: every long row in the
# hub kernel)
CLASSES = ["c0", "c1", "c2", "c3", "hub"]


def _set_class(monkeypatch, cls):
    if cls in ("c1", "c2", "c3"):
        monkeypatch.setenv("GSP_TEST_PV_DRAIN_WIDE", cls[1:])
    elif cls == "hub":
        monkeypatch.setenv("GSP_TEST_PV_DRAIN_LDS", "300")


@pytest.mark.parametrize("cls", CLASSES[:4])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "n%d_v%d_f%d" % c[:3])
def test_drain_all_matches_oracle(case, cls, monkeypatch):
    _set_class(monkeypatch, cls)
    n, V, f, drop, mode, ftick, ppm, seed, ticks = case
    kw = dict(view=V, fanout=f, inbox=0, drop_pct=drop, fail_mode=mode, fail_tick=ftick,
              fail_ppm=ppm, seed=seed)
    longest = _run(n, ticks, kw, every=4)
    assert longest > 7


@pytest.mark.parametrize("cls", CLASSES)
@pytest.mark.parametrize("evict_order", [0, 1])
def test_drain_all_events_and_rows_run(monkeypatch, evict_order, cls):
    """Every join / remove / evict record of the long rows, every row run exactly once (the
    split kernels skip the long rows; the drain kernels run them), in every row class."""
    _set_class(monkeypatch, cls)
    monkeypatch.setenv("GSP_TEST_PV_COUNT_ROWS", "1")
    kw = dict(view=32, fanout=8, inbox=0, drop_pct=10, fail_mode=1, fail_tick=6, fail_ppm=30000,
              seed=17, tremove=10, evict_order=evict_order)
    _run(2500, 20, kw, events=True, rows_run=True, every=5)


RANDOM, BLOCK, SINGLE, HALF = 1, 2, 3, 4
EXT_CASES = [
    # (n, view, fanout, drop, policy, shards, tfail, swim, ticks): the protocol extensions
    # drained (MP1Node.h:22's TFAIL, SWIM probing, the JOINREP's introducer list)
    (2000, 32, 8, 10, None, 1, 5, 0, 22),
    (2000, 32, 8, 10, None, 1, 0, 2, 22),
    (2000, 48, 6, 20, dict(drop_window=(3, 20), step_rate=0.02, intro_list=4,
                           fail_events=[(10, SINGLE, 0), (14, BLOCK, 50000)]), 1, 5, 2, 24),
    (3000, 32, 8, 10, dict(step_rate=0.006, intro_list=16, fail_events=[(9, HALF, 0)]), 1, 0, 0, 20),
    (2000, 48, 6, 20, dict(drop_window=(3, 20), step_rate=0.02, intro_list=4), 3, 5, 2, 20),
]


@pytest.mark.parametrize("cls", ["c0", "c3", "hub"])
@pytest.mark.parametrize("case", EXT_CASES, ids=lambda c: "n%d_v%d_f%d_%s_g%d_tf%d_sw%d" % (
    c[0], c[1], c[2], "pol" if c[4] else "plain", c[5], c[6], c[7]))
def test_drain_all_protocol_extensions(case, cls, monkeypatch):
    """TFAIL (a payload holds what the sender gossiped at t - 1), SWIM (the probe of t - 1
    answered or not before TREMOVE) and the JOINREP's bounded introducer list, every message
    merged: GPU = oracle in the LDS classes and the hub kernel, with events."""
    _set_class(monkeypatch, cls)
    monkeypatch.setenv("GSP_TEST_PV_COUNT_ROWS", "1")
    n, V, f, drop, pol, shards, tfail, swim, ticks = case
    kw = dict(view=V, fanout=f, inbox=0, drop_pct=drop, fail_mode=RANDOM, fail_tick=6,
              fail_ppm=30000, seed=41, tfail=tfail, swim=swim)
    longest = _run(n, ticks, kw, policy=pol, events=True, rows_run=pol is None, group=shards,
                   every=4)
    assert longest > 7


@pytest.mark.parametrize("form", ["0:1", "1:1", "0:0"])
def test_drain_all_kernel_forms(monkeypatch, form):
    """The one-kernel form (GSP_TEST_PV_SPLIT=0) with and without row order (GSP_TEST_PV_SORT): a long
    row reaches pview_tick_kernel there and must be left to the drain kernel."""
    split, sort = form.split(":")
    monkeypatch.setenv("GSP_TEST_PV_SPLIT", split)
    monkeypatch.setenv("GSP_TEST_PV_SORT", sort)
    monkeypatch.setenv("GSP_TEST_PV_COUNT_ROWS", "1")
    kw = dict(view=32, fanout=8, inbox=0, drop_pct=0, fail_mode=2, fail_tick=5, fail_ppm=50000, seed=29)
    _run(2000, 14, kw, rows_run=True, every=7)


def test_drain_all_hbm_paths(monkeypatch):
    """GSP_TEST_PV_DRAIN_LDS=300: every long row (more than 300 ids) is sorted and folded in
    the hub kernel's HBM buffers instead of LDS."""
    _set_class(monkeypatch, "hub")
    kw = dict(view=32, fanout=8, inbox=0, drop_pct=10, fail_mode=1, fail_tick=5, fail_ppm=20000, seed=31)
    _run(3000, 16, kw, every=4)


def test_drain_all_join_burst_past_1000_senders(monkeypatch):
    """2,000 nodes start in one tick knowing only the introducer (no introducer list) and all
    gossip to it: node 0 is sent more than 1,000 messages a tick and merges every one of them
    (the inbox-7 engine drops all but 7).  Its tuples pass the HBM buffers (8,192 tuples at
    n = 5,000), so it merges them in chunks of messages with its list carried between chunks;
    with a low LDS bound its segment sort takes the HBM path too."""
    kw = dict(view=64, fanout=3, inbox=0, drop_pct=10, fail_mode=1, fail_tick=6, fail_ppm=20000,
              seed=43)
    pol = dict(step_rate=0.0005, intro_list=0)
    longest = _run(5000, 8, kw, policy=pol, every=2, check=range(0, 40))
    assert longest > 1000, "node 0 must be sent more than 1,000 messages (got %d)" % longest
    monkeypatch.setenv("GSP_TEST_PV_DRAIN_LDS", "1024")
    assert _run(5000, 6, kw, policy=pol, every=3, check=range(0, 10)) > 1000


def test_drain_all_hub_merges_blocks_in_hbm():
    """n = 20,000: the HBM buffers hold 32,768 tuples, so node 0's chunks of a join burst pass
    the 16,384-tuple LDS blocks -- each chunk's runs are sorted block by block in LDS and the
    blocks merged in HBM, and the fold runs over several 8 K-tuple register blocks."""
    kw = dict(view=64, fanout=3, inbox=0, drop_pct=10, fail_mode=1, fail_tick=6, fail_ppm=20000,
              seed=47)
    pol = dict(step_rate=0.0005, intro_list=0)
    longest = _run(20000, 6, kw, policy=pol, every=2, check=range(0, 12))
    assert longest > 600, "node 0 must be sent more than 600 messages (got %d)" % longest


def test_drain_all_row_shards():
    """Row shards (in-process group of 3): the long rows' senders come from other shards' rows
    (received views, csr_slot < 0)."""
    kw = dict(view=32, fanout=8, inbox=0, drop_pct=10, fail_mode=2, fail_tick=6, fail_ppm=50000, seed=37)
    _run(2400, 14, kw, group=3, every=7)


def test_drain_all_rejects_n_past_the_hub_buffers():
    from gossip_protocol_amd._lib import GspError
    with pytest.raises(GspError, match="drain all"):
        PviewEngine((1 << 21) - 700, view=32, inbox=0, max_ticks=2)


# ---- BASELINE config 5 at its real size, drained ------------------------
PV_FULL = dict(view=256, fanout=3, inbox=0, drop_pct=10, fail_mode=2, fail_tick=10,
               fail_ppm=50000, seed=0x5EED)


def _full_dead(n, seed=0x5EED, ftick=10, ppm=50000):
    """the crashed block of config 5, from the oracle's Philox (oracle/pview_oracle.c)"""
    from tests.oracle_binding import load_oracle
    start = load_oracle().gsp_oracle_draw(0x4641494C, seed, ftick, 0xFFFFFFFF, 0, 0) % n
    m = n * ppm // 1000000
    dead = np.zeros(n, bool)
    dead[(start + np.arange(m)) % n] = True
    return dead, m


def _view_abs(eng, x, t):
    """(ids, hb, absolute ts) of x's view at tick t: every entry of a view at t has t - ts <
    TREMOVE <= 31, so ts mod 32 names it; checks the view's form on the way"""
    buf, ln = eng.row(x)
    ids, hb, ts5 = unpack_view(buf, ln)
    assert ln <= 256 and np.all(np.diff(ids) > 0) and x not in ids, "row %d" % x
    assert np.all(buf[ln:] == np.uint64(0xFFFFFFFFFFFFFFFF))
    return ids, hb, t - ((t - ts5) & 31)


def _recompute_rows(eng, cfg, msgs, t, targets):
    """Rows `targets` of tick t recomputed on the host from the views of t - 1 and the message
    list sent at t - 1 (oracle/pview_oracle.c gsp_pview_oracle_row_step with inbox 0: every
    message merged in ascending sender order, MP1Node.cpp:200-256, then TREMOVE :339-348 and
    the bounded view's eviction), against the device's rows after tick t."""
    from tests.oracle_binding import pview_row_step
    senders = {}
    hit = np.zeros(msgs.shape[0], bool)
    for r in targets:
        np.equal(msgs, r).any(axis=1, out=hit)
        senders[r] = np.nonzero(hit)[0].tolist()
    prev = {x: _view_abs(eng, x, t - 1) for x in set(targets) | {s for v in senders.values() for s in v}}
    eng.step(1)
    for r in targets:
        (ids, hb, ts), _ = pview_row_step(cfg, t, r, prev[r], senders[r], [prev[s] for s in senders[r]])
        gi, gh, gt = _view_abs(eng, r, t)
        k = len(senders[r])
        assert np.array_equal(gi, ids), "tick %d: ids of row %d (%d senders)" % (t, r, k)
        assert np.array_equal(gh, hb), "tick %d: hb of row %d (%d senders)" % (t, r, k)
        assert np.array_equal(gt, ts), "tick %d: ts of row %d (%d senders)" % (t, r, k)
    return {r: len(senders[r]) for r in targets}


def test_drain_all_full_size_rows_recomputed():
    """Config 5 drained at its real size on one GPU (1,048,576 nodes, V = 256, fanout 3, 10 %
    drop, 5 % contiguous crash at t = 10), ticks 1-14: every tick's node-rounds, delivered =
    every message sent to an alive receiver (nothing overflows), sampled views well formed, and
    from tick 6 on, rows recomputed on the host (_recompute_rows) -- every tick the receiver
    with the most senders (a class-3 row by tick 14) and receivers sent 0, 3 (the split
    kernels), 8-10, 11-14, 15-30 and 31-62 messages (LDS classes 0-3) when there are any."""
    from tests.oracle_binding import PviewCfg
    n, ticks = 1 << 20, 14
    cfg = PviewCfg(n, 256, 3, 0, 10, 20, 1, 2, 10, 50000, 0x5EED)
    dead, m = _full_dead(n)
    rng = np.random.default_rng(11)
    bands = [(0, 0), (3, 3), (8, 10), (11, 14), (15, 30), (31, 62)]
    seen = set()
    with PviewEngine(n, max_ticks=ticks, **PV_FULL) as eng:
        eng.step(5)
        for t in range(6, ticks + 1):
            msgs = eng.messages()                        # sent at t - 1, merged at t
            live = msgs[msgs >= 0]
            cnt = np.bincount(live, minlength=n)
            alive = ~dead if t > 10 else np.ones(n, bool)
            rows = np.nonzero(alive)[0]
            targets = [int(rows[np.argmax(cnt[rows])])]
            for lo, hi in bands:
                cand = rows[(cnt[rows] >= lo) & (cnt[rows] <= hi)]
                if len(cand):
                    targets.append(int(cand[rng.integers(len(cand))]))
            ks = _recompute_rows(eng, cfg, msgs, t, targets)
            seen |= set(ks.values())
            d = eng.digest(t)
            assert d["node_rounds"] == (n if t <= 10 else n - m), t
            assert d["overflow"] == 0 and d["delivered"] == int(cnt[alive].sum()), t
            for x in rng.integers(0, n, 32).tolist():
                _view_abs(eng, x, t)
    # by tick 14 the largest receivers are class-3 rows (31-62 senders); hubs past the LDS
    # classes come later (test_drain_all_full_size_hub_past_1000_senders)
    assert max(seen) > 30, "no class-3 row was recomputed (largest %d senders)" % max(seen)


def test_drain_all_eight_row_shards_full_size():
    """Config 5 drained at full size as 8 row shards in one process (the multi-GPU layout's
    exchange with device copies in place of RCCL): every tick's digest, the message lists and
    sampled views equal the one-shard engine's over 12 ticks."""
    n, ticks, G = 1 << 20, 12, 8
    rng = np.random.default_rng(9)
    sample = sorted(set(rng.integers(0, n, 300).tolist()) | {0, 1, n - 1, n // G, n // G - 1})
    with PviewEngine(n, max_ticks=ticks, **PV_FULL) as one:
        want, msgs = [], []
        for t in range(1, ticks + 1):
            one.step(1)
            want.append(one.digest(t))
            msgs.append(one.messages())
        rows = {r: one.row(r) for r in sample}
    with PviewEngine(n, max_ticks=ticks, group=G, **PV_FULL) as eng:
        for t in range(1, ticks + 1):
            eng.step(1)
            assert eng.digest(t) == want[t - 1], "tick %d" % t
            assert np.array_equal(eng.messages(), msgs[t - 1]), "messages of tick %d" % t
        for r in sample:
            buf, ln = eng.row(r)
            assert ln == rows[r][1] and np.array_equal(buf, rows[r][0]), "row %d" % r


def test_drain_all_full_size_hub_past_1000_senders():
    """Config 5 drained long enough that a receiver is sent more than 1,000 messages in one tick
    (the bounded view's rich-get-richer hubs): that hub's row is recomputed on the
    host -- the hub kernel's chunked HBM path at its real size."""
    from tests.oracle_binding import PviewCfg
    n, ticks = 1 << 20, 90
    cfg = PviewCfg(n, 256, 3, 0, 10, 20, 1, 2, 10, 50000, 0x5EED)
    dead, _ = _full_dead(n)
    with PviewEngine(n, max_ticks=ticks, **PV_FULL) as eng:
        eng.step(40)
        for t in range(41, ticks + 1):
            msgs = eng.messages()
            cnt = np.bincount(msgs[msgs >= 0], minlength=n)
            cnt[dead] = 0
            hub = int(np.argmax(cnt))
            if cnt[hub] > 1000:
                ks = _recompute_rows(eng, cfg, msgs, t, [hub])
                assert ks[hub] > 1000
                return
            eng.step(1)
    pytest.fail("no receiver was sent more than 1,000 messages by tick %d" % ticks)
