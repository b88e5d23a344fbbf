"""PARTIAL-VIEW engine on the GPU against oracle/pview_oracle.c (BASELINE config 5 rules).

Per tick: every digest field (node-rounds, merges, sends, drops, deliveries, inbox overflow,
joins, removes, evictions, event hash) identical; periodically the message lists and full
views (ids and hb exactly, ts mod 32) identical.  Cases cover eviction pressure (small V),
inbox overflow (small K, large fanout), drops and both failure modes, and views larger
than the population.
"""
import numpy as np
import pytest

from gossip_protocol_amd.pview import PviewEngine, unpack_view
from tests.oracle_binding import PviewOracle

pytestmark = pytest.mark.gpu

CASES = [
    # n, view, fanout, inbox, drop, fail_mode, fail_tick, ppm, seed, ticks
    (300, 256, 3, 7, 0, 0, 10, 0, 1, 30),          # V > n - 1: everyone known
    (2000, 64, 3, 7, 10, 1, 8, 30000, 7, 36),      # eviction every tick
    (5000, 256, 3, 7, 10, 2, 10, 50000, 11, 22),   # config-5 rules, smaller n
    (3000, 32, 8, 2, 0, 1, 5, 20000, 3, 30),       # inbox overflow
    (1500, 100, 5, 4, 30, 2, 6, 100000, 99, 28),   # V not a power of 2
]


def _cmp_rows(eng, orc, rows):
    for r in rows:
        ids_o, hb_o, ts_o = orc.row(r)
        buf, ln = eng.row(r)
        ids, hb, ts5 = unpack_view(buf, ln)
        assert ln == len(ids_o), "len row %d: %d vs %d" % (r, ln, len(ids_o))
        assert np.array_equal(ids, ids_o), "ids row %d" % r
        assert np.array_equal(hb, hb_o), "hb row %d" % r
        assert np.array_equal(ts5, ts_o & 31), "ts row %d" % r
        assert np.all(buf[ln:] == np.uint64(0xFFFFFFFFFFFFFFFF))
        if orc.fail_tick(r) >= eng_tick(eng):
            assert eng.own_hb(r) == orc.own_hb(r)


def eng_tick(eng):
    return eng._tick


@pytest.mark.parametrize("case", CASES, ids=lambda c: "n%d_v%d_f%d_k%d" % c[:4])
def test_pview_matches_oracle(case):
    _run_case(case)


# h0 = 100: an adopted orphan (hb 1, ts t) and its copies sit e = h0 + ts - hb >= 31 deep in
# their age's eviction bins, so the boundary often falls in an age's last bin and takes the
# exact hb-histogram path of the kernel; the long case reaches large e with h0 = 1
@pytest.mark.parametrize("case", [(2000, 64, 3, 7, 10, 1, 8, 30000, 4, 30, 100),
                                  (1000, 48, 4, 7, 5, 0, 10, 0, 6, 70, 1)],
                         ids=["h0_100", "h0_1_70ticks"])
def test_pview_eviction_bins_match_oracle(case):
    _run_case(case[:-1], h0=case[-1])


# the tick kernel's launch forms -- GSP_TEST_PV_SPLIT: 0 one 256-lane kernel for every row, 1 rows
# bucketed by k into four kernels on exact grids (the bucket sizes read back each tick; round 5
# -- they replace round 3's predicted grids and overflow kernel); the second field 0 turns off
# the one-shard receiver CSR scattered from the send kernel's returned slots
# (GSP_TEST_PV_POS_SCATTER=0: the atomic fill-counter scatter instead)
def _set_form(monkeypatch, form):
    split, pos = (form.split(":") + ["1"])[:2]
    monkeypatch.setenv("GSP_TEST_PV_SPLIT", split)
    monkeypatch.setenv("GSP_TEST_PV_POS_SCATTER", pos)


@pytest.mark.parametrize("form", ["0", "1", "1:0", "0:0"])
@pytest.mark.parametrize("case", [CASES[1], CASES[2], CASES[4]], ids=lambda c: "n%d_v%d" % c[:2])
def test_pview_kernel_forms_match_oracle(case, form, monkeypatch):
    _set_form(monkeypatch, form)
    _run_case(case)


# every launch form with the event stream on (a row run twice
# would duplicate its event records, which digests and views cannot see) and a per-tick count
# of the rows the tick kernels ran, which must be every row exactly once
# (GSP_TEST_PV_COUNT_ROWS=1, gsp_pview_rows_run)
@pytest.mark.parametrize("form", ["1", "0"])
@pytest.mark.parametrize("case", [CASES[1], CASES[3]], ids=lambda c: "n%d_v%d" % c[:2])
def test_pview_kernel_forms_events_and_rows_run(case, form, monkeypatch):
    from gossip_protocol_amd import _lib
    _set_form(monkeypatch, form)
    monkeypatch.setenv("GSP_TEST_PV_COUNT_ROWS", "1")
    n, V, f, K, drop, mode, ftick, ppm, seed, ticks = case
    kw = dict(view=V, fanout=f, inbox=K, drop_pct=drop, fail_mode=mode, fail_tick=ftick,
              fail_ppm=ppm, seed=seed, tremove=10)
    orc = PviewOracle(n, **kw)
    kinds = set()
    with PviewEngine(n, max_ticks=ticks, events=True, **kw) as eng:
        eng.drain_events()
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            assert eng.digest(t) == want, "tick %d" % t
            assert eng.rows_run(t) == n, "tick %d: the tick kernels ran %d rows of %d" % (
                t, eng.rows_run(t), n)
            rec, lost = eng.drain_events()
            assert lost == 0
            k, tk, r, x = _lib.split_events(rec)
            assert np.all(tk == t)
            ok, orr, ox = orc.events()
            assert sorted(zip(k.tolist(), r.tolist(), x.tolist())) == \
                sorted(zip(ok.tolist(), orr.tolist(), ox.tolist())), "events tick %d" % t
            kinds |= set(ok.tolist())
    assert kinds == {1, 2, 3}                           # joins, removes and evictions


def test_pview_rows_run_queued_ticks(monkeypatch):
    """gsp_pview_step(k) queues k ticks in one call: still every row exactly once per tick."""
    monkeypatch.setenv("GSP_TEST_PV_COUNT_ROWS", "1")
    n = 20000
    with PviewEngine(n, view=64, fanout=3, inbox=7, drop_pct=10, fail_mode=2, fail_tick=5,
                     fail_ppm=50000, seed=3, max_ticks=16) as eng:
        eng.step(16)
        assert [eng.rows_run(t) for t in range(1, 17)] == [n] * 16


def test_pview_rows_run_needs_the_env():
    from gossip_protocol_amd._lib import GspError
    with PviewEngine(500, view=32, max_ticks=2) as eng:
        eng.step(1)
        with pytest.raises(GspError, match="GSP_TEST_PV_COUNT_ROWS"):
            eng.rows_run(1)


# evict_order 1 (round 4): eviction ties by the rotated id (x - m) mod n, m = Philox(EVICT; t, r)
# mod n -- the plain protocol's kernel with the kExtRot bit, and the superset kernel with events
@pytest.mark.parametrize("case", [CASES[1], CASES[2], CASES[3]], ids=lambda c: "n%d_v%d" % c[:2])
def test_pview_rotated_eviction_matches_oracle(case):
    _run_case(case, evict_order=1)


def test_pview_rotated_eviction_events_match_oracle():
    from gossip_protocol_amd import _lib
    n, ticks = 2000, 30
    kw = dict(view=48, fanout=3, inbox=5, drop_pct=20, fail_mode=1, fail_tick=6, fail_ppm=30000,
              seed=23, tremove=12, evict_order=1)
    orc = PviewOracle(n, **kw)
    with PviewEngine(n, max_ticks=ticks, events=True, **kw) as eng:
        eng.drain_events()
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            assert eng.digest(t) == want, "tick %d" % t
            rec, lost = eng.drain_events()
            k, tk, r, x = _lib.split_events(rec)
            ok, orr, ox = orc.events()
            assert sorted(zip(k.tolist(), r.tolist(), x.tolist())) == \
                sorted(zip(ok.tolist(), orr.tolist(), ox.tolist())), "events tick %d" % t


def _run_case(case, h0=1, evict_order=0):
    n, V, f, K, drop, mode, ftick, ppm, seed, ticks = case
    kw = dict(view=V, fanout=f, inbox=K, drop_pct=drop, fail_mode=mode, fail_tick=ftick,
              fail_ppm=ppm, seed=seed, h0=h0, evict_order=evict_order)
    orc = PviewOracle(n, **kw)
    rng = np.random.default_rng(seed)
    with PviewEngine(n, max_ticks=ticks, **kw) as eng:
        eng._tick = 0
        src, dst = orc.messages()
        m = eng.messages()
        assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
            sorted(zip(src.tolist(), dst.tolist()))
        _cmp_rows(eng, orc, range(0, n, max(1, n // 50)))
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            eng._tick = t
            got = eng.digest(t)
            assert got == want, "tick %d\n got %s\nwant %s" % (t, got, want)
            if t % 5 == 0 or t == ftick + 1:
                src, dst = orc.messages()
                m = eng.messages()
                assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                    sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
                _cmp_rows(eng, orc, sorted(set(rng.integers(0, n, 40).tolist())))
        _cmp_rows(eng, orc, range(n) if n <= 2000 else range(0, n, 7))


# Row shards launch the split kernels without a host wait for the bucket sizes (PviewTickArgs.
# nowait: every k range on `rows` workgroups, those past their bucket exit at once; the drain
# classes on persistent grids; their sizes copied back without a wait). GSP_TEST_PV_NOWAIT=1
# forces that form on one shard, =0 puts the exact grids back on an in-process group. Ticks are
# queued four at a time, so the host runs ahead of the device.
@pytest.mark.parametrize("inbox", [7, 0])
@pytest.mark.parametrize("nowait,group", [("1", 1), ("0", 3)], ids=["nowait_g1", "exact_g3"])
def test_pview_nowait_grids_match_oracle(inbox, nowait, group, monkeypatch):
    monkeypatch.setenv("GSP_TEST_PV_NOWAIT", nowait)
    monkeypatch.setenv("GSP_TEST_PV_COUNT_ROWS", "1")
    n, ticks = 2500, 16
    kw = dict(view=32, fanout=8 if inbox == 0 else 3, inbox=inbox, drop_pct=10, fail_mode=1,
              fail_tick=6, fail_ppm=30000, seed=23)
    orc = PviewOracle(n, **kw)
    with PviewEngine(n, max_ticks=ticks, group=group, **kw) as eng:
        for t0 in range(0, ticks, 4):
            want = [orc.step() for _ in range(4)]
            eng.step(4)
            for i, w in enumerate(want):
                t = t0 + i + 1
                assert eng.digest(t) == w, "tick %d" % t
                assert eng.rows_run(t) == n, "tick %d: %d rows run" % (t, eng.rows_run(t))
        eng._tick = ticks
        _cmp_rows(eng, orc, range(0, n, 3))
        if inbox == 0:                               # the class sizes reached the host
            st = eng.drain_stats()
            assert sum(st["rows"]) > 0 and sum(st["messages"]) >= 8 * sum(st["rows"])


SHARD_CASES = [
    # n, view, fanout, inbox, drop, fail_mode, fail_tick, ppm, seed, ticks, shards
    (3000, 64, 3, 7, 10, 2, 6, 50000, 5, 20, 2),
    (2500, 256, 3, 7, 10, 1, 8, 30000, 21, 16, 3),   # uneven shard sizes
    (1200, 32, 8, 2, 0, 1, 5, 20000, 8, 18, 8),      # 8 shards, inbox overflow
]


@pytest.mark.parametrize("case", SHARD_CASES, ids=lambda c: "n%d_v%d_g%d" % (c[0], c[1], c[-1]))
def test_pview_row_shards_match_oracle(case):
    """Row-sharded engine (in-process group: the same pack / gather / CSR kernels as the
    RCCL path, exchange by device copies) against the oracle: digests every tick, message
    lists and views periodically, and cross-shard bytes moved."""
    n, V, f, K, drop, mode, ftick, ppm, seed, ticks, G = case
    kw = dict(view=V, fanout=f, inbox=K, drop_pct=drop, fail_mode=mode, fail_tick=ftick,
              fail_ppm=ppm, seed=seed)
    orc = PviewOracle(n, **kw)
    with PviewEngine(n, max_ticks=ticks, group=G, **kw) as eng:
        assert eng.layout() == (G, 0, 0, n)
        eng._tick = 0
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            eng._tick = t
            assert eng.digest(t) == want, "tick %d" % t
            if t % 6 == 0:
                src, dst = orc.messages()
                m = eng.messages()
                assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                    sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
        _cmp_rows(eng, orc, range(n))
        assert eng.perf()["xgmi_bytes"] > 0


def test_pview_rccl_one_rank():
    """The RCCL code path of the row-sharded engine with a world of one (all-gather of the
    counts, the send/recv group with no peers) matches the one-GPU engine."""
    from gossip_protocol_amd.scale import nccl_unique_id
    n, ticks = 2000, 12
    kw = dict(view=64, fanout=3, inbox=7, drop_pct=10, fail_mode=1, fail_tick=5,
              fail_ppm=30000, seed=17, max_ticks=ticks)
    with PviewEngine(n, **kw) as a, PviewEngine(n, rank=0, world=1, nccl_id=nccl_unique_id(),
                                                **kw) as b:
        a.step(ticks)
        b.step(ticks)
        for t in range(1, ticks + 1):
            assert a.digest(t) == b.digest(t)
        for r in range(0, n, 37):
            assert a.row(r)[1] == b.row(r)[1] and np.array_equal(a.row(r)[0], b.row(r)[0])


def test_pview_capacity_error_stops_the_job(monkeypatch):
    """A receiver sent more messages than the receipt bound (1,024; lowered to 2 through the
    test-only GSP_TEST_MAX_SEGMENT) stops the job at that tick: its tick kernel and every later
    one run no row.  The flag reaches the host by an async copy at the end of each step call:
    sync() (and every read) reports it, and so does every step call made after the copy
    landed -- never state computed from a skipped row."""
    from gossip_protocol_amd._lib import GspError
    monkeypatch.setenv("GSP_TEST_MAX_SEGMENT", "2")
    with PviewEngine(300, view=64, fanout=8, inbox=7, max_ticks=10) as eng:
        eng.step(1)
        with pytest.raises(GspError, match="more than 2 messages at tick 1"):
            eng.sync()
        with pytest.raises(GspError, match="more than 2 messages at tick 1"):
            eng.step(1)
        with pytest.raises(GspError, match="at tick 1"):
            eng.digest(1)
    monkeypatch.delenv("GSP_TEST_MAX_SEGMENT")
    with PviewEngine(300, view=64, fanout=8, inbox=7, max_ticks=10) as eng:
        eng.step(3)
        assert eng.digest(3)["node_rounds"] == 300


def test_pview_row_exchange_past_its_posted_size_stops_the_job(monkeypatch):
    """The row exchange posts sizes derived from earlier ticks' counts (RCCL needs them when the
    call is posted; no host wait on the stream).  GSP_TEST_ROWX_TIGHT=1 makes an in-process
    group post and check them with no margin, so a count above every earlier one must stop the
    job loudly -- GSP_ERR_CAPACITY naming the tick -- never merge a truncated exchange."""
    from gossip_protocol_amd._lib import GspError
    monkeypatch.setenv("GSP_TEST_ROWX_TIGHT", "1")
    with PviewEngine(3000, view=64, fanout=3, inbox=7, drop_pct=10, fail_mode=2, fail_tick=5,
                     fail_ppm=50000, seed=5, group=3, max_ticks=30) as eng:
        with pytest.raises(GspError, match="row exchange at tick"):
            eng.step(30)
            eng.sync()


@pytest.mark.parametrize("form", ["group3", "rank"])
def test_pview_capacity_error_stops_every_shard(monkeypatch, form):
    """An overflow in one row shard stops the whole job: an in-process group's shards read one
    flag, and a rank's flag travels with the row-exchange counts, so every rank returns the
    error at the same tick instead of one rank leaving the others in a collective."""
    from gossip_protocol_amd._lib import GspError
    from gossip_protocol_amd.scale import nccl_unique_id
    monkeypatch.setenv("GSP_TEST_MAX_SEGMENT", "2")
    kw = dict(view=64, fanout=8, inbox=7, max_ticks=10)
    kw.update(group=3) if form == "group3" else kw.update(rank=0, world=1, nccl_id=nccl_unique_id())
    with PviewEngine(300, **kw) as eng:
        eng.step(1)
        with pytest.raises(GspError, match="at tick 1"):
            eng.sync()
        with pytest.raises(GspError, match="at tick 1"):
            eng.step(1)
            eng.sync()
        with pytest.raises(GspError, match="at tick 1"):
            eng.digest(1)


def test_pview_full_size_properties():
    """BASELINE config 5 at its real size on one GPU: 1,048,576 nodes, V = 256, fanout 3,
    inbox 7, 10 % drop, 5 % contiguous crash at t = 10 -- the bench's line item, checked.

    * node-rounds = the alive count (every node up to tick 10, n - 52,428 after);
    * the message list of tick 12 is the digest's sent - dropped, crashed nodes send nothing,
      and tick 13 delivers or overflows exactly the messages addressed to alive nodes;
    * sampled views are sorted, distinct, never list their owner and hold <= V entries;
    * rows of tick 13 recomputed on the host from the tick-12 views and the message list by
      oracle/pview_oracle.c's per-row rule (gsp_pview_oracle_row_step: the reference's merge /
      TREMOVE rules, MP1Node.cpp:234-301, 339-348, plus the bounded view's eviction) equal the
      device's -- for receivers with 0, 1, 3 and more than 7 (inbox overflow) messages, which
      exercises the 21-bit id field, every view-count variant class and eviction at full load.
    """
    from tests.oracle_binding import PviewCfg, load_oracle, pview_row_step
    n, seed, ftick, ppm = 1 << 20, 0x5EED, 10, 50000
    kw = dict(view=256, fanout=3, inbox=7, drop_pct=10, fail_mode=2, fail_tick=ftick,
              fail_ppm=ppm, seed=seed)
    cfg = PviewCfg(n, 256, 3, 7, 10, 20, 1, 2, ftick, ppm, seed)
    # the crashed block, from the oracle's Philox (oracle/pview_oracle.c pv_fail_ticks)
    start = load_oracle().gsp_oracle_draw(0x4641494C, seed, ftick, 0xFFFFFFFF, 0, 0) % n
    m = n * ppm // 1000000
    dead = np.zeros(n, bool)
    dead[(start + np.arange(m)) % n] = True
    with PviewEngine(n, max_ticks=16, **kw) as eng:
        eng.step(12)
        ds = {t: eng.digest(t) for t in range(1, 13)}
        for t in range(1, 13):
            assert ds[t]["node_rounds"] == (n if t <= ftick else n - m), t
            assert ds[t]["delivered"] <= 7 * ds[t]["node_rounds"]
        msgs = eng.messages()                       # sent at tick 12, merged at 13
        assert msgs.shape == (n, 3)
        assert (msgs[dead] < 0).all()
        live = msgs[msgs >= 0]
        assert len(live) == ds[12]["sent"] - ds[12]["dropped"]
        cnt = np.bincount(live, minlength=n)
        rng = np.random.default_rng(5)
        alive_rows = np.nonzero(~dead)[0]
        targets = []
        for want in (0, 1, 3):
            cand = alive_rows[cnt[alive_rows] == want]
            targets.append(int(cand[rng.integers(len(cand))]))
        cand = alive_rows[cnt[alive_rows] > 7]
        assert len(cand) > 0
        targets.append(int(cand[rng.integers(len(cand))]))
        targets.append(int(alive_rows[np.argmax(cnt[alive_rows])]))
        senders = {r: np.nonzero((msgs == r).any(axis=1))[0].tolist() for r in targets}

        def view(x, t):                             # (ids, hb, absolute ts) of x at tick t
            buf, ln = eng.row(x)
            ids, hb, ts5 = unpack_view(buf, ln)
            assert ln <= 256 and np.all(np.diff(ids) > 0) and x not in ids
            return ids, hb, t - ((t - ts5) & 31)

        prev = {x: view(x, 12) for x in set(targets) | {s for v in senders.values() for s in v}}
        for x in rng.integers(0, n, 64).tolist():
            view(x, 12)
        eng.step(1)
        d13 = eng.digest(13)
        assert d13["delivered"] + d13["overflow"] == int(cnt[~dead].sum())
        for r in targets:
            (ids, hb, ts), _ = pview_row_step(cfg, 13, r, prev[r], senders[r],
                                              [prev[s] for s in senders[r]])
            gi, gh, gt = view(r, 13)
            assert np.array_equal(gi, ids), "ids of row %d (%d senders)" % (r, len(senders[r]))
            assert np.array_equal(gh, hb), "hb of row %d" % r
            assert np.array_equal(gt, ts), "ts of row %d" % r


def test_pview_eight_row_shards_full_size():
    """BASELINE config 5 at full size as 8 row shards in one process: the
    multi-GPU layout's pack / gather / CSR / exchange kernels with the RCCL send / recv
    replaced by device copies -- the best proxy of the 8-GPU run on a one-GPU box.  Every
    tick's digest equals the one-shard engine's, sampled views are identical, and the bytes
    that cross shards per tick (the per-(sender, shard) deduplicated sender views plus the
    12-byte message records, EmulNet.cpp:87-177 across shards) are reported next to DESIGN's
    estimate of 4.2 GB per tick at G = 8."""
    import json
    import os
    n, ticks, G = 1 << 20, 12, 8
    kw = dict(view=256, fanout=3, inbox=7, drop_pct=10, fail_mode=2, fail_tick=10,
              fail_ppm=50000, seed=0x5EED)
    rng = np.random.default_rng(8)
    sample = sorted(set(rng.integers(0, n, 300).tolist()) | {0, 1, n - 1, n // G, n // G - 1})
    with PviewEngine(n, max_ticks=ticks, **kw) as one:
        one.step(ticks)
        want = [one.digest(t) for t in range(1, ticks + 1)]
        rows = {r: one.row(r) for r in sample}
    with PviewEngine(n, max_ticks=ticks, group=G, **kw) as eng:
        assert eng.layout() == (G, 0, 0, n)
        xgmi = []
        for t in range(1, ticks + 1):
            before = eng.perf()["xgmi_bytes"]
            eng.step(1)
            xgmi.append(eng.perf()["xgmi_bytes"] - before)
            assert eng.digest(t) == want[t - 1], "tick %d" % t
        for r in sample:
            buf, ln = eng.row(r)
            assert ln == rows[r][1] and np.array_equal(buf, rows[r][0]), "row %d" % r
    # every tick after the first moves each alive sender's view to ~2 other shards, packed on
    # the wire (ids as 16-bit low halves + 33 run bounds, 1,096 B per view instead of 2,048 B):
    # round 4 accounted 4.0-4.6 GB per tick, VERDICT r04 item 4 asks for <= 3.0 GB
    assert all(1e9 < x <= 3.0e9 for x in xgmi[1:]), xgmi
    rec = {"n": n, "shards": G, "ticks": ticks, "xgmi_bytes_per_tick": xgmi}
    out = os.environ.get("GSP_TEST_RECORD_DIR")
    if out:
        with open(os.path.join(out, "pview_rows8_xgmi.json"), "w") as f:
            json.dump(rec, f)
    print(json.dumps(rec))
