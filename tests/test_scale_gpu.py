"""SCALE mode on the GPU against the scale-protocol oracle (oracle/scale_oracle.c).

Small n (the oracle finishes in seconds): every tick's digest (node-rounds, merges, sends,
drops, deliveries, join/remove counts, order-independent event hash) must be identical,
the message lists identical, and full membership state identical: presence and heartbeat
exactly, timestamps modulo 32 (the device's packed representation; DESIGN.md proves every
comparison the protocol makes is exact under it).
"""
import numpy as np
import pytest

from gossip_protocol_amd.scale import FAIL_BLOCK, FAIL_NONE, FAIL_RANDOM, ScaleEngine, unpack
from tests.oracle_binding import ScaleOracle

pytestmark = pytest.mark.gpu

CASES = [
    # n, fanout, drop_pct, fail_mode, fail_tick, fail_ppm, seed, ticks
    (64, 3, 0, FAIL_NONE, 10, 0, 1, 40),
    (300, 3, 10, FAIL_RANDOM, 10, 50000, 7, 45),
    (2048, 3, 0, FAIL_RANDOM, 10, 10000, 0x5EED, 40),
    (2100, 5, 10, FAIL_BLOCK, 8, 50000, 99, 36),      # ragged: n not a multiple of 2048
    (4096, 1, 30, FAIL_RANDOM, 5, 20000, 3, 30),
]


def _compare_state(eng, orc, n, rows):
    for r in rows:
        pres_o, hb_o, ts_o = orc.row(r)
        pres_d, hb_d, ts5_d = unpack(eng.row(r))
        assert np.array_equal(pres_d, pres_o.astype(bool)), "presence row %d" % r
        assert np.array_equal(hb_d[pres_d], hb_o[pres_d]), "hb row %d" % r
        assert np.array_equal(ts5_d[pres_d], ts_o[pres_d] & 31), "ts row %d" % r
        if orc.fail_tick(r) >= eng.tick:
            assert eng.own_hb(r) == orc.own_hb(r), "own hb row %d" % r


VARIANTS = {
    # name: (shards in one process, layout, packed merge, cache policy)
    "fused": (1, "columns", 1, 1),
    "fused_scalar_merge": (1, "columns", 0, 0),
    "fused_nt_all": (1, "columns", 1, 3),
    "columns2": (2, "columns", 1, 1),
    "columns3": (3, "columns", 1, 1),
    "columns4_scalar": (4, "columns", 0, 2),
    "rows2": (2, "rows", 1, 1),
    "rows3": (3, "rows", 1, 1),
    "rows8_scalar": (8, "rows", 0, 2),
    "fused_pipe": (1, "columns", 1, 5),
    "rows3_pipe": (3, "rows", 1, 5),
    "columns2_pipe": (2, "columns", 1, 5),
}
VARIANT_CASES = [(c, "fused") for c in CASES] + [
    (CASES[1], "fused_scalar_merge"), (CASES[3], "fused_nt_all"), (CASES[1], "columns2"),
    (CASES[3], "columns3"), (CASES[4], "columns2"), (CASES[2], "columns4_scalar"),
    (CASES[0], "rows2"), (CASES[1], "rows3"), (CASES[3], "rows2"), (CASES[4], "rows3"),
    (CASES[2], "rows8_scalar"), (CASES[3], "fused_pipe"), (CASES[4], "fused_pipe"),
    (CASES[1], "rows3_pipe"), (CASES[3], "columns2_pipe")]


@pytest.mark.parametrize("case,variant", VARIANT_CASES,
                         ids=lambda x: x if isinstance(x, str) else "n%d_f%d_d%d_m%d" % x[:4])
def test_scale_matches_oracle(case, variant):
    n, f, drop, mode, ftick, ppm, seed, ticks = case
    group, layout, packed, policy = VARIANTS[variant]
    orc = ScaleOracle(n, fanout=f, drop_pct=drop, fail_mode=mode, fail_tick=ftick, fail_ppm=ppm,
                      seed=seed)
    rng = np.random.default_rng(seed)
    with ScaleEngine(n, fanout=f, drop_pct=drop, fail_mode=mode, fail_tick=ftick, fail_ppm=ppm,
                     seed=seed, max_ticks=ticks, group=group, layout=layout) as eng:
        eng.set_merge(packed)
        eng.set_cache_policy(policy)
        # tick-0 sends (pre-joined bootstrap)
        src, dst = orc.messages()
        m = eng.messages()
        got = sorted((s, d) for s in range(n) for d in m[s] if d >= 0)
        assert got == sorted(zip(src.tolist(), dst.tolist()))
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            got = eng.digest(t)
            assert got == want, "tick %d digest\n got %s\nwant %s" % (t, got, want)
            if t % 7 == 0 or t in (1, ftick + 1, ftick + 21, ticks):
                src, dst = orc.messages()
                m = eng.messages()
                gm = sorted((s, d) for s in range(n) for d in m[s] if d >= 0)
                assert gm == sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
                rows = sorted(set(rng.integers(0, n, 24).tolist()) | {0, n - 1})
                _compare_state(eng, orc, n, rows)
        _compare_state(eng, orc, n, range(n) if n <= 512 else range(0, n, 61))
        perf = eng.perf()
        assert perf["ticks"] == ticks and perf["merge_ms"] > 0
        if layout == "rows" and group > 1:
            assert perf["xgmi_bytes"] > 0


TFAIL_CASES = [
    # (case, shards, layout, merge, tfail): TFAIL suspicion, the reference's
    # TFAIL = 5 (MP1Node.h:22) and a few others
    (CASES[2], 1, "columns", 1, 5),
    (CASES[1], 1, "columns", 0, 5),
    (CASES[3], 1, "columns", 1, 3),
    (CASES[4], 1, "columns", 1, 12),
    (CASES[1], 2, "columns", 1, 5),
    (CASES[3], 3, "rows", 1, 5),
]


@pytest.mark.parametrize("case,shards,layout,merge,tfail", TFAIL_CASES,
                         ids=lambda x: "n%d_f%d_d%d_m%d" % x[:4] if isinstance(x, tuple) else str(x))
def test_tfail_matches_oracle(case, shards, layout, merge, tfail):
    """TFAIL suspicion: members tfail or more ticks stale are listed but neither gossiped nor
    chosen as peers nor counted.  Digests every tick, messages and rows vs the oracle."""
    n, f, drop, mode, ftick, ppm, seed, ticks = case
    orc = ScaleOracle(n, fanout=f, drop_pct=drop, fail_mode=mode, fail_tick=ftick, fail_ppm=ppm,
                      seed=seed, tfail=tfail)
    plain = ScaleOracle(n, fanout=f, drop_pct=drop, fail_mode=mode, fail_tick=ftick,
                        fail_ppm=ppm, seed=seed)
    differs = False
    with ScaleEngine(n, fanout=f, drop_pct=drop, fail_mode=mode, fail_tick=ftick, fail_ppm=ppm,
                     seed=seed, max_ticks=ticks, group=shards, layout=layout, tfail=tfail) as eng:
        eng.set_merge(merge)
        for t in range(1, ticks + 1):
            want = orc.step()
            differs |= want != plain.step()
            eng.step(1)
            assert eng.digest(t) == want, "tick %d" % t
            if t % 9 == 0 or t == ticks:
                src, dst = orc.messages()
                m = eng.messages()
                assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                    sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
        _compare_state(eng, orc, n, range(0, n, 7))
    assert differs, "suspicion changed nothing: the case does not exercise TFAIL"
    orc.close()
    plain.close()


SWIM_CASES = [
    # (case, shards, layout, merge, tfail, swim): SWIM ping/ack probing
    (CASES[1], 1, "columns", 1, 0, 2),
    (CASES[1], 1, "columns", 0, 0, 1),
    (CASES[3], 1, "columns", 1, 0, 1),
    (CASES[4], 1, "columns", 1, 0, 3),
    (CASES[2], 1, "columns", 1, 5, 2),
    (CASES[1], 3, "rows", 1, 0, 2),
    (CASES[3], 2, "rows", 1, 5, 1),
    (CASES[1], 2, "columns", 1, 0, 2),
    (CASES[3], 3, "columns", 0, 5, 1),
    (CASES[4], 2, "columns", 1, 0, 3),
]


@pytest.mark.parametrize("case,shards,layout,merge,tfail,swim", SWIM_CASES,
                         ids=lambda x: "n%d_f%d_d%d_m%d" % x[:4] if isinstance(x, tuple) else str(x))
def test_swim_matches_oracle(case, shards, layout, merge, tfail, swim):
    """SWIM probing: one probe target per node per tick, answered -> ts refreshed, unanswered
    -> removed at the next tick.  Digests every tick, messages and rows vs the oracle."""
    n, f, drop, mode, ftick, ppm, seed, ticks = case
    orc = ScaleOracle(n, fanout=f, drop_pct=drop, fail_mode=mode, fail_tick=ftick, fail_ppm=ppm,
                      seed=seed, tfail=tfail, swim=swim)
    plain = ScaleOracle(n, fanout=f, drop_pct=drop, fail_mode=mode, fail_tick=ftick,
                        fail_ppm=ppm, seed=seed, tfail=tfail)
    differs = False
    with ScaleEngine(n, fanout=f, drop_pct=drop, fail_mode=mode, fail_tick=ftick, fail_ppm=ppm,
                     seed=seed, max_ticks=ticks, group=shards, layout=layout, tfail=tfail,
                     swim=swim) as eng:
        eng.set_merge(merge)
        for t in range(1, ticks + 1):
            want = orc.step()
            differs |= want != plain.step()
            eng.step(1)
            assert eng.digest(t) == want, "tick %d" % t
            if t % 9 == 0 or t == ticks:
                src, dst = orc.messages()
                m = eng.messages()
                assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                    sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
                _compare_state(eng, orc, n, range(t % 5, n, 11))
        _compare_state(eng, orc, n, range(0, n, 3))
    assert differs, "probing changed nothing: the case does not exercise SWIM"
    orc.close()
    plain.close()


@pytest.mark.parametrize("swim", [0, 2])
@pytest.mark.parametrize("tfail", [0, 5])
def test_rccl_rank_path_one_rank(tfail, swim):
    """The RCCL code path (ncclCommInitRank, all-gather, all-reduce MAX) with a world of one:
    a one-rank communicator still runs the column protocol and must match the oracle, with
    TFAIL suspicion and SWIM probing (whose probe results cross the same all-reduce) on."""
    from gossip_protocol_amd.scale import nccl_unique_id
    n, ticks = 1024, 16
    kw = dict(fanout=3, drop_pct=10, fail_mode=FAIL_RANDOM, fail_tick=5, fail_ppm=20000, seed=4,
              tfail=tfail, swim=swim)
    orc = ScaleOracle(n, **kw)
    with ScaleEngine(n, max_ticks=ticks, rank=0, world=1, nccl_id=nccl_unique_id(), **kw) as eng:
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            assert eng.digest(t) == want, t
        _compare_state(eng, orc, n, range(0, n, 37))


# The launch form bench.py's headline runs (ScaleEngine(65536, group=8): 8 in-process column
# tiles sharing one CSR, one count table, one pick resolve over every tile's bitmap and one
# finalize; DESIGN.md "Column tiles"), against the oracle at n where it runs in seconds:
# n = 16,384 gives 2,048-column tiles; n = 12,000 a ragged tile 5 (columns 10,240..11,999)
# and two empty tiles.  The per-entry rules are MP1Node.cpp:234-256 (merge) and :335-348 (ops).
RANDOM8 = dict(fanout=3, drop_pct=10, fail_mode=FAIL_RANDOM, fail_tick=6, fail_ppm=20000,
               seed=21, tremove=8)
COLUMNS8 = [
    # id, n, engine / oracle keywords, policy, events, ticks
    ("plain", 16384, RANDOM8, None, False, 16),
    ("ragged", 12000, dict(fanout=4, drop_pct=0, fail_mode=FAIL_BLOCK, fail_tick=5,
                           fail_ppm=50000, seed=5, tremove=7), None, False, 15),
    ("tfail_swim", 16384, dict(RANDOM8, drop_pct=20, seed=33, tremove=9, tfail=4, swim=2), None,
     False, 15),
    ("policy_events", 16384, dict(RANDOM8, seed=44), dict(
        drop_window=(3, 9), step_rate=0.005, intro_list=8, fail_events=[(9, 3, 0), (11, 2, 20000)]),
     True, 15),
]


@pytest.mark.parametrize("case", COLUMNS8, ids=lambda c: c[0])
def test_columns8_matches_oracle(case):
    """8 column tiles in one process (the headline form) = the oracle: every digest, every
    tick's event multiset (policy case), messages and sampled rows along the run, then every
    61st row in full."""
    from gossip_protocol_amd import _lib
    from gossip_protocol_amd.scale import make_policy
    from tests.oracle_binding import make_policy as oracle_policy
    _, n, kw, pol, events, ticks = case
    orc = ScaleOracle(n, policy=oracle_policy(**pol) if pol else None, **kw)
    rng = np.random.default_rng(n)
    with ScaleEngine(n, max_ticks=ticks, group=8, policy=make_policy(**pol) if pol else None,
                     events=events, **kw) as eng:
        assert eng.layout() == (8, 0, 2048)
        src, dst = orc.messages()
        m = eng.messages()
        assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
            sorted(zip(src.tolist(), dst.tolist()))
        if events:
            eng.drain_events()
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            assert eng.digest(t) == want, "tick %d\n got %s\nwant %s" % (t, eng.digest(t), want)
            if events:
                rec, lost = eng.drain_events()
                k, tk, r, x = _lib.split_events(rec)
                ok, orr, ox = orc.events()
                assert lost == 0 and np.all(tk == t)
                assert sorted(zip(k.tolist(), r.tolist(), x.tolist())) == \
                    sorted(zip(ok.tolist(), orr.tolist(), ox.tolist())), "events tick %d" % t
            if t % 5 == 0 or t == kw["fail_tick"] + 1:
                src, dst = orc.messages()
                m = eng.messages()
                assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
                    sorted(zip(src.tolist(), dst.tolist())), "messages tick %d" % t
                rows = sorted(set(rng.integers(0, n, 16).tolist()) | {0, 2047, 2048, n - 1})
                _compare_state(eng, orc, n, rows)
        _compare_state(eng, orc, n, range(0, n, 61))
    orc.close()


def test_columns_equal_fused_full_size():
    """Config-3 size: 4 column shards (in-process exchange) give the one-GPU results."""
    n, ticks = 65536, 14
    kw = dict(fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000, seed=0x5EED,
              max_ticks=ticks)
    with ScaleEngine(n, **kw) as a:
        a.step(ticks)
        da = [a.digest(t) for t in range(1, ticks + 1)]
        ra = {r: a.row(r) for r in (0, 12345, n - 1)}
        ma = a.messages()
    with ScaleEngine(n, group=4, **kw) as b:
        assert b.layout() == (4, 0, 16384)
        b.step(ticks)
        db = [b.digest(t) for t in range(1, ticks + 1)]
        for r, row in ra.items():
            assert np.array_equal(b.row(r), row), r
        assert np.array_equal(b.messages(), ma)
    assert da == db


def test_columns8_equal_fused_full_size_with_events():
    """The headline workload itself (config 3: 65,536 nodes, fanout 3, 1 % random crash; here
    at t = 2 so that the removals start inside the run) as bench.py launches it -- 8 column
    tiles -- against the fused one-GPU kernel: every tick's digest, every tick's drained event
    records (sorted 64-bit records, tick field included), the messages and sampled rows."""
    n, ticks = 65536, 30
    kw = dict(fanout=3, fail_mode=FAIL_RANDOM, fail_tick=2, fail_ppm=10000, seed=0x5EED,
              max_ticks=ticks, events=True, event_cap=1 << 26)
    rows = (0, 8191, 8192, 40000, n - 1)
    ref = {}
    with ScaleEngine(n, **kw) as a:
        a.drain_events()
        for t in range(1, ticks + 1):
            a.step(1)
            rec, lost = a.drain_events()
            assert lost == 0
            ref[t] = (a.digest(t), np.sort(rec))
        ra = {r: a.row(r) for r in rows}
        ma = a.messages()
    removes = 0
    with ScaleEngine(n, group=8, **kw) as b:
        assert b.layout() == (8, 0, 8192)
        b.drain_events()
        for t in range(1, ticks + 1):
            b.step(1)
            rec, lost = b.drain_events()
            assert lost == 0
            assert b.digest(t) == ref[t][0], t
            assert np.array_equal(np.sort(rec), ref[t][1]), "event records of tick %d" % t
            removes += b.digest(t)["removes"]
        for r, row in ra.items():
            assert np.array_equal(b.row(r), row), r
        assert np.array_equal(b.messages(), ma)
    assert removes > 1000000          # the crash wave (655 nodes) is inside the run


def test_rows_equal_fused_full_size():
    """Config-3 size: 4 row shards (in-process: the pack / gather / CSR kernels of the RCCL
    row path, exchange by device copies) give the one-GPU results."""
    n, ticks = 65536, 14
    kw = dict(fanout=3, fail_mode=FAIL_RANDOM, fail_tick=10, fail_ppm=10000, seed=0x5EED,
              max_ticks=ticks)
    with ScaleEngine(n, **kw) as a:
        a.step(ticks)
        da = [a.digest(t) for t in range(1, ticks + 1)]
        ra = {r: a.row(r) for r in (0, 16383, 16384, 40000, n - 1)}
        ma = a.messages()
    with ScaleEngine(n, group=4, layout="rows", **kw) as b:
        b.step(ticks)
        db = [b.digest(t) for t in range(1, ticks + 1)]
        for r, row in ra.items():
            assert np.array_equal(b.row(r), row), r
        assert np.array_equal(b.messages(), ma)
        assert b.perf()["xgmi_bytes"] > 0
    assert da == db


def test_rccl_rows_one_rank():
    """The RCCL row path (count broadcasts, all-gather, send/recv group with no peers) with a
    world of one matches the oracle."""
    from gossip_protocol_amd.scale import nccl_unique_id
    n, ticks = 1500, 14
    orc = ScaleOracle(n, fanout=3, drop_pct=10, fail_mode=FAIL_RANDOM, fail_tick=5,
                      fail_ppm=20000, seed=8)
    with ScaleEngine(n, fanout=3, drop_pct=10, fail_mode=FAIL_RANDOM, fail_tick=5, fail_ppm=20000,
                     seed=8, max_ticks=ticks, rank=0, world=1, nccl_id=nccl_unique_id(),
                     layout="rows") as eng:
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            assert eng.digest(t) == want, t
        _compare_state(eng, orc, n, range(0, n, 37))


def test_scale_full_size_properties():
    """BASELINE config 3 size (65,536 full view): size-independent properties.

    * conservation: delivered + lost-to-crashed = sent - dropped of the previous tick;
    * node-rounds equal the alive count; merges = delivered + sum of sender list sizes;
    * a sampled row recomputed on the host from the previous tick's rows and the message
      list equals the device's row (checks the fused kernel at full size).
    """
    n = 65536
    with ScaleEngine(n, fanout=3, drop_pct=0, fail_mode=FAIL_RANDOM, fail_tick=10,
                     fail_ppm=10000, seed=0x5EED, max_ticks=40) as eng:
        eng.step(12)
        d10, d11, d12 = eng.digest(10), eng.digest(11), eng.digest(12)
        alive = d12["node_rounds"]
        assert 0.985 * n < alive < 0.995 * n          # nodes crash at the end of tick 10
        assert d10["node_rounds"] == n and d11["node_rounds"] == alive
        assert d12["delivered"] <= d11["sent"] - d11["dropped"]
        assert d12["merges"] >= d12["delivered"]
        # host recompute of a few rows for tick 13
        msgs = eng.messages()           # sent at tick 12, delivered at 13
        rows_prev = {}
        targets = [5, 4097, n - 3]
        senders = {}
        for s in range(n):
            for dd in msgs[s]:
                if dd in targets:
                    senders.setdefault(int(dd), []).append(s)
        need = set(targets) | {s for v in senders.values() for s in v}
        for r in need:
            rows_prev[r] = eng.row(r).astype(np.uint32)
        eng.step(1)
        t5, tr = 13 & 31, 20
        for r in targets:
            e = rows_prev[r].copy()
            for s in sorted(senders.get(r, [])):
                v = rows_prev[s]
                he, hv = e >> 5, v >> 5
                upd = np.where(hv > he, (v & 0xFFE0) | t5, e)
                add = np.where((v != 0) & (((t5 - v) & 31) < tr), v, 0)
                e = np.where(e != 0, upd, add)
                e[s] = (((e[s] >> 5) + 1) << 5) | t5
            e[r] = 0
            e = np.where((e != 0) & (((t5 - e) & 31) >= tr), 0, e)
            assert np.array_equal(e.astype(np.uint16), eng.row(r)), "row %d" % r


def test_capacity_error_stops_the_job(monkeypatch):
    """A receiver sent more messages than a test's segment bound (none by default -- round 4:
    segments past the LDS sort's 1,024 are sorted in HBM; lowered to 2 here through the
    test-only GSP_TEST_MAX_SEGMENT) stops the job loudly: the device flags the
    tick and every later tick kernel runs no row.  The flag reaches the host by an async copy
    at the end of each step call: sync() and every read return GSP_ERR_CAPACITY, and so does
    every gsp_scale_step call made after the copy landed -- never state computed from a
    skipped row."""
    from gossip_protocol_amd._lib import GspError
    monkeypatch.setenv("GSP_TEST_MAX_SEGMENT", "2")
    with ScaleEngine(256, fanout=8, max_ticks=10) as eng:
        eng.step(1)                      # tick 1: ~8 messages per receiver > 2
        with pytest.raises(GspError, match="more than 2 messages at tick 1"):
            eng.sync()
        with pytest.raises(GspError, match="more than 2 messages at tick 1"):
            eng.step(1)
        with pytest.raises(GspError, match="at tick 1"):
            eng.digest(1)
    monkeypatch.delenv("GSP_TEST_MAX_SEGMENT")
    with ScaleEngine(256, fanout=8, max_ticks=10) as eng:   # the default bound: no error
        eng.step(3)
        assert eng.digest(3)["node_rounds"] == 256


@pytest.mark.parametrize("tiles", [2, 4])
@pytest.mark.parametrize("variant", ["plain", "tfail_swim", "policy_events"])
def test_rccl_rank_path_tiled(tiles, variant):
    """A rank holding `tiles` column tiles (gsp_scale_create_rank_tiled) over an RCCL
    communicator of one rank: the tiles share the rank's CSR / counts / picks, the counts of its
    tiles go through the in-place all-gather and the picks through the all-reduce MAX.  Every
    digest, the message list and sampled rows equal the oracle."""
    from gossip_protocol_amd.scale import make_policy, nccl_unique_id
    from tests.oracle_binding import make_policy as oracle_policy
    n, ticks = 4096 * tiles, 14
    kw = dict(fanout=3, drop_pct=10, fail_mode=FAIL_RANDOM, fail_tick=5, fail_ppm=20000, seed=6)
    pol = None
    if variant == "tfail_swim":
        kw.update(tfail=5, swim=2)
    if variant == "policy_events":
        # 20 joiners a tick (step_rate 0.05): every new node gossips to the introducer first
        # (a burst of > 1024 joiners: test_policy_gpu.py::test_full_view_join_burst_*)
        pol = dict(drop_window=(2, 9), step_rate=0.05, intro_list=4, fail_events=[(8, 3, 0)])
    orc = ScaleOracle(n, policy=oracle_policy(**pol) if pol else None, **kw)
    with ScaleEngine(n, max_ticks=ticks, rank=0, world=1, nccl_id=nccl_unique_id(), tiles=tiles,
                     policy=make_policy(**pol) if pol else None,
                     events=variant == "policy_events", **kw) as eng:
        assert eng.layout()[0] == tiles
        for t in range(1, ticks + 1):
            want = orc.step()
            eng.step(1)
            assert eng.digest(t) == want, t
            if variant == "policy_events":
                from gossip_protocol_amd import _lib
                rec, lost = eng.drain_events()
                k, tk, r, x = _lib.split_events(rec)
                ok, orr, ox = orc.events()
                assert lost == 0 and sorted(zip(k.tolist(), r.tolist(), x.tolist())) == \
                    sorted(zip(ok.tolist(), orr.tolist(), ox.tolist())), t
        src, dst = orc.messages()
        m = eng.messages()
        assert sorted((s, d) for s in range(n) for d in m[s] if d >= 0) == \
            sorted(zip(src.tolist(), dst.tolist()))
        _compare_state(eng, orc, n, range(0, n, 131))
    orc.close()


def test_config4_one_gpu_32_tiles_properties():
    """BASELINE config 4 (262,144 nodes, full view) on ONE GPU: 32 in-process column tiles of
    8,192 columns (the tile width config 3 runs fastest at); the table pair is 2 x 128 GiB of
    the MI355X's HBM.  Size-independent properties, as test_scale_full_size_properties:
    conservation of messages, node-rounds = alive nodes, and three rows of tick t + 1
    recomputed on the host from the tick-t rows and the message list with the reference's
    per-entry rules (MP1Node.cpp:234-256 merge, :335-348 TREMOVE)."""
    n = 262144
    with ScaleEngine(n, fanout=3, drop_pct=0, fail_mode=FAIL_RANDOM, fail_tick=3,
                     fail_ppm=10000, seed=0x5EED, max_ticks=8, group=32) as eng:
        assert eng.layout() == (32, 0, 8192)
        eng.step(5)
        d3, d4, d5 = eng.digest(3), eng.digest(4), eng.digest(5)
        alive = d5["node_rounds"]
        assert d3["node_rounds"] == n and d4["node_rounds"] == alive
        assert 0.985 * n < alive < 0.995 * n          # nodes crash at the end of tick 3
        assert d5["delivered"] <= d4["sent"] - d4["dropped"]
        assert d5["merges"] >= d5["delivered"] and d5["sent"] == 3 * alive
        msgs = eng.messages()           # sent at tick 5, delivered at 6
        from gossip_protocol_amd import _lib
        crash = _lib.fail_schedule(n, 0x5EED, FAIL_RANDOM, 3, 10000)
        targets = [r for r in (7, 8, 131071, 131072, n - 2, n - 3) if crash[r] > 6][::2][:3]
        dst = msgs.reshape(-1)
        src = np.repeat(np.arange(n), 3)
        senders = {r: sorted(src[dst == r].tolist()) for r in targets}
        need = set(targets) | {s for v in senders.values() for s in v}
        rows_prev = {r: eng.row(r).astype(np.uint32) for r in need}
        eng.step(1)
        t5, tr = 6 & 31, 20
        for r in targets:
            e = rows_prev[r].copy()
            for s in senders[r]:
                v = rows_prev[s]
                he, hv = e >> 5, v >> 5
                upd = np.where(hv > he, (v & 0xFFE0) | t5, e)
                add = np.where((v != 0) & (((t5 - v) & 31) < tr), v, 0)
                e = np.where(e != 0, upd, add)
                e[s] = (((e[s] >> 5) + 1) << 5) | t5
            e[r] = 0
            e = np.where((e != 0) & (((t5 - e) & 31) >= tr), 0, e)
            assert np.array_equal(e.astype(np.uint16), eng.row(r)), "row %d" % r


@pytest.mark.parametrize("form", ["rows3", "columns2", "rank_columns", "rank_rows"])
def test_capacity_error_stops_every_shard(monkeypatch, form):
    """A receiver overflow stops every shard of the job together: the shards of
    an in-process group read one flag; ranks of a communicator exchange it each tick (columns:
    inside the picks all-reduce; rows: with the row-exchange counts) and never return early
    from a step on their own async mirror, so no rank is left waiting in a collective."""
    from gossip_protocol_amd._lib import GspError
    from gossip_protocol_amd.scale import nccl_unique_id
    monkeypatch.setenv("GSP_TEST_MAX_SEGMENT", "2")
    kw = dict(fanout=8, max_ticks=10)
    if form == "rows3":
        kw.update(group=3, layout="rows")
    elif form == "columns2":
        kw.update(group=2)
    else:
        kw.update(rank=0, world=1, nccl_id=nccl_unique_id(),
                  layout="rows" if form == "rank_rows" else "columns")
    with ScaleEngine(2048, **kw) as eng:
        eng.step(1)                      # tick 1: ~8 messages per receiver > 2
        with pytest.raises(GspError, match="at tick 1"):
            eng.sync()
        with pytest.raises(GspError, match="at tick 1"):
            eng.step(1)
            eng.sync()
        with pytest.raises(GspError, match="at tick 1"):
            eng.digest(1)
