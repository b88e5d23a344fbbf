"""The partial-view restatement's per-row helper (CPU only).

gsp_pview_oracle_row_step is the rule gsp_pview_oracle_step applies to every row; the
full-size GPU test (tests/test_pview_gpu.py::test_pview_full_size_properties) uses it to
recompute sampled rows of a 1,048,576-node run that no whole-table oracle can hold.  Here it
must reproduce the oracle's own next-tick rows, from the previous tick's views and the
message list, on a small population.
"""
import numpy as np

from tests.oracle_binding import PviewCfg, PviewOracle, pview_row_step


def test_row_step_equals_oracle_step():
    kw = dict(view=48, fanout=4, inbox=3, drop_pct=10, fail_mode=1, fail_tick=4,
              fail_ppm=50000, seed=21)
    n = 600
    orc = PviewOracle(n, **kw)
    cfg = PviewCfg(n, kw["view"], kw["fanout"], kw["inbox"], kw["drop_pct"], 20, 1,
                   kw["fail_mode"], kw["fail_tick"], kw["fail_ppm"], kw["seed"])
    checked = overflowed = 0
    for t in range(1, 9):
        views = {r: orc.row(r) for r in range(n)}
        src, dst = orc.messages()
        d = orc.step()
        for r in range(0, n, 7):
            if orc.fail_tick(r) < t:
                continue
            snd = src[dst == r].tolist()
            got, dr = pview_row_step(cfg, t, r, views[r], snd, [views[s] for s in snd])
            want = orc.row(r)
            for a, b in zip(got, want):
                assert np.array_equal(a, b), (t, r)
            checked += 1
            overflowed += dr["overflow"] > 0
        assert d["node_rounds"] > 0
    assert checked > 500 and overflowed > 0


def test_rotated_eviction_keeps_the_rotated_id_prefix():
    """evict_order 1: among entries tied on (age, hb) the kept ones are those first in the
    rotated id order (x - m) mod n, m = Philox(EVICT; t, r) mod n -- here a row whose own view
    (V entries) and one sender's view (V more, all fresh, same hb) tie everywhere, so exactly
    the V smallest rotated ids survive; with evict_order 0 the V smallest ids."""
    from tests.oracle_binding import Policy, load_oracle
    n, V, t, r, seed = 5000, 32, 7, 1234, 99
    rng = np.random.default_rng(3)
    ids = np.sort(rng.choice(np.arange(n)[np.arange(n) != r], 2 * V, replace=False))
    own_ids, snd_ids = np.sort(ids[::2]), np.sort(ids[1::2])
    sender = int(snd_ids[0])
    snd_view_ids = np.sort(np.concatenate([snd_ids[1:], [own_ids[0]]]))   # the sender skips itself
    hb = lambda a: np.full(len(a), 5, np.int32)
    ts = lambda a: np.full(len(a), t - 1, np.int32)
    for order in (0, 1):
        cfg = PviewCfg(n, V, 3, 7, 0, 20, 1, 0, 10, 0, seed, 0, 0, Policy(), order)
        (gi, gh, gt), d = pview_row_step(cfg, t, r, (own_ids, hb(own_ids), ts(own_ids)), [sender],
                                         [(snd_view_ids, hb(snd_view_ids), ts(snd_view_ids))])
        assert len(gi) == V and np.all(np.diff(gi) > 0)
        # the sender's own entry is (hb 1, ts t): age 0, alone in the best bin, always kept
        assert sender in gi
        tied = np.setdiff1d(np.union1d(own_ids, snd_view_ids), [sender])
        m = load_oracle().gsp_oracle_draw(0x45564354, seed, t, r, 0, 0) % n if order else 0
        want = np.sort(tied[np.argsort((tied - m) % n, kind="stable")[:V - 1]])
        assert np.array_equal(np.setdiff1d(gi, [sender]), want), order
        assert d["evicts"] == len(tied) - (V - 1)


def test_drain_all_is_an_unbounded_inbox():
    """inbox = 0 drains every message (MP1Node.cpp:200-212): with every in-degree below 200 the
    oracle at inbox 0 and at inbox 200 run the same protocol -- same digests (no overflow in
    either), same views -- while inbox 2 discards messages and diverges."""
    kw = dict(view=32, fanout=6, drop_pct=10, fail_mode=1, fail_tick=4, fail_ppm=30000, seed=5)
    n = 800
    a, b, c = (PviewOracle(n, inbox=k, **kw) for k in (0, 200, 2))
    over = 0
    for t in range(1, 13):
        src, dst = a.messages()
        assert np.bincount(dst, minlength=n).max() < 200
        da, db, dc = a.step(), b.step(), c.step()
        assert da == db and da["overflow"] == 0, t
        over += dc["overflow"]
    for r in range(0, n, 13):
        for x, y in zip(a.row(r), b.row(r)):
            assert np.array_equal(x, y)
    assert over > 0
    for o in (a, b, c):
        o.close()
