"""The scale-protocol restatement on the CPU (oracle/scale_oracle.c): properties that hold
independently of the GPU, including the TFAIL suspicion variant.

TFAIL is defined by the reference (MP1Node.h:22, TFAIL 5) and never used; the variant is
build-defined, so these checks pin its semantics by invariants, not by reference output
("parity unpinned" for the variant itself, DESIGN.md "Scale mode").
"""
import numpy as np

from tests.oracle_binding import ScaleOracle

KW = dict(fanout=3, drop_pct=10, fail_mode=1, fail_tick=6, fail_ppm=40000, seed=21)


def _run(n, ticks, **kw):
    o = ScaleOracle(n, **kw)
    d = [o.step() for _ in range(ticks)]
    return o, d


def test_tfail_zero_is_the_reference_protocol():
    a, da = _run(96, 30, **KW)
    b, db = _run(96, 30, tfail=0, **KW)
    assert da == db
    a.close()
    b.close()


def test_tfail_invariants():
    n, ticks, tf, tr = 128, 40, 5, 20
    o, digests = _run(n, ticks, tfail=tf, tremove=tr, **KW)
    plain, pd = _run(n, ticks, **KW)
    assert digests != pd                      # suspicion is exercised at this size
    t = ticks
    src, dst = o.messages()                   # sent at tick t
    for s, d in zip(src.tolist(), dst.tolist()):
        pres, hb, ts = o.row(s)
        # a peer is a listed member the sender does not suspect
        assert pres[d] and t - ts[d] < tf
    for r in range(0, n, 5):
        if o.fail_tick(r) < t:                # a crashed row is frozen at its fail tick
            continue
        pres, hb, ts = o.row(r)
        listed = pres.astype(bool)
        assert not listed[r]
        # suspected members stay listed until TREMOVE
        assert np.all(t - ts[listed] < tr)
    o.close()
    plain.close()


# ---- SWIM ping/ack probing (mp1_specifications.pdf p.3; not in the reference).
# Build-defined like TFAIL: pinned by invariants here, GPU vs oracle in tests/test_scale_gpu.py.

def test_swim_answered_probes_change_only_timestamps():
    """No drops, no failures: every probe is answered, so nothing is removed and the digests
    equal the plain protocol's; a probe target's ts is refreshed to the resolving tick."""
    kw = dict(fanout=3, drop_pct=0, fail_mode=0, seed=5)
    o, d = _run(80, 30, swim=2, **kw)
    plain, pd = _run(80, 30, **kw)
    assert d == pd
    assert all(x["removes"] == 0 for x in d)
    fresher = 0
    for r in range(80):
        pres, hb, ts = o.row(r)
        pp, ph, pt = plain.row(r)
        assert np.array_equal(pres, pp) and np.array_equal(hb, ph)
        assert np.all(ts >= pt)                    # refreshes only move ts forward
        fresher += int(np.sum(ts != pt))
    assert fresher > 0
    o.close()
    plain.close()


def test_swim_unanswered_probes_remove_their_target():
    """drop_pct = 100: no path survives, so every alive node removes its probe target at the
    next tick -- n removals per tick until TREMOVE."""
    n, tr = 64, 20
    o, d = _run(n, tr - 1, swim=3, fanout=3, drop_pct=100, fail_mode=0, seed=9, tremove=tr)
    assert [x["removes"] for x in d] == [n] * (tr - 1)
    for r in range(n):
        assert int(o.row(r)[0].sum()) == n - 1 - (tr - 1)
    o.close()


def test_swim_detects_crashes_before_tremove():
    """Crashed members are removed by probes before the TREMOVE timeout could remove them;
    without probing the first removal comes TREMOVE ticks after the last heartbeat."""
    kw = dict(fanout=3, drop_pct=0, fail_mode=1, fail_tick=5, fail_ppm=100000, seed=3)
    o, d = _run(128, 20, swim=1, **kw)
    plain, pd = _run(128, 20, **kw)
    early = sum(x["removes"] for x in d[:15])
    assert early > 0 and sum(x["removes"] for x in pd[:15]) == 0
    dead = {r for r in range(128) if o.fail_tick(r) < 20}
    assert dead
    detected = 0
    for r in range(128):
        if r in dead:
            continue
        pres = o.row(r)[0]
        detected += sum(1 for x in dead if not pres[x])
        live_gone = [x for x in range(128) if x not in dead and x != r and not pres[x]]
        assert not live_gone                        # no drops: a live member is never removed
    assert detected > 0                             # probes removed crashed members by tick 20
    o.close()
    plain.close()


def test_threaded_oracle_equals_single_threaded():
    """The oracle's step and send phase run over row blocks on OpenMP threads, concatenated in
    row order: every digest, message list, event list and row equals the one-thread run."""
    from tests.oracle_binding import load_oracle, make_policy
    L = load_oracle()
    kw = dict(fanout=3, drop_pct=10, fail_mode=1, fail_tick=6, fail_ppm=40000, seed=21, tremove=8,
              swim=2, tfail=4, policy=make_policy(step_rate=0.05, intro_list=3, drop_window=(2, 9)))
    runs = []
    try:
        for threads in (1, 5):
            L.gsp_oracle_set_threads(threads)
            o = ScaleOracle(203, **kw)
            trace = []
            for _ in range(18):
                d = o.step()
                src, dst = o.messages()
                k, r, x = o.events()
                trace.append((d, src.tolist(), dst.tolist(), k.tolist(), r.tolist(), x.tolist(),
                              o.joinreps().tolist()))
            rows = [tuple(a.tolist() for a in o.row(r)) for r in range(203)]
            runs.append((trace, rows))
            o.close()
    finally:
        L.gsp_oracle_set_threads(0)
    assert runs[0] == runs[1]
    assert sum(len(t[3]) for t in runs[0][0]) > 0
