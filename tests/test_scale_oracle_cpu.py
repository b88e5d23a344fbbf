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
