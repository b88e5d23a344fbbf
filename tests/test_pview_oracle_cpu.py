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
