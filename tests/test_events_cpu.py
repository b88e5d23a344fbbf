"""gsp_events_write_log against the reference's own dbg.log (host code; no GPU).

Every "Node <x> joined / removed at time <t>" line of the reference's dbg.log (Log.cpp:116-130,
written from MP1Node.cpp:276 / 297 / 343) is turned into an event record (kind, t, r, x) and
written back by the library's writer: the output must be the reference's lines exactly, in
the writer's canonical order -- t ascending, then the logging node descending, which is
already the reference's order (phase P runs nodes n-1 .. 0, Application.cpp:138) -- and
within one node and tick joins, removes, member ascending.  Runs over the N = 10 fixtures and
the N = 70 / 300 / 600 ones (negative address bytes of ids >= 128, Log.cpp:73).
"""
import gzip
import os
import re

import numpy as np
import pytest

from gossip_protocol_amd import _lib
from tests.oracle_binding import BIG_CONFS, CONFS, GOLDEN, GOLDEN_BIG

LINE = re.compile(r"^ (\S+) \[(\d+)\] Node (\S+) (joined|removed) at time (\d+)$")
KIND = {"joined": _lib.EVENT_JOIN, "removed": _lib.EVENT_REMOVE}


def _index(addr):
    """Log.cpp:73's "%d.%d.%d.%d:%d" of the signed id bytes -> node index (id - 1)."""
    b = [int(v) & 0xFF for v in addr.split(":")[0].split(".")]
    return (b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24) - 1


def _event_lines(text):
    out = []
    for ln in text.split("\n"):
        m = LINE.match(ln)
        if m:
            assert m.group(2) == m.group(5)
            out.append((ln, KIND[m.group(4)], int(m.group(2)), _index(m.group(1)), _index(m.group(3))))
    return out


def _fixture(path):
    with gzip.open(path, "rb") as f:
        return f.read().decode()


CASES = [os.path.join(GOLDEN, "glibc", c, "1", "dbg.log.gz") for c in CONFS] + \
    [os.path.join(GOLDEN_BIG, "philox", c, "3", "dbg.log.gz") for c in BIG_CONFS]


@pytest.mark.parametrize("path", CASES, ids=lambda p: "/".join(p.split(os.sep)[-4:-1]))
def test_event_log_writer_matches_reference_lines(tmp_path, path):
    ref = _event_lines(_fixture(path))
    assert len(ref) > 20
    # the reference's own order is (t ascending, logging node descending)
    keys = [(t, -r) for _, _, t, r, _ in ref]
    assert keys == sorted(keys)
    rec = np.array([(k << 62) | (t << 42) | (r << 21) | x for _, k, t, r, x in ref], np.uint64)
    rng = np.random.default_rng(0)
    rng.shuffle(rec)                                   # the writer sorts
    out = tmp_path / "dbg.log"
    _lib.write_event_log(rec, str(out))
    got = out.read_text()
    assert got.startswith("131\n")
    want = sorted(ref, key=lambda e: (e[2], -e[3], e[1], e[4]))
    assert got[4:].split("\n")[1:] == [e[0] for e in want]
    # a second call appends without a second header
    _lib.write_event_log(rec[:3], str(out))
    assert out.read_text().split("\n").count("131") == 1
