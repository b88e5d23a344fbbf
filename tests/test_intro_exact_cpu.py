"""The exact engine's opt-in bounded introducer list (gsp_params.intro_list) in the oracle.

The reference's JOINREP carries the introducer's whole list and its receiver ignores it
(MP1Node.cpp:221-233); with intro_list = B the joiner merges B Philox-chosen entries of it
with the GOSSIP payload rules (MP1Node.cpp:244-258).  Variant semantics are build-defined:
*parity unpinned* against the reference, which has no such behaviour; B = 0 must stay the
reference byte for byte (the golden fixtures), and the GPU engine must equal this oracle
(tests/test_intro_exact_gpu.py).
"""
import pytest

from tests import grader
from tests.oracle_binding import CONFS, golden, run_oracle_mp1


def _read(p):
    with open(p, "rb") as f:
        return f.read()


@pytest.mark.parametrize("conf", CONFS)
def test_intro_list_zero_is_the_reference(tmp_path, conf):
    out = run_oracle_mp1(conf, 5, "philox", str(tmp_path), intro_list=0)
    for name in ("dbg.log", "state.txt"):
        assert _read(out[name]) == golden("philox", conf, 5, name)


@pytest.mark.parametrize("conf", CONFS)
@pytest.mark.parametrize("b", [2, 4])
def test_intro_list_changes_the_run(tmp_path, conf, b):
    """At N = 10 the joiner's first GOSSIP from the introducer carries the same list, so the
    variant mostly reorders: joins logged from the JOINREP (queue position of the JOINREP)
    instead of the GOSSIP, hence other list orders, send orders and draws.  The run must
    differ from the reference, be deterministic, and score as the reference does."""
    ref = run_oracle_mp1(conf, 9, "philox", str(tmp_path / "ref"))
    var = run_oracle_mp1(conf, 9, "philox", str(tmp_path / "var"), intro_list=b)
    again = run_oracle_mp1(conf, 9, "philox", str(tmp_path / "again"), intro_list=b)
    assert _read(ref["dbg.log"]) != _read(var["dbg.log"])
    assert _read(ref["state.txt"]) != _read(var["state.txt"])
    for name in ("dbg.log", "state.txt", "msgcount.log"):
        assert _read(var[name]) == _read(again[name])
    assert grader.score(_read(var["dbg.log"]), conf) == grader.score(_read(ref["dbg.log"]), conf)
