"""EXACT mode on the GPU: bit-exact against the reference (configs 1-2).

Runs the reference Application's schedule through the C ABI (the HIP kernels do every
merge / ops / send list / draw) and compares dbg.log, msgcount.log, the end-of-tick state
of every node and the driver's stdout lines with the golden outputs of the reference
itself (tests/golden/ref): 3 testcases x 5 seeds x {glibc rand() stream, Philox replay}.
"""
import pytest

from gossip_protocol_amd import exact
from tests.oracle_binding import CONFS, FILES, MODES, SEEDS, conf_path, golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("conf", CONFS)
@pytest.mark.parametrize("seed", SEEDS)
def test_exact_bitexact_vs_reference(tmp_path, mode, conf, seed):
    out = exact.run_application(conf_path(conf), seed, mode, str(tmp_path))
    for name in FILES:
        with open(out[name], "rb") as f:
            got = f.read()
        want = golden(mode, conf, seed, name)
        if got != want:
            gl, wl = got.decode().splitlines(), want.decode().splitlines()
            first = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b),
                         min(len(gl), len(wl)))
            pytest.fail("%s differs at line %d:\n got: %s\nwant: %s" % (
                name, first, gl[first] if first < len(gl) else "<eof>",
                wl[first] if first < len(wl) else "<eof>"))
    st = out["stats"]
    assert st.batches == 700 and st.node_rounds > 0 and st.device_ms > 0


def test_conf_drop_window_is_the_exact_drivers(tmp_path, monkeypatch):
    """The drop window the scale engines map a reference .conf's DROP_MSG to
    (gsp_scale_params_from_conf) is exactly the set of ticks whose sends the byte-exact driver
    runs with dropmsg = 1 (Application.cpp:177, 198: set / cleared at the END of t = 50 / 300)."""
    from gossip_protocol_amd.scale import params_from_conf as scale_conf
    seen = {}
    orig = exact.Engine.process

    def record(self, tick, order, ops, dropmsg):
        seen[tick] = dropmsg
        return orig(self, tick, order, ops, dropmsg)
    monkeypatch.setattr(exact.Engine, "process", record)
    exact.run_application(conf_path("msgdropsinglefailure"), 5, "glibc", str(tmp_path))
    p = scale_conf(conf_path("msgdropsinglefailure"))
    assert sorted(t for t, d in seen.items() if d) == \
        list(range(p.policy.drop_from, p.policy.drop_until))


def test_exact_stale_payload_is_rejected():
    """A GOSSIP whose sender re-ran before delivery cannot be replayed: loud error."""
    p = exact.params_from_conf(conf_path("singlefailure"))
    with exact.Engine(p, 0, "glibc", 1) as e:
        e.process(0, [3, 2, 1, 0], [0, 0, 0, 0], 0)
        e.recv(1, [0, 1, 2, 3])
        e.process(1, [0], [exact.OP_LOOP], 0)           # introducer replies, gossips
        e.process(1, [0], [exact.OP_OPS], 0)            # ...and re-runs ops (new snapshot)
        e.recv(2, [1])
        with pytest.raises(Exception, match="stale payload"):
            e.process(2, [1], [exact.OP_LOOP], 0)


from tests.oracle_binding import BIG_FILES, BIG_RUNS, golden_big, outputs_for_big  # noqa: E402


@pytest.mark.parametrize("conf,seed,mode", BIG_RUNS, ids=lambda x: str(x))
def test_exact_bitexact_vs_reference_big(tmp_path, conf, seed, mode):
    """Past the reference's N = 10 testcases: MAX_NNB 70 / 300 / 600 against the reference's
    own outputs (tests/golden/ref_big).  Covers msgcount.log's node-67 layout
    (EmulNet.cpp:204-211), negative address bytes of ids >= 128 (Log.cpp:73), strcmp()
    delivery aliasing of ids 256 / 512 (EmulNet.cpp:154), the full 30,000-message buffer
    (EmulNet.cpp:92) and the id < 10 payload filter at N > 10 (MP1Node.cpp:245)."""
    got = outputs_for_big(exact.run_application(conf_path(conf), seed, mode, str(tmp_path)))
    for name in BIG_FILES:
        want = golden_big(mode, conf, seed, name)
        if got[name] != want:
            gl, wl = got[name].decode().splitlines(), want.decode().splitlines()
            first = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b),
                         min(len(gl), len(wl)))
            pytest.fail("%s differs at line %d:\n got: %s\nwant: %s" % (
                name, first, gl[first][:300] if first < len(gl) else "<eof>",
                wl[first][:300] if first < len(wl) else "<eof>"))


@pytest.mark.parametrize("conf", CONFS)
def test_exact_merge_count_matches_oracle(tmp_path, conf):
    """gsp_exact_stats.merges (1 + |payload| per GOSSIP handled, counted on the device) equals
    the restatement's count -- the figure bench.py's reference CPU baseline reports per second."""
    from tests.oracle_binding import load_oracle, run_oracle_mp1
    got = exact.run_application(conf_path(conf), 1, "glibc", str(tmp_path / "gpu"))["stats"].merges
    run_oracle_mp1(conf, 1, "glibc", str(tmp_path / "cpu"))
    assert got == load_oracle().gsp_oracle_mp1_merges() > 0
