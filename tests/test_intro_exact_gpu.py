"""The exact engine's opt-in bounded introducer list (gsp_params.intro_list) on the GPU:
byte-identical to oracle/mp1_oracle.c's restatement of the variant (dbg.log, msgcount.log,
end-of-tick state, stdout) on the reference testcases and two of the N > 10 ones, both RNG
modes.  intro_list = 0 is covered by test_exact_gpu.py (the reference's own outputs)."""
import pytest

from gossip_protocol_amd import exact
from tests.oracle_binding import CONFS, FILES, MODES, conf_path, run_oracle_mp1

pytestmark = pytest.mark.gpu

CASES = [(c, m, b) for c in CONFS for m in MODES for b in (2, 5)] + \
    [(c, m, 4) for c in ("n70_single", "n300_drop") for m in MODES]


@pytest.mark.parametrize("conf,mode,b", CASES, ids=lambda x: str(x))
def test_intro_list_matches_oracle(tmp_path, conf, mode, b):
    want = run_oracle_mp1(conf, 9, mode, str(tmp_path / "oracle"), intro_list=b)
    got = exact.run_application(conf_path(conf), 9, mode, str(tmp_path / "gpu"), intro_list=b)
    for name in FILES:
        with open(got[name], "rb") as f:
            g = f.read()
        with open(want[name], "rb") as f:
            w = f.read()
        if g != w:
            gl, wl = g.decode().splitlines(), w.decode().splitlines()
            first = next((i for i, (a, c) in enumerate(zip(gl, wl)) if a != c), min(len(gl), len(wl)))
            pytest.fail("%s differs at line %d:\n got: %s\nwant: %s" % (
                name, first, gl[first][:300] if first < len(gl) else "<eof>",
                wl[first][:300] if first < len(wl) else "<eof>"))
