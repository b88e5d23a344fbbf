"""Pin the CPU oracle before trusting it (CPU only).

* the oracle restatement (oracle/mp1_oracle.c) reproduces, byte for byte, every golden
  output the REFERENCE produced (tests/golden/ref, made by tests/golden/make_golden.py
  from oracle/_ref = /root/reference compiled unmodified): 3 testcases x 5 seeds x
  {glibc, philox} x {dbg.log, msgcount.log, state.txt, stdout.txt};
* the reference's own committed dbg.log (singlefailure, node 5 failed) is the seed-10
  glibc run;
* the glibc stream restatement matches the real libc rand();
* Philox4x32-10 matches the Random123 known-answer vectors;
* Grader.sh's checks (Grader.sh:29-190) hold on every golden run.
"""
import ctypes
import os
import re

import pytest

from tests import grader
from tests.oracle_binding import (CONFS, FILES, GOLDEN, MODES, SEEDS, golden, load_oracle,
                                  run_oracle_mp1)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("conf", CONFS)
@pytest.mark.parametrize("seed", SEEDS)
def test_oracle_matches_reference_fixtures(tmp_path, mode, conf, seed):
    out = run_oracle_mp1(conf, seed, mode, str(tmp_path))
    for name in FILES:
        with open(out[name], "rb") as f:
            got = f.read()
        assert got == golden(mode, conf, seed, name), "%s %s %s %s" % (mode, conf, seed, name)


def test_reference_committed_dbg_log_is_seed10():
    with open(os.path.join(GOLDEN, "reference_committed_dbg.log"), "rb") as f:
        committed = f.read()
    assert committed == golden("glibc", "singlefailure", 10, "dbg.log")


def test_glibc_stream_matches_libc_rand():
    L = load_oracle()
    libc = ctypes.CDLL("libc.so.6")
    for seed in [0, 1, 10, 1234567, 1760572800, 0x7FFFFFFF, 0xFFFFFFFF]:
        n = 2000
        buf = (ctypes.c_int32 * n)()
        L.gsp_glibc_stream(seed & 0xFFFFFFFF, buf, n)
        libc.srand(ctypes.c_uint(seed & 0xFFFFFFFF))
        want = [libc.rand() for _ in range(n)]
        assert list(buf) == want, seed


KAT = [  # Random123 kat_vectors, philox4x32 R=10: ctr[4] key[2] -> out[4]
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_oracle_philox_known_answers(ctr, key, want):
    L = load_oracle()
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    L.gsp_oracle_philox(c, k, o)
    assert tuple(o) == want


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", SEEDS)
def test_grader_checks_hold_on_golden(mode, seed):
    for conf in CONFS:
        assert grader.score(golden(mode, conf, seed, "dbg.log"), conf) == 30, (mode, conf, seed)


def test_golden_state_shape():
    st = golden("glibc", "singlefailure", 10, "state.txt").decode().splitlines()
    assert len(st) == 700 * 10
    assert re.match(r"^0 1 1 1 0 0 0$", st[0])


# ---- past N = 10: the reference's own outputs at MAX_NNB 70 / 300 / 600 -------------------
from tests.oracle_binding import (BIG_FILES, BIG_RUNS, golden_big, outputs_for_big)  # noqa: E402


@pytest.mark.parametrize("conf,seed,mode", BIG_RUNS, ids=lambda x: str(x))
def test_oracle_matches_reference_big(tmp_path, conf, seed, mode):
    """The C restatement reproduces the reference at N = 70 / 300 / 600: dbg.log,
    msgcount.log, stdout byte for byte and the end-of-tick state of every node at every tick
    (per-tick SHA-256, full lines at selected ticks)."""
    got = outputs_for_big(run_oracle_mp1(conf, seed, mode, str(tmp_path)))
    for name in BIG_FILES:
        assert got[name] == golden_big(mode, conf, seed, name), "%s %s %s %s" % (
            conf, seed, mode, name)


def test_big_fixtures_reach_the_reference_quirks(tmp_path):
    """The large-N fixtures exercise what N = 10 never does (each a reference behaviour the
    parity tests would otherwise leave unpinned)."""
    # msgcount.log's node-67 layout (EmulNet.cpp:204-211)
    mc = golden_big("glibc", "n70_multi", 3, "msgcount.log").decode()
    assert "node  67 special    0" in mc and "node  67 sent_total" in mc
    # signed-char address bytes of ids >= 128 (Log.cpp:73): id 128 prints as -128.0.0.0
    assert b" -128.0.0.0:0 [0] APP" in golden_big("glibc", "n300_single", 3, "dbg.log")
    # strcmp() address aliasing (EmulNet.cpp:154): ids 256, 512 (first byte 0) share one
    # class, so node 256 -- which receives first (ascending order) -- also takes the messages
    # sent to 512; node 512 receives nothing in a whole run although it is sent to
    lines = golden_big("glibc", "n600_single", 3, "msgcount.log").decode().splitlines()
    tot = {int(l.split()[1]): (int(l.split()[3]), int(l.split()[5]))
           for l in lines if "sent_total" in l}
    assert tot[512][1] == 0 and tot[256][1] > tot[255][1]
    # the 30,000-message EmulNet buffer fills (EmulNet.cpp:92): messages to the multi-failure
    # victims linger; the oracle counts the sends it rejected for that reason
    L = load_oracle()
    run_oracle_mp1("n600_multidrop", 3, "glibc", str(tmp_path))
    assert L.gsp_oracle_mp1_buffer_full_rejects() > 0
    run_oracle_mp1("n70_multi", 3, "glibc", str(tmp_path))
    assert L.gsp_oracle_mp1_buffer_full_rejects() == 0
    # the id < 10 payload filter (MP1Node.cpp:245) at N > 10: only ids 1..9 spread
    # indirectly, so far fewer join lines than the N (N - 1) of a full view
    joins = golden_big("glibc", "n300_single", 3, "dbg.log").count(b"joined")
    assert joins < 300 * 299 // 4
