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
