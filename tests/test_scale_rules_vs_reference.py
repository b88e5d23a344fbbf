"""Bridge: the scale protocol's per-row rules ARE the reference's (CPU only).

The scale engines (full view and partial view) implement MP1Node::recvCallBack's GOSSIP merge
and nodeLoopOps' TREMOVE scan per member entry (oracle/scale_oracle.c restates them; the GPU
is bit-exact against that restatement).  This test pins that restatement to the REFERENCE on
identical inputs: for every golden run the reference produced (tests/golden/ref: 3 testcases
x 5 seeds x {glibc, philox}, 700 ticks, 10 nodes) and every node-round, it takes

  * the receiver's row of tick t - 1 and every GOSSIP sender's row as it sent it, from the
    reference's own end-of-tick state dump (state.txt),
  * the order the receiver handled its messages in -- the EmulNet delivery permutation,
    from the pinned mp1 restatement (gsp_oracle_mp1_set_queue_trace; it reproduces every
    golden file byte for byte, tests/test_oracle_golden.py),

feeds each GOSSIP to scale_oracle.c's exported merge (gsp_scale_oracle_merge_msg) and the
TREMOVE scan (gsp_scale_oracle_remove_scan) when the node ran nodeLoopOps, and asserts the
result equals the reference's row of tick t (as a set of (id, hb, ts): list ORDER is the one
thing the scale layout does not keep).  The reference-only parts stay on this side: JOINREQ /
JOINREP add the sender (MP1Node.cpp:221-233) and payloads are cut to ids < 10
(MP1Node.cpp:245), the hard-coded filter the scale protocol drops.
"""
import ctypes
import os

import numpy as np
import pytest

from tests.oracle_binding import CONFS, MODES, SEEDS, golden, load_oracle, run_oracle_mp1

T_REMOVE = 20
JOINREQ, JOINREP, GOSSIP = 0, 1, 3


def _state(mode, conf, seed):
    """{(t, id): (inGroup, bFailed, {x: (hb, ts)})} from the reference's state dump."""
    st = {}
    for line in golden(mode, conf, seed, "state.txt").decode().splitlines():
        f = line.split()
        t, i, in_group, failed = int(f[0]), int(f[1]), int(f[3]), int(f[4])
        lst = {}
        for e in f[7:]:
            x, hb, ts = (int(v) for v in e.split(":"))
            lst[x] = (hb, ts)
        st[(t, i)] = (in_group, failed, lst)
    return st


def _row(lst, n, keep=lambda x: True):
    P = np.zeros(n, np.uint8)
    H = np.zeros(n, np.int32)
    S = np.zeros(n, np.int32)
    for x, (hb, ts) in lst.items():
        if keep(x):
            P[x - 1], H[x - 1], S[x - 1] = 1, hb, ts
    return P, H, S


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("conf", CONFS)
@pytest.mark.parametrize("seed", SEEDS)
def test_scale_rules_reproduce_reference_rows(tmp_path, mode, conf, seed):
    L = load_oracle()
    L.gsp_scale_oracle_merge_msg.argtypes = [ctypes.c_int32] * 5 + [ctypes.c_void_p] * 3 + [
        ctypes.c_int32] + [ctypes.c_void_p] * 5
    L.gsp_scale_oracle_remove_scan.argtypes = [ctypes.c_int32] * 5 + [ctypes.c_void_p] * 5
    L.gsp_scale_oracle_remove_scan.restype = ctypes.c_int32
    trace = os.path.join(str(tmp_path), "queue.txt")
    L.gsp_oracle_mp1_set_queue_trace(trace.encode())
    try:
        run_oracle_mp1(conf, seed, mode, str(tmp_path))
    finally:
        L.gsp_oracle_mp1_set_queue_trace(None)
    queues = {}
    for line in open(trace):
        t, r, src, typ, st = (int(v) for v in line.split())
        queues.setdefault((t, r), []).append((src, typ, st))
    state = _state(mode, conf, seed)
    n = 10
    joins, removes, h = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_uint64()
    rounds = gossips = 0
    for t in range(1, 700):
        for i in range(n):
            r = i + 1
            # nodeLoop ran: active (t > 0.25 i, Application.cpp:153), started before t, alive
            if not (t > 0.25 * i) or t == int(0.25 * i) or state[(t - 1, r)][1]:
                continue
            P, H, S = _row(state[(t - 1, r)][2], n)
            for src, typ, st in queues.get((t, r), []):
                assert st == t - 1                 # one-tick latency (EmulNet delivery)
                if typ in (JOINREQ, JOINREP):      # MP1Node.cpp:221-233 (reference-only)
                    if not P[src - 1]:
                        P[src - 1], H[src - 1], S[src - 1] = 1, 1, t
                    continue
                Ps, Hs, Ss = _row(state[(st, src)][2], n, keep=lambda x: 0 <= x < 10)
                L.gsp_scale_oracle_merge_msg(n, t, T_REMOVE, 0, i, P.ctypes.data, H.ctypes.data,
                                             S.ctypes.data, src - 1, Ps.ctypes.data,
                                             Hs.ctypes.data, Ss.ctypes.data, ctypes.byref(joins),
                                             ctypes.byref(h))
                gossips += 1
            in_group, _, want = state[(t, r)]
            if in_group:                           # nodeLoopOps (MP1Node.cpp:185-190)
                L.gsp_scale_oracle_remove_scan(n, t, T_REMOVE, 0, i, P.ctypes.data, H.ctypes.data,
                                               S.ctypes.data, ctypes.byref(removes),
                                               ctypes.byref(h))
            got = {x + 1: (int(H[x]), int(S[x])) for x in range(n) if P[x]}
            assert got == want, "tick %d node %d" % (t, r)
            rounds += 1
    assert rounds > 3000 and gossips > 15000 and removes.value > 0
