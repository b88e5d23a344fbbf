"""Bridge: the PARTIAL VIEW's per-entry rules ARE the reference's (CPU only).

oracle/pview_oracle.c folds every member id of a receiver's view over its messages with one
rule function (pv_rule: the sender entry, the payload max-merge and the fresh-copy insert of
MP1Node.cpp:234-301) and removes with one predicate (pv_expired: MP1Node.cpp:339-348); the
GPU's partial-view kernels are bit-exact against that restatement (tests/test_pview_gpu.py).
This test pins those two functions to the REFERENCE on identical inputs, the way
tests/test_scale_rules_vs_reference.py pins the full view's: for every golden run the
reference produced (tests/golden/ref: 3 testcases x 5 seeds x {glibc, philox}, 700 ticks, 10
nodes) and every node-round it takes

  * the receiver's view of tick t - 1 and each GOSSIP sender's view as it sent it, from the
    reference's own end-of-tick state dump (state.txt), ids ascending (V = 16 >= 10: no
    eviction, and every message is merged: no inbox bound);
  * the order the receiver handled its messages in (the EmulNet delivery permutation, from
    the pinned mp1 restatement's queue trace),

feeds each GOSSIP to gsp_pview_oracle_merge_msg and, when the node ran nodeLoopOps,
gsp_pview_oracle_remove_scan, and asserts the view equals the reference's list of tick t as a
set of (id, hb, ts).  Reference-only parts stay on this side: JOINREQ / JOINREP add their
sender as (1, t) when absent (MP1Node.cpp:221-233, 265-280), payloads are cut to ids < 10
(MP1Node.cpp:245).  The bounded-view choices (eviction order, inbox bound, initial views)
have no reference counterpart: they stay "parity unpinned" (DESIGN.md 4b).
"""
import ctypes
import os

import numpy as np
import pytest

from tests.oracle_binding import CONFS, MODES, SEEDS, load_oracle, run_oracle_mp1
from tests.test_scale_rules_vs_reference import _state

T_REMOVE = 20
V = 16
JOINREQ, JOINREP, GOSSIP = 0, 1, 3


def _view(lst, keep=lambda x: True):
    ids = sorted(x for x in lst if keep(x))
    a = np.zeros((3, V), np.int32)
    for i, x in enumerate(ids):
        a[0, i], a[1, i], a[2, i] = x, lst[x][0], lst[x][1]
    return a, len(ids)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("conf", CONFS)
@pytest.mark.parametrize("seed", SEEDS)
def test_pview_rules_reproduce_reference_rows(tmp_path, mode, conf, seed):
    L = load_oracle()
    L.gsp_pview_oracle_merge_msg.argtypes = [ctypes.c_int32] * 3 + [ctypes.c_void_p] * 3 + [
        ctypes.c_int32] * 3 + [ctypes.c_void_p] * 3 + [ctypes.c_int32, ctypes.c_void_p]
    L.gsp_pview_oracle_merge_msg.restype = ctypes.c_int32
    L.gsp_pview_oracle_remove_scan.argtypes = [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 3 + [
        ctypes.c_int32, ctypes.c_void_p]
    L.gsp_pview_oracle_remove_scan.restype = ctypes.c_int32
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
    joins, removes = ctypes.c_int64(), ctypes.c_int64()
    rounds = gossips = 0
    for t in range(1, 700):
        for i in range(n):
            r = i + 1
            # nodeLoop ran: active (t > 0.25 i, Application.cpp:153), started before t, alive
            if not (t > 0.25 * i) or t == int(0.25 * i) or state[(t - 1, r)][1]:
                continue
            view, m = _view(state[(t - 1, r)][2])
            for src, typ, st in queues.get((t, r), []):
                assert st == t - 1                 # one-tick latency (EmulNet delivery)
                if typ in (JOINREQ, JOINREP):      # MP1Node.cpp:221-233 (reference-only)
                    if src not in view[0, :m]:
                        cur = {int(view[0, k]): (int(view[1, k]), int(view[2, k])) for k in range(m)}
                        cur[src] = (1, t)
                        view, m = _view(cur)
                    continue
                pay, pm = _view(state[(st, src)][2], keep=lambda x: 0 <= x < 10)
                m = L.gsp_pview_oracle_merge_msg(t, T_REMOVE, r, view[0].ctypes.data,
                                                 view[1].ctypes.data, view[2].ctypes.data, m, V,
                                                 src, pay[0].ctypes.data, pay[1].ctypes.data,
                                                 pay[2].ctypes.data, pm, ctypes.byref(joins))
                assert m >= 0
                gossips += 1
            in_group, _, want = state[(t, r)]
            if in_group:                           # nodeLoopOps (MP1Node.cpp:185-190)
                m = L.gsp_pview_oracle_remove_scan(t, T_REMOVE, view[0].ctypes.data,
                                                   view[1].ctypes.data, view[2].ctypes.data, m,
                                                   ctypes.byref(removes))
            assert list(view[0, :m]) == sorted(view[0, :m])     # the view stays in id order
            got = {int(view[0, k]): (int(view[1, k]), int(view[2, k])) for k in range(m)}
            assert got == want, "tick %d node %d" % (t, r)
            rounds += 1
    assert rounds > 3000 and gossips > 15000 and removes.value > 0 and joins.value > 0
