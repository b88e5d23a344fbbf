"""The receive-side entry points: EmulNet::ENrecv with a driver callback and direct
MP1Node::recvCallBack calls (EmulNet.cpp:144-177, MP1Node.cpp:44-56, 200-260).

tests/drivers/recv_driver.cpp runs the reference Application's schedule with the receive side
driven four ways (wrapper = recvLoop; observe = own callback into mp1q; direct = own callback
into a driver list, then recvCallBack per message; filter = drop / rewrite / reorder before
checkMessages; inject = GOSSIPs the driver builds and sends with EmulNet::ENsend, with their
own vector_list).  The one source is built against the reference's own classes
(oracle/_ref/RecvDriver, compiled from /root/reference's sources) and against the facade over
the GPU engine (gossip_protocol_amd/bin/RecvDriver); stdout (with a checksum of every payload
the callbacks saw), dbg.log and msgcount.log must agree byte for byte.

The CPU tests pin the driver: its reference build reproduces the reference's golden outputs in
the three modes that do not change the protocol.  The GPU engine tests cover the C ABI calls
directly (sizes-only queries, capacity and payload validation, one-message processing).
"""
import os
import shutil
import subprocess

import pytest

from tests.oracle_binding import CONFS, conf_path, golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "RecvDriver")
GPU_DRIVER = os.path.join(ROOT, "gossip_protocol_amd", "bin", "RecvDriver")
OUTPUTS = ("stdout", "dbg.log", "msgcount.log")


def _run(binary, where, conf, mode, seed):
    os.makedirs(where, exist_ok=True)
    shutil.copy(conf_path(conf), where)
    env = dict(os.environ, GSP_SEED=str(seed), GSP_RNG="glibc")
    r = subprocess.run([binary, os.path.basename(conf_path(conf)), mode], cwd=where, env=env,
                       capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    out = {"stdout": r.stdout}
    for name in OUTPUTS[1:]:
        with open(os.path.join(where, name), "rb") as f:
            out[name] = f.read()
    return out


def _need(path):
    if not os.path.exists(path):
        pytest.skip("%s not built (make app; make -C oracle with /root/reference present)" % path)


@pytest.mark.parametrize("mode", ["wrapper", "observe", "direct", "switch"])
@pytest.mark.parametrize("conf", CONFS)
def test_reference_driver_reproduces_the_golden_outputs(tmp_path, conf, mode):
    """The driver is a faithful Application: on the reference's own classes, the receive
    paths that keep the protocol unchanged give the reference Application's outputs."""
    _need(REF_DRIVER)
    out = _run(REF_DRIVER, str(tmp_path), conf, mode, 1)
    assert out["stdout"].rsplit(b"recv_driver:", 1)[0] == golden("glibc", conf, 1, "stdout.txt")
    for name in OUTPUTS[1:]:
        assert out[name] == golden("glibc", conf, 1, name), name


CASES = [(c, m, 1) for c in CONFS for m in ("wrapper", "observe", "direct", "filter", "inject",
                                            "inject_direct", "switch", "members")] + \
        [(c, m, 10) for c in CONFS for m in ("direct", "filter", "switch", "members")]


@pytest.mark.gpu
@pytest.mark.parametrize("conf,mode,seed", CASES, ids=lambda x: str(x))
def test_facade_receive_paths_match_the_reference(tmp_path, conf, mode, seed):
    _need(REF_DRIVER)
    _need(GPU_DRIVER)
    want = _run(REF_DRIVER, str(tmp_path / "ref"), conf, mode, seed)
    got = _run(GPU_DRIVER, str(tmp_path / "gpu"), conf, mode, seed)
    if mode not in ("wrapper", "inject", "members"):      # the callback modes see messages
        assert b"messages=0 " not in want["stdout"]
    for name in OUTPUTS:
        if got[name] != want[name]:
            gl, wl = got[name].decode().splitlines(), want[name].decode().splitlines()
            first = next((i for i, (a, b) in enumerate(zip(gl, wl)) if a != b),
                         min(len(gl), len(wl)))
            pytest.fail("%s differs at line %d:\n got: %s\nwant: %s" % (
                name, first, gl[first] if first < len(gl) else "<eof>",
                wl[first] if first < len(wl) else "<eof>"))


def _joined_engine():
    """Nodes 0..3 started at tick 0 (the introducer and three JOINREQs in the buffer)."""
    from gossip_protocol_amd import exact
    p = exact.params_from_conf(conf_path("singlefailure"))
    e = exact.Engine(p, 0, "glibc", 1)
    e.process(0, [3, 2, 1, 0], [exact.OP_START] * 4, 0)
    return e


@pytest.mark.gpu
def test_detach_sizes_take_nothing_and_detach_counts_receipts():
    from gossip_protocol_amd import exact
    with _joined_engine() as e:
        assert e.detach_sizes(1, 0) == (3, 0)          # three JOINREQs, empty joiner lists
        assert e.detach_sizes(1, 0) == (3, 0)
        msgs = e.detach(1, 0)
        # delivery order of the reference's top-down scan (EmulNet.cpp:151): last sent first
        assert [(m[0], m[1]) for m in msgs] == [(2, 0), (3, 0), (4, 0)]
        assert e.detach_sizes(1, 0) == (0, 0)
        _, recv = e.counters(2)
        assert recv[1 * 2 + 1] == 3                     # id 1 received 3 at tick 1
        for src, typ, batch, pl in reversed(msgs):      # hand them back, in reverse
            assert e.queue_push(0, src, typ, pl) == 0
        e.process(1, [0], [exact.OP_LOOP], 0)
        assert [x[0] for x in e.member_list(0)] == [4, 3, 2]


@pytest.mark.gpu
def test_payload_validation():
    with _joined_engine() as e:
        for bad in ([(2, 1, 0), (2, 1, 0)], [(0, 1, 0)], [(11, 1, 0)], [(2, 1, 0, 7)]):
            assert e.queue_push(0, 2, 3, bad) == -1, bad
        assert e.queue_push(0, 99, 3, []) == -1          # sender outside 1..N
        assert e.queue_push(0, 2, 2, []) == -1           # no such message type
        assert e.queue_push(0, 2, 3, [(3, 5, 0)]) == 0


@pytest.mark.gpu
def test_recv_callback_handles_one_message_and_keeps_the_queue():
    from gossip_protocol_amd import exact
    with _joined_engine() as e:
        e.recv(1, [0])                                   # three JOINREQs queued at node 0
        assert e.recv_callback(1, 0, 3, 0, []) == 0      # JOINREQ from id 3, handled now
        assert [x[0] for x in e.member_list(0)] == [3]
        assert e.detach_sizes(2, 1)[0] == 0              # JOINREP id 1 -> id 2 not sent...
        assert e.detach_sizes(2, 2)[0] == 1              # ...the reply went to id 3 only
        e.process(1, [0], [exact.OP_CHECK], 0)           # then the queue, untouched: 2, 3, 4
        assert [x[0] for x in e.member_list(0)] == [3, 2, 4]


@pytest.mark.gpu
def test_gossip_payload_from_the_driver_is_merged():
    """A GOSSIP whose vector_list the driver wrote: the rules of MP1Node.cpp:234-257 apply to
    that list (sender hb bump / add, payload entries with id < 10 merged or added)."""
    with _joined_engine() as e:
        assert e.recv_callback(5, 0, 2, 3, [(3, 7, 4), (4, 2, 5)]) == 0
        assert e.member_list(0) == [(2, 1, 5), (3, 7, 4), (4, 2, 5)]
        assert e.recv_callback(6, 0, 2, 3, [(3, 9, 1), (2, 40, 1)]) == 0
        # sender 2: bumped to 2, then its own payload entry (hb 40) is newer: hb 40 at t = 6
        assert e.member_list(0) == [(2, 40, 6), (3, 9, 6), (4, 2, 5)]


@pytest.mark.gpu
def test_snapshots_keep_send_time_lists():
    """With snapshots on, a GOSSIP whose sender has committed again since the send still merges
    the list it was sent with (the stale case test_exact_gpu rejects without them)."""
    from gossip_protocol_amd import exact
    with _joined_engine() as e:
        e.payload_snapshots(True)
        e.recv(1, [0, 1, 2, 3])
        e.process(1, [0], [exact.OP_LOOP], 0)            # introducer joins 2,3,4, gossips
        sent_list = e.member_list(0)
        assert e.recv_callback(1, 0, 2, 3, [(3, 50, 1)]) == 0   # a newer list is committed
        assert e.member_list(0) != sent_list
        msgs = e.detach(2, 2)                            # id 3 takes its messages itself
        gossip = [m for m in msgs if m[1] == 3]
        assert gossip and all(m[3] == sent_list for m in gossip)
        e.recv(2, [1])                                   # id 2 through the batched path
        e.process(2, [1], [exact.OP_LOOP], 0)
        assert e.member_list(1) == [(1, 1, 2)] + [x for x in sent_list if x[0] != 2]


@pytest.mark.gpu
def test_null_payload_push_keeps_the_version_alive():
    """a detached GOSSIP handed back with a NULL payload (gsp_queue_push, payload =
    the sender's version at send time) must count as in flight again.  Here id 3 takes its
    messages and hands them back without lists while id 2's GOSSIP of the same version is still
    queued, then the sender commits a newer list: both receivers must still merge the list the
    GOSSIP was sent with (a double release of that version would make the second consumer fail
    with GSP_ERR_ORDER)."""
    from gossip_protocol_amd import exact
    with _joined_engine() as e:
        e.payload_snapshots(True)
        e.recv(1, [0, 1, 2, 3])
        e.process(1, [0], [exact.OP_LOOP], 0)            # introducer joins 2, 3, 4 and gossips
        sent_list = e.member_list(0)
        msgs = e.detach(2, 2)                            # id 3 takes its messages...
        assert any(m[1] == 3 for m in msgs)
        for src, typ, batch, _ in reversed(msgs):        # ...and hands them back, no lists
            assert e.queue_push(2, src, typ, None, send_batch=batch) == 0
        assert e.recv_callback(1, 0, 2, 3, [(3, 50, 1)]) == 0   # the sender commits a newer list
        assert e.member_list(0) != sent_list
        e.recv(2, [1])                                   # id 2: its own copy of the GOSSIP
        e.process(2, [1, 2], [exact.OP_LOOP, exact.OP_LOOP], 0)
        want = [(1, 1, 2)] + [x for x in sent_list if x[0] != 2]
        assert e.member_list(1) == want
        got3 = dict((x[0], x[1]) for x in e.member_list(2))
        assert 1 in got3                                 # id 3 merged its pushed-back messages
        for ident, hb, _ in sent_list:                   # the send-time list's entries
            if ident not in (1, 3):
                assert got3.get(ident) == hb, (ident, got3)
