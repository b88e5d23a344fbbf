"""Python mirror of the reference's EXACT-mode interface over the C ABI.

`Engine` wraps one gsp_engine (include/gossip/gossip.h).  `run_application` drives it
with the reference Application's per-tick schedule (/root/reference/Application.cpp:90-202):
phase R = recvLoop for i ascending, phase P = nodeStart / nodeLoop for i descending, the
"@@time" line, then fail().  It writes the same files the reference writes (dbg.log,
msgcount.log) plus an end-of-tick state dump in the format of oracle/ref_hooks.cpp, so
parity tests compare it byte-for-byte with the reference's golden outputs.
"""
import ctypes
import os

from . import _lib
from ._lib import check, lib

RNG = {"glibc": 0, "philox": 1}
OP_START, OP_LOOP, OP_CHECK, OP_OPS = 0, 1, 2, 3


def params_from_conf(path):
    p = _lib.GspParams()
    check(lib().gsp_params_from_conf(path.encode(), ctypes.byref(p)), "gsp_params_from_conf")
    return p


class Engine:
    def __init__(self, params, device=0, rng="glibc", seed=0, dbg_log=None):
        self._h = ctypes.c_void_p()
        check(lib().gsp_create(ctypes.byref(params), device, RNG[rng], seed,
                               dbg_log.encode() if dbg_log else None, ctypes.byref(self._h)),
              "gsp_create")
        self.n = params.max_nnb

    def close(self):
        if self._h:
            check(lib().gsp_destroy(self._h), "gsp_destroy")
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def recv(self, tick, order):
        arr = (ctypes.c_int32 * len(order))(*order)
        check(lib().gsp_tick_recv(self._h, tick, arr, len(order)), "gsp_tick_recv")

    def process(self, tick, order, ops, dropmsg):
        arr = (ctypes.c_int32 * len(order))(*order)
        oa = (ctypes.c_int8 * len(ops))(*ops)
        check(lib().gsp_tick_process(self._h, tick, arr, oa, len(order), int(dropmsg)),
              "gsp_tick_process")

    def rand(self, tick):
        v = ctypes.c_int32()
        check(lib().gsp_rand(self._h, tick, ctypes.byref(v)), "gsp_rand")
        return v.value

    def log(self, node, tick, text):
        check(lib().gsp_log(self._h, node, tick, text.encode()), "gsp_log")

    def set_failed(self, node, failed=True):
        check(lib().gsp_set_failed(self._h, node, int(failed)), "gsp_set_failed")

    def member(self, node):
        v = _lib.GspMemberView()
        check(lib().gsp_get_member(self._h, node, ctypes.byref(v)), "gsp_get_member")
        return v

    def member_list(self, node):
        buf = (_lib.GspEntry * self.n)()
        cnt = ctypes.c_int32()
        check(lib().gsp_member_list(self._h, node, buf, self.n, ctypes.byref(cnt)),
              "gsp_member_list")
        return [(buf[i].id, buf[i].heartbeat, buf[i].timestamp) for i in range(cnt.value)]

    def state_dump(self, tick, path):
        check(lib().gsp_state_dump(self._h, tick, path.encode()), "gsp_state_dump")

    def write_msgcount(self, path, tick):
        check(lib().gsp_write_msgcount(self._h, path.encode(), tick), "gsp_write_msgcount")

    def log_bytes(self):
        n = ctypes.c_size_t()
        check(lib().gsp_log_bytes(self._h, None, 0, ctypes.byref(n)), "gsp_log_bytes")
        buf = ctypes.create_string_buffer(n.value + 1)
        check(lib().gsp_log_bytes(self._h, buf, n.value, ctypes.byref(n)), "gsp_log_bytes")
        return buf.raw[:n.value]

    # driver-side receive (gossip.h): ENrecv with a driver callback, Queue::enqueue, direct
    # recvCallBack; a message is (src_id, type, send_batch, [(id, heartbeat, timestamp), ...])
    def payload_snapshots(self, on=True):
        check(lib().gsp_payload_snapshots(self._h, int(on)), "gsp_payload_snapshots")

    def detach_sizes(self, tick, node):
        n, np_ = ctypes.c_int32(), ctypes.c_int64()
        check(lib().gsp_recv_detach(self._h, tick, node, None, 0, None, 0, ctypes.byref(n),
                                    ctypes.byref(np_)), "gsp_recv_detach")
        return n.value, np_.value

    def detach(self, tick, node):
        cnt, total = self.detach_sizes(tick, node)
        msgs = (_lib.GspQueuedMsg * max(1, cnt))()
        pl = (_lib.GspEntry * max(1, total))()
        n, np_ = ctypes.c_int32(), ctypes.c_int64()
        check(lib().gsp_recv_detach(self._h, tick, node, msgs, cnt, pl, total, ctypes.byref(n),
                                    ctypes.byref(np_)), "gsp_recv_detach")
        out = []
        for m in msgs[:n.value]:
            ents = [(pl[k].id, pl[k].heartbeat, pl[k].timestamp)
                    for k in range(m.payload_off, m.payload_off + m.payload_len)]
            out.append((m.src_id, m.type, m.send_batch, ents))
        return out

    @staticmethod
    def _msg(src_id, type_, payload, send_batch=-1):
        m = _lib.GspQueuedMsg(src_id=src_id, type=type_, send_batch=send_batch)
        if payload is None:
            return m, None
        m.payload_len = len(payload)
        arr = (_lib.GspEntry * max(1, len(payload)))()
        for k, ent in enumerate(payload):
            ident, hb, ts = ent[:3]
            arr[k] = _lib.GspEntry(id=ident, port=ent[3] if len(ent) > 3 else 0, heartbeat=hb,
                                   timestamp=ts)
        return m, arr

    def queue_push(self, node, src_id, type_, payload, send_batch=-1):
        m, arr = self._msg(src_id, type_, payload, send_batch)
        return lib().gsp_queue_push(self._h, node, ctypes.byref(m), arr)

    def recv_callback(self, tick, node, src_id, type_, payload, dropmsg=0, send_batch=-1):
        m, arr = self._msg(src_id, type_, payload, send_batch)
        return lib().gsp_recv_callback(self._h, tick, node, ctypes.byref(m), arr, int(dropmsg))

    def counters(self, ticks):
        n = self.n + 1
        sent = (ctypes.c_int32 * (n * ticks))()
        recv = (ctypes.c_int32 * (n * ticks))()
        check(lib().gsp_counters(self._h, sent, recv, ticks), "gsp_counters")
        return list(sent), list(recv)

    def stats(self):
        s = _lib.GspExactStats()
        check(lib().gsp_exact_stats_get(self._h, ctypes.byref(s)), "gsp_exact_stats_get")
        return s


def run_application(conf_path, seed, rng="glibc", out_dir=".", device=0, ticks=None,
                    state_dump=True, intro_list=0):
    """Run one testcase the way the reference Application does; returns output paths.
    intro_list: gsp_params.intro_list, the opt-in bounded introducer list (0 = reference)."""
    p = params_from_conf(conf_path)
    p.intro_list = intro_list
    n = p.max_nnb
    T = p.total_running_time if ticks is None else ticks
    os.makedirs(out_dir, exist_ok=True)
    dbg = os.path.join(out_dir, "dbg.log")
    state_path = os.path.join(out_dir, "state.txt")
    if state_dump and os.path.exists(state_path):
        os.remove(state_path)
    stdout_lines = []
    failed = [False] * n
    dropmsg = 0
    with Engine(p, device, rng, seed, dbg) as e:
        for i in range(n):                                   # Application.cpp:58-68
            e.log(i, 0, "APP")
        for t in range(T):                                   # Application.cpp:99-104
            start_t = [int(p.step_rate * i) for i in range(n)]
            recv = [i for i in range(n) if t > start_t[i] and not failed[i]]
            e.recv(t, recv)                                  # Application.cpp:125-135
            order, ops = [], []
            for i in range(n - 1, -1, -1):                   # Application.cpp:138-163
                if t == start_t[i]:
                    order.append(i)
                    ops.append(OP_START)
                    stdout_lines.append("%d-th introduced node is assigned with the address: %d:0"
                                        % (i, i + 1))
                    failed[i] = False
                elif t > start_t[i] and not failed[i]:
                    order.append(i)
                    ops.append(OP_LOOP)
            e.process(t, order, ops, dropmsg)
            if t % 500 == 0 and 0 in order and ops[order.index(0)] == OP_LOOP:
                e.log(0, t, "@@time=%d" % t)
            # Application::fail (Application.cpp:173-202)
            if p.drop_msg and t == 50:
                dropmsg = 1
            if p.single_failure and t == 100:
                victim = e.rand(t) % n
                e.log(victim, t, "Node failed at time=%d" % t)
                failed[victim] = True
                e.set_failed(victim, True)
            elif t == 100:
                first = e.rand(t) % n // 2
                for i in range(first, first + n // 2):
                    e.log(i, t, "Node failed at time = %d" % t)
                    failed[i] = True
                    e.set_failed(i, True)
            if p.drop_msg and t == 300:
                dropmsg = 0
            if state_dump:
                e.state_dump(t, state_path)
        e.write_msgcount(os.path.join(out_dir, "msgcount.log"), T)
        stats = e.stats()
    with open(os.path.join(out_dir, "stdout.txt"), "w") as f:
        f.write("".join(l + "\n" for l in stdout_lines))
    return {"dbg.log": dbg, "msgcount.log": os.path.join(out_dir, "msgcount.log"),
            "state.txt": os.path.join(out_dir, "state.txt"),
            "stdout.txt": os.path.join(out_dir, "stdout.txt"), "stats": stats}
