"""ctypes binding of libgossip_amd.so -- the C ABI declared in include/gossip/gossip.h.

This is the same stub a maintainer would add on the reference side to call the engine
from Python.  There is no fallback: if the in-tree shared library is
missing, every entry point raises, so a GPU test can never pass on a CPU path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgossip_amd.so")
# kernel A/B experiments (scripts/ab_*.py): GSP_LIB_VARIANT=<tag> loads the in-tree
# libgossip_amd.<tag>.so built by `make lib-variant`
if os.environ.get("GSP_LIB_VARIANT"):
    LIB_PATH = os.path.join(_HERE, "libgossip_amd.%s.so" % os.environ["GSP_LIB_VARIANT"])

c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_uint64 = ctypes.c_uint64
P = ctypes.POINTER


class GspParams(ctypes.Structure):
    _fields_ = [("max_nnb", c_int32), ("single_failure", c_int32), ("drop_msg", c_int32),
                ("msg_drop_prob", ctypes.c_double), ("step_rate", ctypes.c_double),
                ("max_msg_size", c_int32), ("en_buff_size", c_int32),
                ("total_running_time", c_int32), ("tremove", c_int32),
                ("id_filter_limit", c_int32), ("intro_list", c_int32)]


class GspMemberView(ctypes.Structure):
    _fields_ = [("id", c_int32), ("port", ctypes.c_int16), ("inited", ctypes.c_int8),
                ("in_group", ctypes.c_int8), ("failed", ctypes.c_int8),
                ("heartbeat", c_int64), ("n_members", c_int32)]


class GspEntry(ctypes.Structure):
    _fields_ = [("id", c_int32), ("port", ctypes.c_int16), ("heartbeat", c_int64),
                ("timestamp", c_int64)]


class GspQueuedMsg(ctypes.Structure):
    _fields_ = [("src_id", c_int32), ("type", c_int32), ("send_batch", c_int64),
                ("payload_off", c_int64), ("payload_len", c_int32), ("pad", c_int32)]


class GspExactStats(ctypes.Structure):
    _fields_ = [("batches", c_int64), ("node_rounds", c_int64), ("merges", c_int64),
                ("draws", c_int64), ("sends_admitted", c_int64), ("device_ms", ctypes.c_double)]


MAX_FAIL_EVENTS = 8


class GspFailEvent(ctypes.Structure):
    _fields_ = [("tick", c_int32), ("mode", c_int32), ("ppm", c_int32)]


class GspPolicy(ctypes.Structure):
    """gsp_policy: driver policies of the scale engines (join schedule + bounded introducer
    list, drop window, crash events); all zeros = off."""
    _fields_ = [("drop_from", c_int32), ("drop_until", c_int32), ("step_rate", ctypes.c_double),
                ("intro_list", c_int32), ("n_fail_events", c_int32),
                ("fail_events", GspFailEvent * MAX_FAIL_EVENTS)]


def make_policy(drop_window=None, step_rate=0.0, intro_list=0, fail_events=()):
    """A GspPolicy: drop_window=(from, until), step_rate (node i starts at (int)(step_rate*i)),
    intro_list (JOINREP payload bound), fail_events=[(tick, mode, ppm), ...]."""
    p = GspPolicy()
    if drop_window:
        p.drop_from, p.drop_until = drop_window
    p.step_rate = step_rate
    p.intro_list = intro_list
    if len(fail_events) > MAX_FAIL_EVENTS:
        raise ValueError("at most %d failure events" % MAX_FAIL_EVENTS)
    p.n_fail_events = len(fail_events)
    for i, (tick, mode, ppm) in enumerate(fail_events):
        p.fail_events[i] = GspFailEvent(tick, mode, ppm)
    return p


class GspScaleParams(ctypes.Structure):
    _fields_ = [("n", c_int32), ("fanout", c_int32), ("drop_pct", c_int32),
                ("tremove", c_int32), ("h0", c_int32), ("fail_mode", c_int32),
                ("fail_tick", c_int32), ("fail_ppm", c_int32), ("seed", c_uint64),
                ("max_ticks", c_int32), ("tfail", c_int32), ("swim", c_int32),
                ("policy", GspPolicy), ("events", c_int32), ("event_cap", c_int64)]


class GspScaleDigest(ctypes.Structure):
    _fields_ = [("tick", c_int64), ("node_rounds", c_int64), ("merges", c_int64),
                ("sent", c_int64), ("dropped", c_int64), ("delivered", c_int64),
                ("joins", c_int64), ("removes", c_int64), ("event_hash", c_uint64)]


class GspScalePerf(ctypes.Structure):
    _fields_ = [("ticks", c_int64), ("merge_launches", c_int64), ("merge_ms", ctypes.c_double),
                ("csr_ms", ctypes.c_double), ("bytes_per_tick", ctypes.c_double),
                ("xgmi_bytes", ctypes.c_double)]


class GspPviewParams(ctypes.Structure):
    _fields_ = [("n", c_int32), ("view", c_int32), ("fanout", c_int32), ("inbox", c_int32),
                ("drop_pct", c_int32), ("tremove", c_int32), ("h0", c_int32),
                ("fail_mode", c_int32), ("fail_tick", c_int32), ("fail_ppm", c_int32),
                ("seed", c_uint64), ("max_ticks", c_int32), ("tfail", c_int32), ("swim", c_int32),
                ("policy", GspPolicy), ("events", c_int32), ("event_cap", c_int64),
                ("evict_order", c_int32)]


class GspPviewDigest(ctypes.Structure):
    _fields_ = [("tick", c_int64), ("node_rounds", c_int64), ("merges", c_int64),
                ("sent", c_int64), ("dropped", c_int64), ("delivered", c_int64),
                ("overflow", c_int64), ("joins", c_int64), ("removes", c_int64),
                ("evicts", c_int64), ("event_hash", c_uint64)]


# name -> (restype, argtypes); every name here must be exported (tests check it)
SIGNATURES = {
    "gsp_last_error": (ctypes.c_char_p, []),
    "gsp_abi_version": (ctypes.c_int, []),
    "gsp_device_count": (ctypes.c_int, []),
    "gsp_replay_draw": (ctypes.c_uint32, [ctypes.c_uint32, c_uint64] + [ctypes.c_uint32] * 4),
    "gsp_philox4x32_10": (ctypes.c_int, [P(ctypes.c_uint32), P(ctypes.c_uint32),
                                         P(ctypes.c_uint32)]),
    "gsp_params_default": (ctypes.c_int, [P(GspParams)]),
    "gsp_params_from_conf": (ctypes.c_int, [ctypes.c_char_p, P(GspParams)]),
    "gsp_create": (ctypes.c_int, [P(GspParams), ctypes.c_int, ctypes.c_int, c_uint64,
                                  ctypes.c_char_p, P(ctypes.c_void_p)]),
    "gsp_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "gsp_tick_recv": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(c_int32), c_int32]),
    "gsp_tick_process": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(c_int32), P(ctypes.c_int8),
                                        c_int32, c_int32]),
    "gsp_send": (ctypes.c_int, [ctypes.c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32,
                                P(c_int32)]),
    "gsp_send_list": (ctypes.c_int, [ctypes.c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32,
                                     P(GspEntry), c_int32, P(c_int32)]),
    "gsp_rand": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(c_int32)]),
    "gsp_srand": (ctypes.c_int, [ctypes.c_void_p, c_uint64]),
    "gsp_log": (ctypes.c_int, [ctypes.c_void_p, c_int32, c_int32, ctypes.c_char_p]),
    "gsp_set_failed": (ctypes.c_int, [ctypes.c_void_p, c_int32, c_int32]),
    "gsp_get_member": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(GspMemberView)]),
    "gsp_member_list": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(GspEntry), c_int32,
                                       P(c_int32)]),
    "gsp_member_lists": (ctypes.c_int, [ctypes.c_void_p, P(c_int32), c_int32, P(GspEntry),
                                        P(c_int32)]),
    "gsp_add_member": (ctypes.c_int, [ctypes.c_void_p, c_int32, c_int32, P(GspEntry), c_int32,
                                      P(c_int32)]),
    "gsp_payload_snapshots": (ctypes.c_int, [ctypes.c_void_p, c_int32]),
    "gsp_recv_detach": (ctypes.c_int, [ctypes.c_void_p, c_int32, c_int32, P(GspQueuedMsg), c_int32,
                                       P(GspEntry), c_int64, P(c_int32), P(c_int64)]),
    "gsp_queue_push": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(GspQueuedMsg), P(GspEntry)]),
    "gsp_recv_callback": (ctypes.c_int, [ctypes.c_void_p, c_int32, c_int32, P(GspQueuedMsg),
                                         P(GspEntry), c_int32]),
    "gsp_write_msgcount": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, c_int32]),
    "gsp_state_dump": (ctypes.c_int, [ctypes.c_void_p, c_int32, ctypes.c_char_p]),
    "gsp_counters": (ctypes.c_int, [ctypes.c_void_p, P(c_int32), P(c_int32), c_int32]),
    "gsp_flush_log": (ctypes.c_int, [ctypes.c_void_p]),
    "gsp_log_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                                     P(ctypes.c_size_t)]),
    "gsp_exact_stats_get": (ctypes.c_int, [ctypes.c_void_p, P(GspExactStats)]),
    "gsp_scale_params_from_conf": (ctypes.c_int, [ctypes.c_char_p, P(GspScaleParams)]),
    "gsp_pview_params_from_conf": (ctypes.c_int, [ctypes.c_char_p, P(GspPviewParams)]),
    "gsp_struct_size": (c_int64, [ctypes.c_char_p]),
    "gsp_scale_create": (ctypes.c_int, [P(GspScaleParams), ctypes.c_int, P(ctypes.c_void_p)]),
    "gsp_scale_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "gsp_scale_step": (ctypes.c_int, [ctypes.c_void_p, c_int32]),
    "gsp_scale_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "gsp_scale_tick": (ctypes.c_int, [ctypes.c_void_p, P(c_int32)]),
    "gsp_scale_digest_get": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(GspScaleDigest)]),
    "gsp_scale_row": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(ctypes.c_uint16), c_int32]),
    "gsp_scale_own_hb": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(c_int32)]),
    "gsp_scale_messages": (ctypes.c_int, [ctypes.c_void_p, P(c_int32), c_int64, P(c_int64)]),
    "gsp_scale_perf_get": (ctypes.c_int, [ctypes.c_void_p, P(GspScalePerf)]),
    "gsp_scale_set_timing": (ctypes.c_int, [ctypes.c_void_p, c_int32]),
    "gsp_scale_set_cache_policy": (ctypes.c_int, [ctypes.c_void_p, c_int32]),
    "gsp_scale_set_merge": (ctypes.c_int, [ctypes.c_void_p, c_int32]),
    "gsp_scale_nccl_id": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "gsp_scale_create_rank": (ctypes.c_int, [P(GspScaleParams), ctypes.c_int, c_int32, c_int32,
                                             ctypes.c_void_p, P(ctypes.c_void_p)]),
    "gsp_scale_create_group": (ctypes.c_int, [P(GspScaleParams), ctypes.c_int, c_int32,
                                              P(ctypes.c_void_p)]),
    "gsp_scale_create_rank_tiled": (ctypes.c_int, [P(GspScaleParams), ctypes.c_int, c_int32,
                                                   c_int32, c_int32, ctypes.c_void_p,
                                                   P(ctypes.c_void_p)]),
    "gsp_scale_create_rank_layout": (ctypes.c_int, [P(GspScaleParams), ctypes.c_int, c_int32,
                                                    c_int32, ctypes.c_void_p, c_int32,
                                                    P(ctypes.c_void_p)]),
    "gsp_scale_create_group_layout": (ctypes.c_int, [P(GspScaleParams), ctypes.c_int, c_int32,
                                                     c_int32, P(ctypes.c_void_p)]),
    "gsp_scale_layout": (ctypes.c_int, [ctypes.c_void_p, P(c_int32), P(c_int32), P(c_int64)]),
    "gsp_scale_hip_stream": (ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_void_p)]),
    "gsp_pview_create": (ctypes.c_int, [P(GspPviewParams), ctypes.c_int, P(ctypes.c_void_p)]),
    "gsp_pview_create_rank": (ctypes.c_int, [P(GspPviewParams), ctypes.c_int, c_int32, c_int32,
                                             ctypes.c_void_p, P(ctypes.c_void_p)]),
    "gsp_pview_create_group": (ctypes.c_int, [P(GspPviewParams), ctypes.c_int, c_int32,
                                              P(ctypes.c_void_p)]),
    "gsp_pview_layout": (ctypes.c_int, [ctypes.c_void_p, P(c_int32), P(c_int32), P(c_int32),
                                        P(c_int32)]),
    "gsp_pview_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "gsp_pview_step": (ctypes.c_int, [ctypes.c_void_p, c_int32]),
    "gsp_pview_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "gsp_pview_digest_get": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(GspPviewDigest)]),
    "gsp_pview_row": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(c_uint64), c_int32, P(c_int32)]),
    "gsp_pview_own_hb": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(c_int32)]),
    "gsp_pview_messages": (ctypes.c_int, [ctypes.c_void_p, P(c_int32), c_int64, P(c_int64)]),
    "gsp_pview_perf_get": (ctypes.c_int, [ctypes.c_void_p, P(GspScalePerf)]),
    "gsp_pview_drain_stats": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(c_int64), P(c_int64),
                                             P(ctypes.c_double)]),
    "gsp_pview_rows_run": (ctypes.c_int, [ctypes.c_void_p, c_int32, P(c_int64)]),
    "gsp_scale_drain_events": (ctypes.c_int, [ctypes.c_void_p, P(c_uint64), c_int64, P(c_int64),
                                              P(c_int64)]),
    "gsp_pview_drain_events": (ctypes.c_int, [ctypes.c_void_p, P(c_uint64), c_int64, P(c_int64),
                                              P(c_int64)]),
    "gsp_events_write_log": (ctypes.c_int, [P(c_uint64), c_int64, ctypes.c_char_p]),
    "gsp_fail_schedule": (ctypes.c_int, [ctypes.c_void_p, c_int32, c_uint64, c_int32, c_int32,
                                         c_int32, P(c_int32)]),
}


class GspError(RuntimeError):
    pass


EVENT_JOIN, EVENT_REMOVE, EVENT_EVICT = 1, 2, 3
# params.events: 0 off, EVENTS_ALL, or an OR of the kind bits (bit k = record kind k)
EVENTS_ALL, EVENTS_JOIN, EVENTS_REMOVE, EVENTS_EVICT = 1, 2, 4, 8


def drain_events(fn, handle):
    """Drain an engine's event ring (gsp_scale_drain_events / gsp_pview_drain_events):
    (records as uint64 numpy array, lost count)."""
    import numpy as np
    n, lost = ctypes.c_int64(), ctypes.c_int64()
    check(fn(handle, None, 0, ctypes.byref(n), ctypes.byref(lost)), "drain_events")
    buf = np.zeros(max(n.value, 1), np.uint64)
    check(fn(handle, buf.ctypes.data_as(P(c_uint64)), n.value, ctypes.byref(n), ctypes.byref(lost)),
          "drain_events")
    return buf[:n.value], lost.value


def split_events(rec):
    """(kind, tick, r, x) arrays of event records."""
    import numpy as np
    rec = np.asarray(rec, np.uint64)
    return ((rec >> np.uint64(62)).astype(np.int32), ((rec >> np.uint64(42)) & np.uint64(0xFFFFF)).astype(np.int32),
            ((rec >> np.uint64(21)) & np.uint64(0x1FFFFF)).astype(np.int32),
            (rec & np.uint64(0x1FFFFF)).astype(np.int32))


def fail_schedule(n, seed, mode, tick, ppm, policy=None):
    """gsp_fail_schedule: every node's crash tick (INT32_MAX = never) as an int32 array."""
    import numpy as np
    out = np.zeros(n, np.int32)
    check(lib().gsp_fail_schedule(ctypes.byref(policy) if policy is not None else None, n, seed,
                                  mode, tick, ppm, out.ctypes.data_as(P(c_int32))),
          "gsp_fail_schedule")
    return out


def write_event_log(rec, path):
    """gsp_events_write_log: the records as dbg.log lines (sorted canonically)."""
    import numpy as np
    rec = np.ascontiguousarray(rec, np.uint64).copy()
    check(lib().gsp_events_write_log(rec.ctypes.data_as(P(c_uint64)), len(rec), path.encode()),
          "gsp_events_write_log")


_lib = None


def lib():
    """Load the in-tree libgossip_amd.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GspError("%s is missing: run `make lib` (or __graft_entry__.build())" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().gsp_last_error()
        raise GspError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))
    return rc
