"""Python side of the PARTIAL-VIEW engine (gsp_pview_* in include/gossip/gossip.h)."""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib

EMPTY = np.uint64(0xFFFFFFFFFFFFFFFF)


def unpack_view(entries, length):
    """(ids, hb, ts mod 32) of the first `length` packed entries."""
    e = np.asarray(entries, dtype=np.uint64)[:length]
    ids = (e >> np.uint64(32)).astype(np.int64)
    p = (e & np.uint64(0xFFFF)).astype(np.int64)
    return ids, p >> 5, p & 31


def params_from_conf(path):
    """gsp_pview_params from a .conf (gsp_pview_params_from_conf)."""
    p = _lib.GspPviewParams()
    check(lib().gsp_pview_params_from_conf(path.encode(), ctypes.byref(p)),
          "gsp_pview_params_from_conf")
    return p


class PviewEngine:
    """One partial-view engine.

    group=G (> 1): G row shards inside this process on `device` (exchange by device copies).
    rank/world/nccl_id: this process holds row shard `rank` of `world` (exchange over RCCL;
    the id comes from scale.nccl_unique_id() on rank 0).  Default: one GPU, all rows.
    """

    def __init__(self, n, view=256, fanout=3, inbox=7, drop_pct=0, tremove=20, h0=1,
                 fail_mode=0, fail_tick=10, fail_ppm=0, seed=0x5EED, max_ticks=256, device=0,
                 group=1, rank=0, world=1, nccl_id=None, tfail=0, swim=0, policy=None,
                 events=False, event_cap=0, evict_order=0, params=None):
        if params is None:
            params = _lib.GspPviewParams(n=n, view=view, fanout=fanout, inbox=inbox,
                                         drop_pct=drop_pct, tremove=tremove, h0=h0,
                                         fail_mode=fail_mode, fail_tick=fail_tick,
                                         fail_ppm=fail_ppm, seed=seed, max_ticks=max_ticks,
                                         tfail=tfail, swim=swim, policy=policy or _lib.GspPolicy(),
                                         events=int(events), event_cap=event_cap,
                                         evict_order=evict_order)
        self.params = params
        n, view, fanout = params.n, params.view, params.fanout
        self._h = ctypes.c_void_p()
        P = ctypes.byref
        if nccl_id is not None:
            idbuf = ctypes.create_string_buffer(nccl_id, 128)
            check(lib().gsp_pview_create_rank(P(self.params), device, rank, world, idbuf,
                                              P(self._h)), "gsp_pview_create_rank")
        elif group > 1:
            check(lib().gsp_pview_create_group(P(self.params), device, group, P(self._h)),
                  "gsp_pview_create_group")
        else:
            check(lib().gsp_pview_create(P(self.params), device, P(self._h)), "gsp_pview_create")
        self.n, self.view, self.fanout = n, view, fanout

    def layout(self):
        """(shards, first shard held, its first row, rows held here)."""
        v = [ctypes.c_int32() for _ in range(4)]
        check(lib().gsp_pview_layout(self._h, *[ctypes.byref(x) for x in v]), "gsp_pview_layout")
        return tuple(x.value for x in v)

    def close(self):
        if self._h:
            check(lib().gsp_pview_destroy(self._h), "gsp_pview_destroy")
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def step(self, ticks=1):
        check(lib().gsp_pview_step(self._h, ticks), "gsp_pview_step")

    def sync(self):
        check(lib().gsp_pview_sync(self._h), "gsp_pview_sync")

    def digest(self, t):
        d = _lib.GspPviewDigest()
        check(lib().gsp_pview_digest_get(self._h, t, ctypes.byref(d)), "gsp_pview_digest_get")
        return {k: getattr(d, k) for k, _ in d._fields_}

    def row(self, r):
        buf = np.zeros(self.view, np.uint64)
        ln = ctypes.c_int32()
        check(lib().gsp_pview_row(self._h, r, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                  self.view, ctypes.byref(ln)), "gsp_pview_row")
        return buf, ln.value

    def own_hb(self, r):
        v = ctypes.c_int32()
        check(lib().gsp_pview_own_hb(self._h, r, ctypes.byref(v)), "gsp_pview_own_hb")
        return v.value

    def messages(self):
        n = ctypes.c_int64()
        check(lib().gsp_pview_messages(self._h, None, 0, ctypes.byref(n)), "gsp_pview_messages")
        buf = np.zeros(max(n.value, 1), np.int32)
        check(lib().gsp_pview_messages(self._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       n.value, ctypes.byref(n)), "gsp_pview_messages")
        return buf[:n.value].reshape(-1, self.fanout)

    def drain_events(self):
        """(records, lost) since the last drain (events=True); see _lib.split_events."""
        return _lib.drain_events(lib().gsp_pview_drain_events, self._h)

    def rows_run(self, t):
        """Tests: rows the tick kernels of tick t ran (GSP_TEST_PV_COUNT_ROWS=1 at create)."""
        v = ctypes.c_int64()
        check(lib().gsp_pview_rows_run(self._h, t, ctypes.byref(v)), "gsp_pview_rows_run")
        return v.value

    def drain_stats(self, classes=5):
        """Drain all (inbox 0): per row class since create, {"rows", "messages", "ms"} lists
        (gsp_pview_drain_stats; classes 0-3 the LDS classes, 4 the hub kernel)."""
        rows = np.zeros(classes, np.int64)
        msgs = np.zeros(classes, np.int64)
        ms = np.zeros(classes, np.float64)
        P = ctypes.POINTER
        check(lib().gsp_pview_drain_stats(self._h, classes, rows.ctypes.data_as(P(ctypes.c_int64)),
                                          msgs.ctypes.data_as(P(ctypes.c_int64)),
                                          ms.ctypes.data_as(P(ctypes.c_double))),
              "gsp_pview_drain_stats")
        return {"rows": rows.tolist(), "messages": msgs.tolist(), "ms": ms.tolist()}

    def perf(self):
        p = _lib.GspScalePerf()
        check(lib().gsp_pview_perf_get(self._h, ctypes.byref(p)), "gsp_pview_perf_get")
        return {k: getattr(p, k) for k, _ in p._fields_}
