"""Python side of the SCALE engine (gsp_scale_* in include/gossip/gossip.h).

Entries come back packed as the device stores them: hb << 5 | (ts mod 32), 0 = absent.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib

FAIL_NONE, FAIL_RANDOM, FAIL_BLOCK, FAIL_SINGLE, FAIL_HALF = 0, 1, 2, 3, 4
make_policy = _lib.make_policy
LAYOUTS = {"columns": 0, "rows": 1}


def unpack(entries):
    e = np.asarray(entries, dtype=np.uint16)
    present = e != 0
    return present, (e >> 5).astype(np.int32), (e & 31).astype(np.int32)


def params_from_conf(path):
    """gsp_scale_params from a .conf (the reference's four keys, then optional scale keys;
    include/gossip/gossip.h gsp_scale_params_from_conf)."""
    p = _lib.GspScaleParams()
    check(lib().gsp_scale_params_from_conf(path.encode(), ctypes.byref(p)),
          "gsp_scale_params_from_conf")
    return p


def nccl_unique_id():
    """RCCL unique id (bytes) for gsp_scale_create_rank; made by rank 0, broadcast by caller."""
    buf = ctypes.create_string_buffer(128)
    check(lib().gsp_scale_nccl_id(buf, 128), "gsp_scale_nccl_id")
    return buf.raw


class ScaleEngine:
    """One scale engine.

    group=G (> 1): G shards inside this process on `device` (exchange by device copies).
    rank/world/nccl_id: this process holds shard `rank` of `world` (exchange over RCCL).
    tiles (with nccl_id): this rank runs its columns as `tiles` column tiles (shared exchange
    inside the rank, gsp_scale_create_rank_tiled); group: G in-process column tiles of one GPU.
    layout: "columns" (column slices of every row) or "rows" (row blocks; sender rows move
    between shards).  Default: one GPU, full rows, fused tick kernel.
    tfail > 0: TFAIL suspicion (members tfail or more ticks stale are listed but not gossiped,
    chosen or counted); 0 is the reference's protocol.
    swim = s > 0: SWIM ping/ack probing, one probe target per node per tick over 1 direct + s - 1
    indirect paths (answered: ts refreshed; unanswered: removed); every layout.
    """

    def __init__(self, n, fanout=3, drop_pct=0, tremove=20, h0=1, fail_mode=FAIL_NONE,
                 fail_tick=10, fail_ppm=0, seed=0x5EED, max_ticks=256, device=0, group=1,
                 rank=0, world=1, nccl_id=None, layout="columns", tfail=0, swim=0, policy=None,
                 events=False, event_cap=0, params=None, tiles=1):
        if params is None:
            params = _lib.GspScaleParams(n=n, fanout=fanout, drop_pct=drop_pct, tremove=tremove,
                                         h0=h0, fail_mode=fail_mode, fail_tick=fail_tick,
                                         fail_ppm=fail_ppm, seed=seed, max_ticks=max_ticks,
                                         tfail=tfail, swim=swim, policy=policy or _lib.GspPolicy(),
                                         events=int(events), event_cap=event_cap)
        self.params = params
        n, fanout = params.n, params.fanout
        self._h = ctypes.c_void_p()
        lay = LAYOUTS[layout]
        if nccl_id is not None and tiles > 1:        # column tiles of this rank (columns)
            idbuf = ctypes.create_string_buffer(nccl_id, 128)
            check(lib().gsp_scale_create_rank_tiled(ctypes.byref(self.params), device, rank, world,
                                                    tiles, idbuf, ctypes.byref(self._h)),
                  "gsp_scale_create_rank_tiled")
        elif nccl_id is not None:
            idbuf = ctypes.create_string_buffer(nccl_id, 128)
            check(lib().gsp_scale_create_rank_layout(ctypes.byref(self.params), device, rank, world,
                                                     idbuf, lay, ctypes.byref(self._h)),
                  "gsp_scale_create_rank_layout")
        elif group > 1:
            check(lib().gsp_scale_create_group_layout(ctypes.byref(self.params), device, group, lay,
                                                      ctypes.byref(self._h)),
                  "gsp_scale_create_group_layout")
        else:
            check(lib().gsp_scale_create(ctypes.byref(self.params), device, ctypes.byref(self._h)),
                  "gsp_scale_create")
        self.n = n
        self.fanout = fanout

    def layout(self):
        g, r, s = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        check(lib().gsp_scale_layout(self._h, ctypes.byref(g), ctypes.byref(r), ctypes.byref(s)),
              "gsp_scale_layout")
        return g.value, r.value, s.value

    def set_merge(self, packed):
        check(lib().gsp_scale_set_merge(self._h, int(packed)), "gsp_scale_set_merge")

    def close(self):
        if self._h:
            check(lib().gsp_scale_destroy(self._h), "gsp_scale_destroy")
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def step(self, ticks=1):
        check(lib().gsp_scale_step(self._h, ticks), "gsp_scale_step")

    def sync(self):
        check(lib().gsp_scale_sync(self._h), "gsp_scale_sync")

    @property
    def tick(self):
        t = ctypes.c_int32()
        check(lib().gsp_scale_tick(self._h, ctypes.byref(t)), "gsp_scale_tick")
        return t.value

    def digest(self, t):
        d = _lib.GspScaleDigest()
        check(lib().gsp_scale_digest_get(self._h, t, ctypes.byref(d)), "gsp_scale_digest_get")
        return {k: getattr(d, k) for k, _ in d._fields_}

    def row(self, r):
        buf = np.zeros(self.n, np.uint16)
        check(lib().gsp_scale_row(self._h, r, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)),
                                  self.n), "gsp_scale_row")
        return buf

    def own_hb(self, r):
        v = ctypes.c_int32()
        check(lib().gsp_scale_own_hb(self._h, r, ctypes.byref(v)), "gsp_scale_own_hb")
        return v.value

    def messages(self):
        n = ctypes.c_int64()
        check(lib().gsp_scale_messages(self._h, None, 0, ctypes.byref(n)), "gsp_scale_messages")
        buf = np.zeros(max(n.value, 1), np.int32)
        check(lib().gsp_scale_messages(self._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       n.value, ctypes.byref(n)), "gsp_scale_messages")
        return buf[:n.value].reshape(-1, self.fanout)

    def perf(self):
        p = _lib.GspScalePerf()
        check(lib().gsp_scale_perf_get(self._h, ctypes.byref(p)), "gsp_scale_perf_get")
        return {k: getattr(p, k) for k, _ in p._fields_}

    def set_timing(self, on):
        check(lib().gsp_scale_set_timing(self._h, int(on)), "gsp_scale_set_timing")

    def set_cache_policy(self, policy):
        check(lib().gsp_scale_set_cache_policy(self._h, int(policy)), "gsp_scale_set_cache_policy")

    def drain_events(self):
        """(records, lost) since the last drain (events=True); see _lib.split_events."""
        return _lib.drain_events(lib().gsp_scale_drain_events, self._h)

    def stream(self):
        s = ctypes.c_void_p()
        check(lib().gsp_scale_hip_stream(self._h, ctypes.byref(s)), "gsp_scale_hip_stream")
        return s.value
