#!/usr/bin/env python3
"""One rank of a multi-GPU parity run (tests/test_rccl_multi_gpu.py launches it under
torch.distributed.run, one fresh process per GPU, no GPU call before it starts).

    python -m torch.distributed.run --nproc-per-node N tests/rccl_ranks.py <case>

cases (the sharded form of EmulNet::ENsend / ENrecv, /root/reference/EmulNet.cpp:87-177):
  columns_tiled   full view, column shards, 2 column tiles per rank: count all-gather and
                  the picks all-reduce MAX over RCCL between the ranks
  rows            full view, row shards: sender rows and message records move between the
                  ranks by grouped ncclSend / ncclRecv, counts by all-gather / broadcast,
                  node 0's row by ncclBroadcast (join schedule)
  pview_rows      partial view, row shards: the same exchange for sender views
  pview_burst, rows_burst
                  a join burst (step_rate 0.0005: most nodes start at one tick knowing only the
                  introducer) -- the partial view drained (inbox 0) and the full view's rows: the
                  sizes posted to RCCL from earlier ticks' counts must absorb the burst's growth
                  (rowx_host.cpp's growth-aware margins)
  pview_capacity, rows_capacity
                  a test's segment bound (GSP_TEST_MAX_SEGMENT) that a receiver of one rank
                  passes first: every rank's sync() must raise GSP_ERR_CAPACITY at the same
                  step, naming the same tick (the flag is all-reduced before the
                  tick kernels read it)

Every rank runs the engine and the CPU oracle on the same inputs.  torch.distributed (gloo)
carries only the RCCL id and the digests.  Checks: each tick's digest summed over ranks
equals the oracle's; each rank's own part of sampled rows equals the oracle's; the messages
each rank's rows sent equal the oracle's; the engine sent bytes to other ranks
(xgmi_bytes > 0).  Rank 0 prints one JSON line; exit status 0 means parity.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RANDOM = 1


def _check_scale_rows(eng, orc, n, rows, cols):
    from gossip_protocol_amd.scale import unpack
    for r in rows:
        pres_o, hb_o, ts_o = orc.row(r)
        pres_d, hb_d, ts5_d = unpack(eng.row(r))
        sl = slice(*cols)
        p = pres_d[sl]
        assert np.array_equal(p, pres_o[sl].astype(bool)), "presence row %d" % r
        assert np.array_equal(hb_d[sl][p], hb_o[sl][p]), "hb row %d" % r
        assert np.array_equal(ts5_d[sl][p], ts_o[sl][p] & 31), "ts row %d" % r


def run(case):
    import torch.distributed as dist
    from gossip_protocol_amd.dist import broadcast_bytes, sum_digests
    from gossip_protocol_amd.scale import ScaleEngine, make_policy, nccl_unique_id
    from tests.oracle_binding import PviewOracle, ScaleOracle
    from tests.oracle_binding import make_policy as oracle_policy
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = int(os.environ.get("LOCAL_RANK", "0"))
    uid = broadcast_bytes(nccl_unique_id() if rank == 0 else None)
    ticks = 12
    bad = []
    if case in ("pview_capacity", "rows_capacity"):
        return run_capacity(case, rank, world, dev, uid)
    if case in ("columns_tiled", "rows", "rows_burst"):
        n = 8192
        kw = dict(fanout=3, drop_pct=10, fail_mode=RANDOM, fail_tick=4, fail_ppm=20000, seed=8,
                  tfail=5, swim=2)
        pol = dict(drop_window=(2, 9), step_rate=0.02, intro_list=4, fail_events=[(7, 3, 0)])
        if case == "rows_burst":
            kw = dict(fanout=3, drop_pct=10, fail_mode=RANDOM, fail_tick=6, fail_ppm=20000, seed=9)
            pol = dict(step_rate=0.0005, intro_list=0)
        orc = ScaleOracle(n, policy=oracle_policy(**pol), **kw)
        eng = ScaleEngine(n, max_ticks=ticks, device=dev, rank=rank, world=world, nccl_id=uid,
                          tiles=2 if case == "columns_tiled" else 1,
                          layout="columns" if case == "columns_tiled" else "rows",
                          policy=make_policy(**pol), **kw)
        shards, first, stride = eng.layout()
        if case == "columns_tiled":
            per = shards // world
            cols = (first * stride, min(n, (first + per) * stride))
            rows_mine = list(range(0, n, 97)) + [n - 1]
        else:
            lo, hi = rank * n // world, (rank + 1) * n // world
            cols = (0, n)
            rows_mine = list(range(lo, hi, 53)) + [hi - 1]
    else:
        n = 20000
        kw = dict(view=64, fanout=3, inbox=5, drop_pct=10, fail_mode=2, fail_tick=5,
                  fail_ppm=50000, seed=13)
        pol = None
        if case == "pview_burst":
            n = 6000
            kw = dict(view=64, fanout=3, inbox=0, drop_pct=10, fail_mode=2, fail_tick=6,
                      fail_ppm=20000, seed=43)
            pol = dict(step_rate=0.0005, intro_list=0)
        from gossip_protocol_amd.pview import PviewEngine
        orc = PviewOracle(n, policy=oracle_policy(**pol) if pol else None, **kw)
        eng = PviewEngine(n, max_ticks=ticks, device=dev, rank=rank, world=world, nccl_id=uid,
                          policy=make_policy(**pol) if pol else None, **kw)
        lo, hi = rank * n // world, (rank + 1) * n // world
        rows_mine = list(range(lo, hi, 37)) + [hi - 1]
    for t in range(1, ticks + 1):
        want = orc.step()
        eng.step(1)
        got = sum_digests(eng.digest(t))
        if got != want:
            bad.append(("digest", t, got, want))
    if case in ("columns_tiled", "rows", "rows_burst"):
        try:
            _check_scale_rows(eng, orc, n, rows_mine, cols)
        except AssertionError as e:
            bad.append(("rows", str(e)))
        m = eng.messages()
        src, dst = orc.messages()
        if case == "columns_tiled":        # every rank holds the whole message list
            got_m = sorted((s, d) for s in range(n) for d in m[s] if d >= 0)
            want_m = sorted(zip(src.tolist(), dst.tolist()))
        else:                              # this rank's rows' sends
            got_m = sorted((lo + i, d) for i in range(hi - lo) for d in m[i] if d >= 0)
            want_m = sorted((s, d) for s, d in zip(src.tolist(), dst.tolist()) if lo <= s < hi)
    else:
        for r in rows_mine:
            ids, hb, ts = orc.row(r)
            e, ln = eng.row(r)
            e = e[:ln]
            gi = (e >> np.uint64(32)).astype(np.int64)
            gv = (e & np.uint64(0xFFFF)).astype(np.int64)
            if not (np.array_equal(gi, ids) and np.array_equal(gv >> 5, hb) and
                    np.array_equal(gv & 31, ts & 31)):
                bad.append(("view", r))
                break
        m = eng.messages()
        src, dst = orc.messages()
        got_m = sorted((lo + i, d) for i in range(hi - lo) for d in m[i] if d >= 0)
        want_m = sorted((s, d) for s, d in zip(src.tolist(), dst.tolist()) if lo <= s < hi)
    if got_m != want_m:
        bad.append(("messages", len(got_m), len(want_m)))
    xgmi = eng.perf()["xgmi_bytes"]
    if world > 1 and not xgmi > 0:
        bad.append(("xgmi_bytes", xgmi))
    eng.close()
    orc.close()
    res = [None] * world
    dist.all_gather_object(res, {"rank": rank, "bad": [str(b)[:300] for b in bad], "xgmi": xgmi})
    if rank == 0:
        print(json.dumps({"case": case, "world": world, "ranks": res}), flush=True)
    dist.destroy_process_group()
    return 0 if not any(r["bad"] for r in res) else 1


def run_capacity(case, rank, world, dev, uid):
    import torch.distributed as dist
    from gossip_protocol_amd._lib import GspError
    from gossip_protocol_amd.scale import ScaleEngine
    os.environ["GSP_TEST_MAX_SEGMENT"] = "9"     # in-degree ~ Poisson(3): a few receivers pass 9
    if case == "pview_capacity":
        from gossip_protocol_amd.pview import PviewEngine
        eng = PviewEngine(20000, view=64, fanout=3, inbox=5, seed=13, max_ticks=30, device=dev,
                          rank=rank, world=world, nccl_id=uid)
    else:
        eng = ScaleEngine(8192, fanout=3, seed=8, max_ticks=30, device=dev, rank=rank, world=world,
                          nccl_id=uid, layout="rows")
    stop = None
    for t in range(1, 31):
        eng.step(1)
        try:
            eng.sync()
        except GspError as e:
            import re
            m = re.search(r"at tick (\d+)", str(e))
            stop = (t, int(m.group(1)) if m else str(e)[:200])
            break
    eng.close()
    res = [None] * world
    dist.all_gather_object(res, {"rank": rank, "stop": stop})
    ok = stop is not None and all(r["stop"] == res[0]["stop"] for r in res)
    if rank == 0:
        print(json.dumps({"case": case, "world": world, "ranks": [dict(r, bad=[] if ok else ["stop"])
                                                                   for r in res]}), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(run(sys.argv[1]))
