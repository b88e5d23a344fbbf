#!/usr/bin/env python3
"""Two RCCL ranks of the scale engine (column shards, optionally 2 tiles each) against the
oracle -- launched with torch.distributed.run --nproc-per-node 2.  torch.distributed (gloo)
only carries the RCCL id and the digests; the engine's own communicator does the exchange.
GSP_SAME_GPU=1 puts both ranks on device 0 (RCCL may refuse duplicate GPUs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = 0 if os.environ.get("GSP_SAME_GPU") else int(os.environ.get("LOCAL_RANK", "0"))
    from gossip_protocol_amd.dist import broadcast_bytes
    from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine, nccl_unique_id
    tiles = int(os.environ.get("GSP_TILES", "1"))
    uid = broadcast_bytes(nccl_unique_id() if rank == 0 else None)
    n, ticks = 8192, 12
    kw = dict(fanout=3, drop_pct=10, fail_mode=FAIL_RANDOM, fail_tick=4, fail_ppm=20000, seed=8,
              tfail=5, swim=2)
    eng = ScaleEngine(n, max_ticks=ticks, device=dev, rank=rank, world=world, nccl_id=uid,
                      tiles=tiles, **kw)
    eng.step(ticks)
    from gossip_protocol_amd.dist import sum_digests
    dg = [sum_digests(eng.digest(t)) for t in range(1, ticks + 1)]
    eng.close()
    if rank == 0:
        from tests.oracle_binding import ScaleOracle
        orc = ScaleOracle(n, **kw)
        bad = [(t, dg[t - 1], w) for t, w in ((t, orc.step()) for t in range(1, ticks + 1))
               if dg[t - 1] != w]
        print("two-rank RCCL run (tiles %d) vs oracle: %s" % (tiles, "OK" if not bad else bad[:2]),
              flush=True)
        if bad:
            sys.exit(1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
