"""The N > 1 host path on CPU: world_size-2 gloo process groups (no GPU needed).

Covers what bench.py --gpus N does around the sharded engine: broadcasting the RCCL unique
id from rank 0, summing per-rank digests (including the 64-bit event hash, modulo 2^64)
and max-reducing timings.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gossip_protocol_amd import dist as gdist
    payload = bytes(range(128)) if rank == 0 else None
    got = gdist.broadcast_bytes(payload)
    d = {"tick": 7, "node_rounds": 100 if rank == 0 else 0, "merges": 5 if rank == 0 else 0,
         "sent": 3 if rank == 0 else 0, "dropped": 0, "delivered": 3 if rank == 0 else 0,
         "joins": rank + 1, "removes": 2 * rank, "event_hash": (0xFFFFFFFFFFFFFFF0 + rank)}
    s = gdist.sum_digests(d)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, got, s, t.item()))
    dist.destroy_process_group()


def test_gloo_world2_glue():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got, s, tmax in res:
        assert got == bytes(range(128))
        assert s["node_rounds"] == 100 and s["merges"] == 5 and s["joins"] == 3
        assert s["removes"] == 2
        assert s["event_hash"] == (0xFFFFFFFFFFFFFFF0 * 2 + 1) % (1 << 64)
        assert tmax == 2.0
