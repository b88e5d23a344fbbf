"""One process per GPU: the host glue around gsp_scale_create_rank.

torch.distributed is plumbing only: it carries the 128-byte RCCL unique id from rank 0 to
the other ranks and reduces the per-rank digests / timings.  The per-tick exchange of the
sharded engine runs inside libgossip_amd.so on its own RCCL communicator.
"""
import torch
import torch.distributed as dist



def broadcast_bytes(payload, src=0):
    """Broadcast a bytes object from `src` to every rank (any backend)."""
    obj = [payload if dist.get_rank() == src else None]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


def sum_digests(d):
    """Job digest from this rank's digest: every count is summed over ranks and the event
    hash is summed modulo 2^64.  Column shards (full view) count per-row quantities on rank
    0 only and per-column ones on every rank; row shards (partial view) count everything on
    the rank that owns the row -- either way the sum is the job's digest."""
    keys = [k for k in d if k not in ("tick", "event_hash")]
    vals = [int(d[k]) for k in keys]
    t = torch.tensor(vals + [int(d["event_hash"]) & 0xFFFFFFFF, int(d["event_hash"]) >> 32],
                     dtype=torch.int64)
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    out = {"tick": d["tick"]}
    for i, k in enumerate(keys):
        out[k] = int(sum(int(p[i]) for p in parts))
    lo = sum(int(p[len(keys)]) for p in parts)
    hi = sum(int(p[len(keys) + 1]) for p in parts)
    out["event_hash"] = ((hi << 32) + lo) & 0xFFFFFFFFFFFFFFFF
    return out


def make_rank_engine(n, local_device, **kw):
    """Column shard `rank` of `world` on `local_device`, communicator set up over RCCL."""
    from .scale import ScaleEngine, nccl_unique_id
    rank, world = dist.get_rank(), dist.get_world_size()
    uid = broadcast_bytes(nccl_unique_id() if rank == 0 else None)
    return ScaleEngine(n, device=local_device, rank=rank, world=world, nccl_id=uid, **kw)


def make_pview_rank_engine(n, local_device, **kw):
    """Row shard `rank` of `world` of the partial-view engine, exchange over RCCL."""
    from .pview import PviewEngine
    from .scale import nccl_unique_id
    rank, world = dist.get_rank(), dist.get_world_size()
    uid = broadcast_bytes(nccl_unique_id() if rank == 0 else None)
    return PviewEngine(n, device=local_device, rank=rank, world=world, nccl_id=uid, **kw)
