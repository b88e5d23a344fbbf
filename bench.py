#!/usr/bin/env python3
"""Headline benchmark: gossip node-rounds/s on the SCALE engine (BASELINE.json configs 3-5).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-pview] [--no-cpu-baseline]

One "step" = one protocol tick over the whole node population: every alive node merges
the rows gossiped to it, bumps its heartbeat, runs the TREMOVE scan and gossips to `fanout`
peers (the reference's nodeLoop, /root/reference/MP1Node.cpp:176-362, at scale).

Headline (`value`, `roofline`): BASELINE config 3 -- 65,536 nodes, full view (65,536 x
65,536 packed u16 table), fanout 3, 1% random crash at t = 10, no drops; ticks 1..W warm up,
W+1..W+K timed.  N > 1: the same workload (strong scaling), column-sharded over N GPUs, one
process per GPU; the engine exchanges per-row counts and peer choices over its own RCCL
communicator, torch.distributed only carries the RCCL id, the barrier and the timing
reductions (DESIGN.md "Multi-GPU").
Second line item (`pview`): BASELINE config 5 -- 1,048,576 nodes, bounded partial view
V = 256, fanout 3, inbox 7, 10% drops, 5% contiguous crash at t = 10; N > 1: row-sharded
over N GPUs with the per-tick sender-view exchange over RCCL send/recv (strong scaling);
reports its own node-rounds/s, tick-kernel roofline and xGMI bytes per tick.
Prints ONE JSON line (rank 0) with the roofline of the fused tick kernel and the CPU
baseline (the oracle restatement, timed on a bounded sample of the same workload).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0       # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
N_NODES = 65536
FANOUT = 3
FAIL_PPM = 10000            # 1 %
FAIL_TICK = 10
SEED = 0x5EED


def cpu_baseline(budget_s=12.0):
    """Oracle restatement (oracle/scale_oracle.c, 1 thread) on a bounded sample.

    The full 65,536-wide table does not fit a CPU run of seconds, so the sample is the same
    protocol at n = 4096 (full view, fanout 3, 1% crash at t = 10); its throughput in table
    entries processed per second is converted to node-rounds/s of the 65,536-wide workload
    (a node-round there processes 65,536 x (1 + k) entries, k = messages merged).
    """
    from tests.oracle_binding import ScaleOracle
    n = 4096
    orc = ScaleOracle(n, fanout=FANOUT, drop_pct=0, fail_mode=1, fail_tick=FAIL_TICK,
                      fail_ppm=FAIL_PPM, seed=SEED)
    t0 = time.perf_counter()
    ticks = rounds = delivered = 0
    while time.perf_counter() - t0 < budget_s and ticks < 60:
        d = orc.step()
        ticks += 1
        rounds += d["node_rounds"]
        delivered += d["delivered"]
    el = time.perf_counter() - t0
    orc.close()
    entries = (rounds + delivered) * n          # own row + one sender row per message
    entries_per_s = entries / el
    k = delivered / max(rounds, 1)
    per_round_65k = N_NODES * (1.0 + k)
    return {"value": entries_per_s / per_round_65k, "unit": "node-rounds/s", "cores": 1,
            "kind": "port",
            "sample": "oracle/scale_oracle.c, n=4096 full view, %d ticks in %.1f s (%.3g entries/s), "
                      "scaled to 65,536-wide rows" % (ticks, el, entries_per_s)}


PV_NODES = 1 << 20
PV_KW = dict(view=256, fanout=3, inbox=7, drop_pct=10, fail_mode=2, fail_tick=10, fail_ppm=50000,
             seed=SEED)


def pview_cpu_baseline(budget_s=10.0):
    """oracle/pview_oracle.c (1 thread) on n = 5000 with config 5's V, fanout, inbox, drops
    and failure rule: per-node work does not depend on n in a bounded view."""
    from tests.oracle_binding import PviewOracle
    o = PviewOracle(5000, **PV_KW)
    t0 = time.perf_counter()
    ticks = rounds = 0
    while time.perf_counter() - t0 < budget_s and ticks < 40:
        rounds += o.step()["node_rounds"]
        ticks += 1
    el = time.perf_counter() - t0
    o.close()
    return {"value": rounds / el, "unit": "node-rounds/s", "cores": 1, "kind": "port",
            "sample": "oracle/pview_oracle.c, n=5000, V=256, %d ticks in %.1f s" % (ticks, el)}


def run_pview(nodes, steps, warmup, world, local, dist, cpu_baseline_on, group=1):
    """Config 5 on `world` GPUs (row shards).  Returns the rank-0 summary (None elsewhere).
    Algorithmic bytes per node-round: own view read + write (2 * V * 8) + one sender view per
    merged message (V * 8) + 4 B per CSR entry."""
    import torch
    from gossip_protocol_amd.pview import PviewEngine
    kw = dict(PV_KW, max_ticks=warmup + steps)
    if dist is not None:
        from gossip_protocol_amd.dist import make_pview_rank_engine
        eng = make_pview_rank_engine(nodes, local, **kw)
    else:
        eng = PviewEngine(nodes, device=local, group=group, **kw)
    eng.step(warmup)
    eng.sync()
    p0 = eng.perf()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step(steps)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    eng.sync()
    p1 = eng.perf()
    rounds = delivered = merges = csr = 0
    for t in range(warmup + 1, warmup + steps + 1):
        d = eng.digest(t)
        rounds += d["node_rounds"]
        delivered += d["delivered"]
        merges += d["merges"]
        csr += d["delivered"] + d["overflow"]
    V = PV_KW["view"]
    launches = max(p1["merge_launches"] - p0["merge_launches"], 1)
    kern_ms = (p1["merge_ms"] - p0["merge_ms"]) / launches
    xch_ms = (p1["csr_ms"] - p0["csr_ms"]) / launches
    bytes_per_launch = ((2.0 * rounds + delivered) * V * 8.0 + csr * 4.0) / steps
    xgmi = (p1["xgmi_bytes"] - p0["xgmi_bytes"]) / steps
    eng.close()
    if dist is not None:
        t = torch.tensor([el, kern_ms, xch_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        u = torch.tensor([rounds, merges, bytes_per_launch, xgmi], dtype=torch.float64,
                         device="cuda")
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        el, kern_ms, xch_ms = (x.item() for x in t)
        rounds, merges, bytes_per_launch, xgmi = (x.item() for x in u)
        if dist.get_rank() != 0:
            return None
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    peak = PEAK_HBM_GBS * world
    out = {
        "metric": "gossip node-rounds/sec (partial view)", "value": rounds / el,
        "unit": "node-rounds/s", "ms_per_step": el * 1e3 / steps, "scaling": "strong",
        "dtype": "u64 entries (id:32 | hb:11 | ts:5)",
        "config": {"workload": "config5: %d nodes, partial view V=256, fanout 3, inbox 7, 10%% "
                               "drop, 5%% contiguous crash at t=10" % nodes,
                   "parallelism": ("rows%d" % world if world > 1 else
                                   "rows%d-in-process" % group if group > 1 else "1gpu")},
        "merges_per_s": merges / el,
        "xgmi_bytes_per_tick": xgmi, "exchange_csr_ms": xch_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": None, "kernel": "pview_tick_kernel",
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": bytes_per_launch},
    }
    if world == 1 and cpu_baseline_on:
        out["cpu_baseline"] = pview_cpu_baseline()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nodes", type=int, default=N_NODES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pview", action="store_true", help="skip the config-5 line item")
    ap.add_argument("--pview-nodes", type=int, default=PV_NODES)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine

    if world > 1:
        # column shards: the same config-3 workload split N ways (strong scaling)
        from gossip_protocol_amd.dist import make_rank_engine
        eng = make_rank_engine(args.nodes, local, fanout=FANOUT, fail_mode=FAIL_RANDOM,
                               fail_tick=FAIL_TICK, fail_ppm=FAIL_PPM, seed=SEED,
                               max_ticks=args.warmup + args.steps)
    else:
        eng = ScaleEngine(args.nodes, fanout=FANOUT, fail_mode=FAIL_RANDOM, fail_tick=FAIL_TICK,
                          fail_ppm=FAIL_PPM, seed=SEED, max_ticks=args.warmup + args.steps,
                          device=local)

    def barrier():
        if dist is not None:
            dist.barrier()

    eng.step(args.warmup)
    eng.sync()
    perf0 = eng.perf()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step(args.steps)
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    eng.sync()
    perf1 = eng.perf()
    xgmi_tick = (perf1["xgmi_bytes"] - perf0["xgmi_bytes"]) / args.steps

    rounds = merges = delivered = 0
    for t in range(args.warmup + 1, args.warmup + args.steps + 1):
        d = eng.digest(t)
        rounds += d["node_rounds"]
        merges += d["merges"]
        delivered += d["delivered"]
    if dist is not None:
        # every rank streams its slice of every processed row and of every sender row
        tot = torch.tensor([rounds, delivered], dtype=torch.float64, device="cuda")
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        rows_all, delivered_all = tot[0].item(), tot[1].item()
    else:
        rows_all, delivered_all = rounds, delivered
    stride = eng.layout()[2]
    launches = perf1["merge_launches"] - perf0["merge_launches"]
    kern_ms = (perf1["merge_ms"] - perf0["merge_ms"]) / max(launches, 1)
    csr_ms = (perf1["csr_ms"] - perf0["csr_ms"]) / max(launches, 1)
    # algorithmic bytes per launch: own row read + write, one sender row per message
    # (2-byte entries), one 4-byte CSR entry per message
    # per shard: its slice (stride columns) of every processed and every sender row; the
    # job moves `world` slices (row counts are kept by rank 0 only, so rows_all = job total)
    bytes_per_launch = ((2.0 * rows_all + delivered_all) * stride * 2.0 +
                        delivered_all * 4.0) * world / args.steps

    if dist is not None:
        # per-row counts live on rank 0 only (sum = job total); each rank moves its own
        # slice's bytes (sum); the step time and kernel time are the slowest rank's (max)
        t = torch.tensor([el, rounds, merges, bytes_per_launch, kern_ms], dtype=torch.float64,
                         device="cuda")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        el = tmax[0].item()
        rounds, merges = tsum[1].item(), tsum[2].item()
        kern_ms = tmax[4].item()
        x = torch.tensor([xgmi_tick], dtype=torch.float64, device="cuda")
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
        xgmi_tick = x.item()
    eng.close()
    pv = None
    if not args.no_pview:
        pv = run_pview(args.pview_nodes, min(args.steps, 30), args.warmup, world, local, dist,
                       not args.no_cpu_baseline)

    if rank == 0:
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9     # summed over ranks
        peak = PEAK_HBM_GBS * world
        traffic = None
        prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(prof):
            try:
                traffic = json.load(open(prof)).get("bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": "gossip node-rounds/sec (+ merge-kernel HBM GB/s, % peak)",
            "value": rounds / el,
            "unit": "node-rounds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic (pre-joined full-view membership, Philox peers/failures)",
            "config": {"workload": "config3: %d nodes full view, fanout %d, 1%% random crash at "
                                   "t=%d, no drops" % (args.nodes, FANOUT, FAIL_TICK),
                       "nodes": args.nodes, "view": args.nodes, "fanout": FANOUT,
                       "entry_bytes": 2,
                       "parallelism": "columns%d" % world if world > 1 else "1gpu"},
            "merges_per_s": merges / el,
            "xgmi_bytes_per_tick": xgmi_tick,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak,
                         "unit": "GB/s", "frac": achieved / peak, "traffic": traffic,
                         "kernel": "scale_tick_kernel", "kernel_ms": kern_ms,
                         "csr_ms": csr_ms, "algorithmic_bytes_per_launch": bytes_per_launch},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        if pv is not None:
            out["pview"] = pv
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
