#!/usr/bin/env python3
"""Headline benchmark: gossip node-rounds/s on the SCALE engine (BASELINE.json configs 3-5).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-pview] [--no-cpu-baseline]

One "step" = one protocol tick over the whole node population: every alive node merges
the rows gossiped to it, bumps its heartbeat, runs the TREMOVE scan and gossips to `fanout`
peers (the reference's nodeLoop, /root/reference/MP1Node.cpp:176-362, at scale).

Headline (`value`, `roofline`): BASELINE config 3 -- 65,536 nodes, full view (65,536 x
65,536 packed u16 table), fanout 3, 1% random crash at t = 10, no drops; ticks 1..W warm up,
W+1..W+K timed, with the device event stream on (every join / remove recorded: the
reference's Log lines, Log.cpp:116-130; the events-off run is reported beside it in
`events_off`).  N > 1: the same workload (strong scaling), column-sharded over N GPUs, one
process per GPU; the engine exchanges per-row counts and peer choices over its own RCCL
communicator, torch.distributed only carries the RCCL id, the barrier and the timing
reductions (DESIGN.md "Multi-GPU").
Second line item (`pview`): BASELINE config 5 -- 1,048,576 nodes, bounded partial view
V = 256, fanout 3, every delivered message merged (inbox 0, as the reference's checkMessages
drains its queue, MP1Node.cpp:200-212), 10% drops, 5% contiguous crash at t = 10; N > 1:
row-sharded over N GPUs with the per-tick sender-view exchange over RCCL send/recv (strong
scaling); reports its own node-rounds/s, tick-kernel roofline, the drain row classes' rows,
messages and kernel time (`drain_classes`), xGMI bytes per tick and the share of removals
that hit live nodes (removes_of_live_frac, from the event run).  `pview_inbox7`: the same
workload with the bounded inbox (at most 7 messages merged per receiver and tick; the share
of delivered messages it discards is inbox_overflow_frac).  `pview_swim`: the drain-all
workload with SWIM probing and TFAIL (detection latency of the t = 10 crashes, removals of live
members, kernel time against the plain run).
Prints ONE JSON line (rank 0) with the roofline of the fused tick kernel and the CPU
baseline (the oracle restatement, timed on a bounded sample of the same workload).
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0       # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
N_NODES = 65536
FANOUT = 3
FAIL_PPM = 10000            # 1 %
FAIL_TICK = 10
SEED = 0x5EED


# xgmi_bytes_per_tick is accounted, not measured: the bytes the library hands to RCCL
# (send/recv, all-gather, all-reduce) per tick, summed over ranks -- no link counter is read
XGMI_SOURCE = "accounted: bytes passed to RCCL calls per tick (not a link counter)"


def host_cpu():
    """CPU model and core counts of this host (the CPU baseline runs on one of them)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "cpus_usable": usable}


REF_APP = os.path.join(ROOT, "oracle", "_ref", "Application")
REF_CONFS = {"singlefailure": (1, 0), "multifailure": (0, 0), "msgdropsinglefailure": (1, 1)}


def ref_node_rounds(dbg, n=10, ticks=700):
    """nodeLoop calls of one reference run (Application.cpp:153-155): node i runs at tick t iff
    t > 0.25 i (double compare) and it has not failed; the failed nodes (Application::fail at
    t = 100, Application.cpp:173-202) are read back from the run's dbg.log lines."""
    failed = set()
    for line in dbg.decode(errors="replace").split("\n"):
        if "Node failed at time" in line:
            failed.add(int(line.split()[0].split(".")[0]) & 0xFF)
    rounds = 0
    for i in range(n):
        active = sum(1 for t in range(ticks) if t > 0.25 * i)
        rounds += active - (ticks - 1 - 100 if (i + 1) in failed else 0)
    return rounds


def reference_cpu_baseline(budget_s=8.0):
    """The REFERENCE itself as the CPU baseline: oracle/_ref/Application -- the unmodified
    /root/reference sources built by oracle/Makefile with the reference's own flags (-g, i.e.
    -O0, Makefile:10) plus a time() pin for the seed -- run single-threaded on this host over
    its three testcases (N = 10, 700 ticks, Application.cpp:90-114) for ~budget_s seconds.
    node-rounds/s = nodeLoop calls / whole-process wall time (constructor and msgcount.log
    included; the reference cannot run the GPU configs: MAX_NODES = 1000, EmulNet.h:10)."""
    import shutil
    import subprocess
    import tempfile
    if not os.path.exists(REF_APP):
        return None
    src = os.path.join(ROOT, "tests", "golden", "ref", "testcases")
    rounds = runs = merges = 0
    wall = 0.0
    try:                    # merges of each run from the pinned restatement (same seed, glibc)
        from tests.oracle_binding import load_oracle, run_oracle_mp1
        load_oracle()
    except Exception:       # noqa: BLE001 -- the oracle library is optional here
        run_oracle_mp1 = None
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "testcases"))
        for c in REF_CONFS:
            shutil.copy(os.path.join(src, c + ".conf"), os.path.join(tmp, "testcases"))
        seed = 1
        t_end = time.perf_counter() + budget_s
        while time.perf_counter() < t_end:
            for c in REF_CONFS:
                env = dict(os.environ, GSP_SEED=str(seed))
                a = time.perf_counter()
                subprocess.run([REF_APP, "testcases/%s.conf" % c], cwd=tmp, env=env, check=True,
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                wall += time.perf_counter() - a
                with open(os.path.join(tmp, "dbg.log"), "rb") as f:
                    rounds += ref_node_rounds(f.read())
                if run_oracle_mp1 is not None:
                    run_oracle_mp1(c, seed, "glibc", os.path.join(tmp, "oracle"))
                    merges += load_oracle().gsp_oracle_mp1_merges()
                runs += 1
            seed += 1
    out = {"value": rounds / wall, "unit": "node-rounds/s", "cores": 1, "kind": "reference",
           "merges_per_s": merges / wall if merges else None,
           "sample": "oracle/_ref/Application (the reference, -O0 as its Makefile builds it), "
                     "%d runs of its 3 testcases (N = 10, 700 ticks, seeds 1..%d), %d node-rounds "
                     "in %.2f s of whole-process wall time, 1 thread" % (runs, seed - 1, rounds, wall)}
    out.update(host_cpu())
    return out


def cpu_baseline(budget_s=12.0):
    """Oracle restatement (oracle/scale_oracle.c, 1 thread) on a bounded sample.

    The full 65,536-wide table does not fit a CPU run of seconds, so the sample is the same
    protocol at n = 4096 (full view, fanout 3, 1% crash at t = 10); its throughput in table
    entries processed per second is converted to node-rounds/s of the 65,536-wide workload
    (a node-round there processes 65,536 x (1 + k) entries, k = messages merged).
    """
    from tests.oracle_binding import ScaleOracle, load_oracle
    load_oracle().gsp_oracle_set_threads(1)        # the single-threaded restatement
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
PV_KW = dict(view=256, fanout=3, inbox=0, drop_pct=10, fail_mode=2, fail_tick=10, fail_ppm=50000,
             seed=SEED)
DRAIN_CLASSES = ["lds0 (192 lanes, <= 3,072 tuples)", "lds1 (256, 4,096)", "lds2 (512, 8,192)",
                 "lds3 (1,024, 16,384)", "hub (1,024 lanes, HBM buffers)"]


def pview_cpu_baseline(budget_s=10.0, inbox=0):
    """oracle/pview_oracle.c (1 thread) on n = 5000 with config 5's V, fanout, inbox, drops
    and failure rule: per-node work does not depend on n in a bounded view."""
    from tests.oracle_binding import PviewOracle
    o = PviewOracle(5000, **dict(PV_KW, inbox=inbox))
    t0 = time.perf_counter()
    ticks = rounds = 0
    while time.perf_counter() - t0 < budget_s and ticks < 40:
        rounds += o.step()["node_rounds"]
        ticks += 1
    el = time.perf_counter() - t0
    o.close()
    return {"value": rounds / el, "unit": "node-rounds/s", "cores": 1, "kind": "port",
            "sample": "oracle/pview_oracle.c, n=5000, V=256, inbox %d, %d ticks in %.1f s" %
                      (inbox, ticks, el)}


def run_pview(nodes, steps, warmup, world, local, dist, cpu_baseline_on, group=1, events=0,
              inbox=None, extra=None):
    """Config 5 on `world` GPUs (row shards).  Returns the rank-0 summary (None elsewhere).
    Algorithmic bytes per node-round: own view read + write (2 * V * 8) + one sender view per
    merged message (V * 8) + 4 B per CSR entry.  events: a kind mask (gsp_pview_params.events);
    the summary is then the event one (event_summary) with the kernel time.  inbox: 0 runs the
    drain-all protocol (every message merged, gsp_pview_params.inbox = 0).  extra: more
    gsp_pview_params fields (the protocol variants: tfail, swim)."""
    import torch
    from gossip_protocol_amd.pview import PviewEngine
    kw = dict(PV_KW, max_ticks=warmup + steps)
    if inbox is not None:
        kw["inbox"] = inbox
    kw.update(extra or {})
    if events:
        kw.update(events=events, event_cap=EVENT_CAP)
    if dist is not None:
        from gossip_protocol_amd.dist import make_pview_rank_engine
        eng = make_pview_rank_engine(nodes, local, **kw)
    else:
        eng = PviewEngine(nodes, device=local, group=group, **kw)
    eng.step(warmup)
    eng.sync()
    if events:
        eng.drain_events()
    p0 = eng.perf()
    d0 = eng.drain_stats() if kw["inbox"] == 0 else None
    if dist is not None:
        dist.barrier()
    _sync()
    t0 = time.perf_counter()
    eng.step(steps)
    _sync()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    eng.sync()
    p1 = eng.perf()
    d1 = eng.drain_stats() if kw["inbox"] == 0 else None
    rounds = delivered = merges = csr = overflow = 0
    for t in range(warmup + 1, warmup + steps + 1):
        d = eng.digest(t)
        rounds += d["node_rounds"]
        delivered += d["delivered"]
        merges += d["merges"]
        overflow += d["overflow"]
        csr += d["delivered"] + d["overflow"]
    V = PV_KW["view"]
    launches = max(p1["merge_launches"] - p0["merge_launches"], 1)
    kern_ms = (p1["merge_ms"] - p0["merge_ms"]) / launches
    xch_ms = (p1["csr_ms"] - p0["csr_ms"]) / launches
    bytes_per_tick = ((2.0 * rounds + delivered) * V * 8.0 + csr * 4.0) / steps
    xgmi = (p1["xgmi_bytes"] - p0["xgmi_bytes"]) / steps
    classes = None
    if d0 is not None:
        # per drain class and tick: rows, messages merged, kernel ms and its algorithmic GB/s
        # (own view read + write and one sender view per message)
        classes = []
        for c, name in enumerate(DRAIN_CLASSES):
            rows_c = (d1["rows"][c] - d0["rows"][c]) / steps
            msgs_c = (d1["messages"][c] - d0["messages"][c]) / steps
            ms_c = (d1["ms"][c] - d0["ms"][c]) / steps
            b = (2.0 * rows_c + msgs_c) * V * 8.0
            classes.append({"class": name, "rows_per_tick": rows_c, "messages_per_tick": msgs_c,
                            "kernel_ms_per_tick": ms_c,
                            "achieved_gbs": b / (ms_c * 1e-3) / 1e9 if ms_c > 0 else None})
    ev = None
    if events:
        from gossip_protocol_amd import _lib
        ev = event_summary(eng, nodes, warmup + steps, dist,
                           _lib.fail_schedule(nodes, PV_KW["seed"], PV_KW["fail_mode"],
                                              PV_KW["fail_tick"], PV_KW["fail_ppm"]))
    eng.close()
    if dist is not None:
        t = torch.tensor([el, kern_ms, xch_ms], dtype=torch.float64, device=_dev())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        u = torch.tensor([rounds, merges, bytes_per_tick, xgmi, overflow, csr],
                         dtype=torch.float64, device=_dev())
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        el, kern_ms, xch_ms = (x.item() for x in t)
        rounds, merges, bytes_per_tick, xgmi, overflow, csr = (x.item() for x in u)
        if dist.get_rank() != 0:
            return None
    if events:
        ev.update({"kinds": events, "kernel_ms": kern_ms, "value_events_on": rounds / el})
        return ev
    achieved = bytes_per_tick / (kern_ms * 1e-3) / 1e9
    peak = PEAK_HBM_GBS * world
    window = [warmup + 1, warmup + steps]
    k_in = kw["inbox"]
    traffic, traffic_note = _pview_traffic(nodes, world, window, k_in)
    out = {
        "metric": "gossip node-rounds/sec (partial view)", "value": rounds / el,
        "unit": "node-rounds/s", "ms_per_step": el * 1e3 / steps, "scaling": "strong",
        "dtype": "u64 entries (id:32 | hb:11 | ts:5)",
        "config": {"workload": "config5: %d nodes, partial view V=256, fanout 3, %s, 10%% "
                               "drop, 5%% contiguous crash at t=10" %
                               (nodes, "inbox %d" % k_in if k_in else "inbox 0 (drain all)"),
                   "inbox": k_in,
                   "parallelism": ("rows%d" % world if world > 1 else
                                   "rows%d-in-process" % group if group > 1 else "1gpu")},
        "merges_per_s": merges / el,
        # the share of delivered messages the bounded inbox discards (0 when draining all)
        "inbox_overflow_frac": overflow / csr if csr else 0.0,
        "xgmi_bytes_per_tick": xgmi, "xgmi_bytes_source": XGMI_SOURCE, "exchange_csr_ms": xch_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "kernel": ("pview_tick_split_kernel (256- and 128-lane rows, per tick)" if k_in else
                                "pview_tick_split_kernel + pview_drain_{lds,hbm}_kernel (rows sent > 7 "
                                "messages), per tick"),
                     "valu": _pview_valu(nodes, world, kern_ms, window, k_in),
                     "window_ticks": window,
                     "kernel_ms_per_tick": kern_ms, "algorithmic_bytes_per_tick": bytes_per_tick},
    }
    if traffic_note:
        out["roofline"]["traffic_note"] = traffic_note
    if classes is not None:
        out["drain_classes"] = classes
    if world == 1 and cpu_baseline_on:
        out["cpu_baseline"] = pview_cpu_baseline(inbox=k_in)
    return out


def _pmc(name, window):
    """A committed PMC summary (profiles/<name>) if it was taken over exactly this run's tick
    window, else (None, the window it covers).  Counter-derived fields are printed only for the
    window they were measured on: the counts of ticks 6-25 say nothing
    about, and must not be divided by the kernel time of, any other window."""
    prof = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(prof):
        return None, None
    try:
        d = json.load(open(prof))
    except Exception:
        return None, None
    w = d.get("window_ticks")
    if w is None or list(w) != list(window):
        return None, w
    return d, w


def _window_note(name, have, window):
    return ("null: profiles/%s covers ticks %d-%d, this run timed ticks %d-%d" %
            (name, have[0], have[1], window[0], window[1])) if have else None


def _pv_pmc_name(kind, inbox):
    """profiles/pmc_<kind>_pview.json: the drain-all run (inbox 0, the headline);
    pmc_<kind>_pview_inbox7.json: the bounded-inbox run."""
    return "pmc_%s_pview%s.json" % (kind, "" if inbox == 0 else "_inbox%d" % inbox)


def _pview_traffic(nodes, world, window, inbox):
    """HBM bytes per tick from the committed PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
    scripts/pmc_traffic.py --pview) for the one-GPU config-5 run of this inbox over the same
    tick window, else (None, note)."""
    if nodes != PV_NODES or world != 1:
        return None, None
    name = _pv_pmc_name("traffic", inbox)
    d, w = _pmc(name, window)
    if d is None:
        return None, _window_note(name, w, window)
    return d.get("bytes_per_launch"), None


def _pview_valu(nodes, world, kern_ms, window, inbox):
    """The tick kernel's actual limiter: VALU issue.  SQ_INSTS_VALU per tick from the committed
    PMC pass over the same tick window (profiles/pmc_sq_pview*.json) over the live mean kernel
    time: wave64 VALU instructions issued per SIMD cycle (1,024 SIMDs at 2.4 GHz), and that rate
    against the SIMD's issue ceiling -- one wave64 VALU instruction per 2 cycles with two or more
    waves resident (MI355X_MICROARCH.md, "Wave scheduling" and the v_fma_f32 row of the
    constants table; 4 cycles is one wave alone); config 5, one GPU."""
    if nodes != PV_NODES or world != 1:
        return None
    name = _pv_pmc_name("sq", inbox)
    d, w = _pmc(name, window)
    if d is None:
        note = _window_note(name, w, window)
        return {"note": note} if note else None
    try:
        insts = d["counters"]["SQ_INSTS_VALU"]["per_launch"]
        salu = d["counters"].get("SQ_INSTS_SALU", {}).get("per_launch")
    except Exception:
        return None
    per_cycle = insts / (1024 * 2.4e9 * kern_ms * 1e-3)
    return {"bound": "valu-issue", "insts_per_launch": insts, "salu_insts_per_launch": salu,
            "insts_per_simd_cycle": per_cycle, "frac_of_2cycle_issue": per_cycle * 2.0,
            "clock_ghz": 2.4, "window_ticks": w}


EVENT_CAP = 1 << 27          # records per shard (1 GB): config 3 records 70.7 M joins + removes
TILE_COLS = 8192             # column tiles of 8,192 columns: config 3 as 8 tiles on one GPU
                             # (DESIGN.md "Column tiles": 6.6 vs 8.0 ms per tick for the fused
                             # row kernel), config 4 as 32


def tiles_for(nodes, world):
    """Column tiles per rank: 8,192-column tiles when the job splits into them evenly."""
    total = nodes // TILE_COLS
    if nodes % (2048 * max(total, 1)) != 0 or total < world or total % world != 0 \
            or total > 64:
        return 1
    return total // world


def run_full(nodes, steps, warmup, world, local, dist, layout="columns", events=False, tiles=None):
    """Full-view workload (config 3 rules) on `world` GPUs: one GPU fused, or column / row
    shards.  Returns job totals (time and kernel time are the slowest rank's).  events: the
    tick kernels also append every join / remove record to the device ring (drained after
    the timed region; event_summary)."""
    import torch
    from gossip_protocol_amd.scale import FAIL_RANDOM, ScaleEngine
    kw = dict(fanout=FANOUT, fail_mode=FAIL_RANDOM, fail_tick=FAIL_TICK, fail_ppm=FAIL_PPM,
              seed=SEED, max_ticks=warmup + steps, layout=layout)
    if events:
        kw.update(events=True, event_cap=EVENT_CAP)
    if dist is not None:
        from gossip_protocol_amd.dist import make_rank_engine
        if tiles is None:     # 8192-column tiles per rank when the slices are wider
            tiles = tiles_for(nodes, world) if layout == "columns" else 1
        if tiles > 1:
            kw["tiles"] = tiles
        eng = make_rank_engine(nodes, local, **kw)
    else:
        if tiles is None:
            tiles = tiles_for(nodes, 1)
        eng = ScaleEngine(nodes, device=local, group=tiles, **kw)
    eng.step(warmup)
    eng.sync()
    if events:
        eng.drain_events()                # the warm-up ticks' records (none: crash at t = 10)
    perf0 = eng.perf()
    if dist is not None:
        dist.barrier()
    _sync()
    t0 = time.perf_counter()
    eng.step(steps)
    _sync()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    eng.sync()
    perf1 = eng.perf()
    xgmi_tick = (perf1["xgmi_bytes"] - perf0["xgmi_bytes"]) / steps
    rounds = merges = delivered = 0
    for t in range(warmup + 1, warmup + steps + 1):
        d = eng.digest(t)
        rounds += d["node_rounds"]
        merges += d["merges"]
        delivered += d["delivered"]
    shards_total, _, stride = eng.layout()
    launches = max(perf1["merge_launches"] - perf0["merge_launches"], 1)
    kern_ms = (perf1["merge_ms"] - perf0["merge_ms"]) / launches
    csr_ms = (perf1["csr_ms"] - perf0["csr_ms"]) / launches
    ev = None
    if events:
        from gossip_protocol_amd import _lib
        ev = event_summary(eng, nodes, warmup + steps, dist,
                           _lib.fail_schedule(nodes, SEED, FAIL_RANDOM, FAIL_TICK, FAIL_PPM))
    eng.close()
    if dist is not None:
        # per-row counts live on rank 0 only (columns) or on the row's owner (rows): the sum is
        # the job total; the step and kernel times are the slowest rank's (max); every rank
        # sends its own exchange bytes (sum)
        u = torch.tensor([rounds, merges, delivered, xgmi_tick], dtype=torch.float64,
                         device=_dev())
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        rounds, merges, delivered, xgmi_tick = (x.item() for x in u)
        m = torch.tensor([el, kern_ms, csr_ms], dtype=torch.float64, device=_dev())
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        el, kern_ms, csr_ms = (x.item() for x in m)
    # algorithmic bytes per tick (all tile launches): own row read + write and one sender row per message
    # (2-byte entries), one 4-byte CSR entry per message; column shards stream their slice
    # (stride columns) of each such row, so the job moves `world` slices; row shards stream
    # whole rows (stride = full width) of their own receivers only
    slices = shards_total if layout == "columns" else 1
    bytes_per_tick = ((2.0 * rounds + delivered) * stride * 2.0 + delivered * 4.0) * slices / steps
    return {"el": el, "rounds": rounds, "merges": merges, "kern_ms": kern_ms, "csr_ms": csr_ms,
            "bytes_per_tick": bytes_per_tick, "xgmi_tick": xgmi_tick, "layout": layout,
            "events": ev, "tiles": shards_total // (world if dist is not None else 1)}


def event_summary(eng, nodes, last_tick, dist, crash):
    """Failure detection read from the drained event stream.  crash: every node's crash tick
    (gsp_fail_schedule; int32 max = never).  For each node that crashed before the last tick,
    the first and the last removal of it after its crash (the last = every live node that
    listed it has removed it) minus its crash tick; removals of nodes that never crashed are
    counted apart (none in the full view without drops; a partial view's churn).  The reference
    logs the same removals as "Node x removed at time t" (MP1Node.cpp:343, Log.cpp:127-130) and
    its grader scores detection from them (Grader.sh).  Ranks combine per-node first / last /
    count."""
    import numpy as np
    import torch
    from gossip_protocol_amd import _lib
    rec, lost = eng.drain_events()
    kind, tk, _, x = _lib.split_events(rec)
    rem = kind == _lib.EVENT_REMOVE
    xr, tr = x[rem].astype(np.int64), tk[rem].astype(np.int64)
    crash = np.asarray(crash, np.int64)
    after = tr > crash[xr]                    # removals of x after its crash
    live_removes = int((crash[xr] >= last_tick).sum())
    xa, ta = xr[after], tr[after]
    first = np.full(nodes, 1 << 30, np.int64)
    last = np.full(nodes, -1, np.int64)
    for t in np.unique(ta)[::-1]:             # descending: the earliest tick is written last
        first[xa[ta == t]] = t
    for t in np.unique(ta):
        last[xa[ta == t]] = t
    count = np.bincount(xa, minlength=nodes).astype(np.int64)
    joins = int((kind == _lib.EVENT_JOIN).sum())
    n_rec, n_rem = len(rec), int(rem.sum())
    if dist is not None:
        f = torch.from_numpy(first).to(_dev())
        l_ = torch.from_numpy(last).to(_dev())
        c = torch.from_numpy(count).to(_dev())
        tot = torch.tensor([n_rec, lost, joins, live_removes, n_rem], dtype=torch.int64,
                           device=_dev())
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        dist.all_reduce(l_, op=dist.ReduceOp.MAX)
        dist.all_reduce(c)
        dist.all_reduce(tot)
        first, last, count = f.cpu().numpy(), l_.cpu().numpy(), c.cpu().numpy()
        n_rec, lost, joins, live_removes, n_rem = (int(v) for v in tot.tolist())
    crashed = crash < last_tick
    det = crashed & (count > 0)
    stat = lambda a: {"min": int(a.min()), "mean": float(a.mean()), "max": int(a.max())} \
        if len(a) else None
    return {"records": n_rec, "lost": int(lost), "joins": joins,
            "removes": n_rem, "last_tick": last_tick,
            "crashed_nodes": int(crashed.sum()), "crashed_nodes_detected": int(det.sum()),
            "removes_per_detected_node": float(count[det].mean()) if det.any() else 0.0,
            "removes_of_live_nodes": live_removes,
            "first_detection_latency_ticks": stat((first - crash)[det]),
            "full_detection_latency_ticks": stat((last - crash)[det])}


def summarize_full(r, nodes, steps, world, warmup):
    achieved = r["bytes_per_tick"] / (r["kern_ms"] * 1e-3) / 1e9     # summed over ranks
    peak = PEAK_HBM_GBS * world
    traffic = traffic_note = None
    window = [warmup + 1, warmup + steps]
    if nodes == N_NODES and world == 1:
        t, w = _pmc("pmc_traffic.json", window)
        if t is not None and t.get("launches_per_tick", 1) == r["tiles"]:
            traffic = t.get("bytes_per_tick", t.get("bytes_per_launch"))
        elif t is None:
            traffic_note = _window_note("pmc_traffic.json", w, window)
    cfg = "config3" if nodes == N_NODES else "config4" if nodes == 262144 else "full view"
    return {
        "metric": "gossip node-rounds/sec (+ merge-kernel HBM GB/s, % peak)",
        "value": r["rounds"] / r["el"], "unit": "node-rounds/s",
        "ms_per_step": r["el"] * 1e3 / steps, "scaling": "strong", "dtype": "u16",
        "data": "synthetic (pre-joined full-view membership, Philox peers/failures)",
        "config": {"workload": "%s: %d nodes full view, fanout %d, 1%% random crash at t=%d, "
                               "no drops" % (cfg, nodes, FANOUT, FAIL_TICK),
                   "nodes": nodes, "view": nodes, "fanout": FANOUT, "entry_bytes": 2,
                   "parallelism": ("%s%d" % (r["layout"], world) +
                                   ("" if r["tiles"] == 1 else "-%dtiles" % r["tiles"])) if world > 1 else
                   "1gpu" if r["tiles"] == 1 else "1gpu-%dtiles" % r["tiles"]},
        "merges_per_s": r["merges"] / r["el"],
        "xgmi_bytes_per_tick": r["xgmi_tick"], "xgmi_bytes_source": XGMI_SOURCE,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": traffic, "window_ticks": window,
                     **({"traffic_note": traffic_note} if traffic_note else {}),
                     "kernel": "scale_tick_kernel",
                     "kernel_ms_per_tick": r["kern_ms"], "launches_per_tick": r["tiles"],
                     "kernel_ms_per_launch": r["kern_ms"] / r["tiles"],
                     ("exchange_csr_ms" if r["layout"] == "rows" else "csr_ms"): r["csr_ms"],
                     "algorithmic_bytes_per_tick": r["bytes_per_tick"]},
    }


def _sync():
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _dev():
    """Device of the timing reductions: the GPU (RCCL) or, for the gloo CPU tests, the host."""
    import torch
    return "cuda" if torch.cuda.is_available() else "cpu"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nodes", type=int, default=N_NODES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pview", action="store_true", help="skip the config-5 line item")
    ap.add_argument("--pview-nodes", type=int, default=PV_NODES)
    ap.add_argument("--no-262k", action="store_true", help="skip the config-4 line item")
    ap.add_argument("--item-budget", type=int, default=420,
                    help="seconds for the secondary line items before the line is printed as is")
    ap.add_argument("--no-events", action="store_true",
                    help="the headline without the event stream, and no event-stream runs")
    ap.add_argument("--no-rows", action="store_true",
                    help="skip the full-view row-layout line items (N > 1)")
    ap.add_argument("--no-events-off", action="store_true",
                    help="skip the events-off run of the headline workload")
    ap.add_argument("--no-swim", action="store_true",
                    help="skip the SWIM + TFAIL config-5 line item")
    ap.add_argument("--no-inbox7", action="store_true",
                    help="skip the bounded-inbox config-5 line item (inbox 7)")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            torch.cuda.set_device(local)
            dist.init_process_group("nccl")
    # the headline records every join / remove on the device (the reference's Log lines)
    full = run_full(args.nodes, args.steps, args.warmup, world, local, dist,
                    events=not args.no_events)
    out = None
    if rank == 0:
        out = summarize_full(full, args.nodes, args.steps, world, args.warmup)
        out["event_stream"] = "on" if not args.no_events else "off"
        out.update({"n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                    "higher_is_better": True, "vs_baseline": None})
        if world == 1 and not args.no_cpu_baseline:
            # the reference itself (N = 10, the only size it runs), with our restatement of
            # the config-3 protocol beside it (scaled to 65,536-wide rows)
            port = cpu_baseline()
            ref = reference_cpu_baseline()
            out["cpu_baseline"] = ref if ref is not None else port
            if ref is not None:
                out["cpu_baseline"]["port"] = port

    # Secondary line items: an exception is recorded in the item (every rank sees the same
    # deterministic capacity / allocation errors); a hang or a one-rank failure that stalls
    # the others' collectives is cut by the watchdog, which prints the line as it stands.
    done = threading.Event()

    def _watchdog():
        if done.wait(args.item_budget):
            return
        if out is not None:
            out["incomplete"] = "secondary line items exceeded %d s" % args.item_budget
            print(json.dumps(out), flush=True)
        os._exit(0)
    threading.Thread(target=_watchdog, daemon=True).start()

    def item(key, fn, sub=None):
        try:
            res = fn()
        except Exception as e:          # noqa: BLE001 -- reported, not swallowed
            res = {"error": "%s: %s" % (type(e).__name__, e)}
        if out is not None and res is not None:
            if sub is None:
                out[key] = res
            else:
                out.setdefault(key, {})[sub] = res

    # the detection latency read from the headline's records, and the same workload with the
    # event stream off beside it: the kernel-time cost of recording
    if not args.no_events and out is not None:
        out["events"] = full["events"]
    def _events_off_item():
        r = run_full(args.nodes, args.steps, args.warmup, world, local, dist, events=False)
        if r is None or out is None:
            return None
        return {"value": r["rounds"] / r["el"], "ms_per_step": r["el"] * 1e3 / args.steps,
                "kernel_ms_per_tick": r["kern_ms"], "kernel_ms_events_on": full["kern_ms"],
                "events_on_overhead_frac": full["kern_ms"] / r["kern_ms"] - 1.0}
    if not args.no_events and not args.no_events_off:
        item("events_off", _events_off_item)
    if not args.no_pview:
        item("pview", lambda: run_pview(args.pview_nodes, min(args.steps, 30), args.warmup, world,
                                        local, dist, not args.no_cpu_baseline))
    def _pv_events(key, inbox=None):
        # the partial view records removes only: its joins and evictions are ~8e8 records per
        # tick at config 5 (6.7 GB, more than the tick's state traffic; scripts/events_cost.py).
        # removes_of_live_frac: the share of removals whose node never crashed -- churn of the
        # bounded view, not failure detection (the reference's grader fails any of them,
        # Grader.sh:69-76)
        r = run_pview(args.pview_nodes, min(args.steps, 30), args.warmup, world, local, dist,
                      False, events=4, inbox=inbox)
        if r is None:
            return None
        r["removes_of_live_frac"] = r["removes_of_live_nodes"] / r["removes"] if r["removes"] else 0.0
        if out is not None and isinstance(out.get(key), dict) and "roofline" in out[key]:
            k0 = out[key]["roofline"]["kernel_ms_per_tick"]
            r.update(kernel_ms_events_off=k0, kernel_overhead_frac=r["kernel_ms"] / k0 - 1.0)
            out[key]["removes_of_live_frac"] = r["removes_of_live_frac"]
        return r
    if not args.no_pview and not args.no_events:
        item("pview", lambda: _pv_events("pview"), "events")
    def _pv_swim():
        # config 5 drained with SWIM ping/ack probing (swim = 2: the direct ping and one
        # indirect ping-req path) and TFAIL = 5 (a member 5 ticks stale is not gossiped): the
        # crashes of t = 10 are found by probes within ticks instead of by TREMOVE at t = 30;
        # a probe that loses both paths to the 10 % drop removes a live member
        # (removes_of_live_frac).  Removal records on, as the pview events run.
        r = run_pview(args.pview_nodes, min(args.steps, 30), args.warmup, world, local, dist,
                      False, events=4, extra=dict(swim=2, tfail=5))
        if r is None:
            return None
        r["protocol"] = "swim=2, tfail=5, inbox 0 (drain all), removal records on"
        r["removes_of_live_frac"] = r["removes_of_live_nodes"] / r["removes"] if r["removes"] else 0.0
        pe = out.get("pview", {}).get("events") if out is not None else None
        if isinstance(pe, dict) and pe.get("kernel_ms"):
            r["kernel_ms_plain"] = pe["kernel_ms"]
            r["kernel_overhead_frac"] = r["kernel_ms"] / pe["kernel_ms"] - 1.0
        return r
    if not args.no_pview and not args.no_events and not args.no_swim:
        item("pview_swim", _pv_swim)
    if not args.no_pview and not args.no_inbox7:
        # config 5 with the bounded inbox (at most 7 messages merged per receiver and tick):
        # the protocol of rounds 1-5's headline, beside the drain-all one
        item("pview_inbox7", lambda: run_pview(args.pview_nodes, min(args.steps, 30), args.warmup,
                                               world, local, dist, False, inbox=7))
        if not args.no_events:
            item("pview_inbox7", lambda: _pv_events("pview_inbox7", inbox=7), "events")
    if not args.no_262k:
        # BASELINE config 4: 262,144 nodes full view, 8,192-column tiles: on one GPU 32 tiles
        # (the table pair is 2 x 128 GiB of the 288 GB HBM), at N > 1 32 / N tiles per rank
        item("full262k", lambda: summarize_full(
            run_full(262144, min(args.steps, 8), 2, world, local, dist), 262144,
            min(args.steps, 8), world, 2))
    if world > 1 and not args.no_rows:
        # the full view ROW-sharded (north star: sender rows cross shards over RCCL send/recv,
        # deduplicated per (sender, shard)); O(f n^2) xGMI bytes per tick against the column
        # layout's O(n), reported beside it (DESIGN.md "Multi-GPU")
        item("full_rows", lambda: summarize_full(
            run_full(args.nodes, min(args.steps, 8), 2, world, local, dist, layout="rows"),
            args.nodes, min(args.steps, 8), world, 2), "config3")
        if not args.no_262k:
            if world >= 4:
                item("full_rows", lambda: summarize_full(
                    run_full(262144, 4, 2, world, local, dist, layout="rows"), 262144, 4, world, 2),
                    "config4")
            else:
                # 2 x 68.7 GB of table rows plus ~2 x 66 GB of send/receive rows per GPU
                item("full_rows", lambda: {"skipped": "row layout at 262,144 nodes needs > 270 GB "
                                                      "per GPU at N = 2 (tables + exchange regions)"},
                     "config4")
    done.set()
    if out is not None:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
