"""bench.py's N > 1 path on CPU: two gloo ranks run bench.main() over stand-in engines.

The engines are replaced by deterministic fakes (the real ones need a GPU), so what runs is
bench.py's own multi-rank logic: barriers around the timed region, the max-over-ranks time
and kernel time, the job-total node-rounds / bytes / xGMI reductions, the three line items
(config 3 headline, config 5 `pview`, config 4 `full262k`, the row-layout `full_rows`) and the
single rank-0 JSON line.
"""
import io
import json
import os
import socket
import contextlib

import torch.distributed as dist
import torch.multiprocessing as mp

N_STEPS, N_WARM = 3, 1


class FakeEngine:
    """Per-tick digest: `rows` node-rounds on rank 0 (column shards count rows on shard 0),
    2 deliveries per round; kernel 2 ms (rank 0) / 3 ms (rank 1) per tick."""

    def __init__(self, n, rank, world, pview=False, rows=False):
        self.n, self.rank, self.world, self.pview, self.rows = n, rank, world, pview, rows
        self.t = 0

    def step(self, k):
        self.t += k

    def sync(self):
        pass

    def perf(self):
        ms = 2.0 + self.rank
        return {"merge_launches": self.t, "merge_ms": ms * self.t, "csr_ms": 0.5 * self.t,
                "xgmi_bytes": 1000.0 * (self.rank + 1) * self.t}

    def digest(self, t):
        if self.pview or self.rows:                  # row shards: every rank counts its rows
            rows = self.n // self.world
        else:
            rows = self.n if self.rank == 0 else 0
        return {"tick": t, "node_rounds": rows, "merges": 3 * rows, "delivered": 2 * rows,
                "overflow": 0}

    def drain_stats(self):
        """Drain all: per class, 10 rows of 12 messages a tick in 0.5 ms (hub: none)."""
        return {"rows": [10 * self.t] * 4 + [0], "messages": [120 * self.t] * 4 + [0],
                "ms": [0.5 * self.t] * 4 + [0.0]}

    def drain_events(self):
        """Removal records split over the ranks (kind 2 = remove, 1 = join): node 5 is removed
        at ticks 12, 13 (rank 0) and 11 (rank 1), node 7 at 30 (rank 0) and 31 (rank 1)."""
        import numpy as np
        rec = {0: [(2, 12, 0, 5), (2, 13, 1, 5), (2, 30, 2, 7)],
               1: [(2, 11, 600, 5), (2, 31, 601, 7), (1, 5, 600, 9)]}[self.rank]
        return np.array([(k << 62) | (t << 42) | (r << 21) | x for k, t, r, x in rec],
                        np.uint64), 0

    def layout(self):
        return (self.world, self.rank, self.n if self.rows else self.n // self.world)

    def close(self):
        pass


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gossip_protocol_amd.dist as gd
    gd.make_rank_engine = lambda n, dev, **kw: FakeEngine(n, rank, world,
                                                          rows=kw.get("layout") == "rows")
    gd.make_pview_rank_engine = lambda n, dev, **kw: FakeEngine(n, rank, world, pview=True)
    import numpy as np
    from gossip_protocol_amd import _lib

    def crash_ticks(n, *a, **k):                     # nodes 5 and 7 crash at t = 0
        c = np.full(n, np.iinfo(np.int32).max, np.int32)
        c[[5, 7]] = 0
        return c
    _lib.fail_schedule = crash_ticks
    import bench
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--steps", str(N_STEPS), "--warmup", str(N_WARM), "--nodes", "1024",
                    "--pview-nodes", "4096", "--no-cpu-baseline"])
    q.put((rank, buf.getvalue()))


def test_bench_two_ranks_gloo():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert outs[1].strip() == ""                      # only rank 0 prints
    lines = [l for l in outs[0].splitlines() if l.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == N_STEPS and d["warmup"] == N_WARM
    assert d["config"]["parallelism"] == "columns2"
    rf = d["roofline"]
    assert rf["kernel_ms_per_tick"] == 3.0                     # slowest rank
    assert rf["peak"] == 16000.0
    # job bytes per launch: (2 rows + 2 rows delivered) * stride(512) * 2 B + CSR, x 2 slices
    assert rf["algorithmic_bytes_per_tick"] == ((2 * 1024 + 2 * 1024) * 512 * 2 + 2 * 1024 * 4) * 2
    assert abs(d["value"] - 1024 * N_STEPS / (d["ms_per_step"] * N_STEPS / 1e3)) < 1e-6 * d["value"]
    assert d["xgmi_bytes_per_tick"] == 3000.0         # sum over ranks
    pv = d["pview"]
    assert pv["config"]["parallelism"] == "rows2"
    assert pv["xgmi_bytes_per_tick"] == 3000.0
    assert pv["roofline"]["kernel_ms_per_tick"] == 3.0
    assert abs(pv["value"] - 4096 * min(N_STEPS, 30) / (pv["ms_per_step"] * min(N_STEPS, 30) / 1e3)) \
        < 1e-6 * pv["value"]
    f = d["full262k"]
    assert f["config"]["nodes"] == 262144 and f["config"]["workload"].startswith("config4")
    fr = d["full_rows"]
    c3 = fr["config3"]
    assert c3["config"]["parallelism"] == "rows2"
    # row shards: whole rows (stride = n) of their own receivers, no slice factor
    assert c3["roofline"]["algorithmic_bytes_per_tick"] == \
        (2 * 512 + 2 * 512) * 2 * 1024 * 2 + 2 * 512 * 2 * 4
    assert abs(c3["value"] - 1024 * min(N_STEPS, 8) / (c3["ms_per_step"] * min(N_STEPS, 8) / 1e3)) \
        < 1e-6 * c3["value"]
    assert "skipped" in fr["config4"]                 # does not fit 2 GPUs
    ev = d["events"]                                  # per-node first / last over the ranks
    assert ev["records"] == 6 and ev["joins"] == 1 and ev["removes"] == 5 and ev["lost"] == 0
    assert ev["crashed_nodes_detected"] == 2 and ev["removes_per_detected_node"] == 2.5
    assert ev["crashed_nodes"] == 2 and ev["removes_of_live_nodes"] == 0
    assert ev["first_detection_latency_ticks"] == {"min": 11, "mean": 20.5, "max": 30}
    assert ev["full_detection_latency_ticks"] == {"min": 13, "mean": 22.0, "max": 31}
    assert d["event_stream"] == "on"                  # the headline records the events
    assert d["events_off"]["events_on_overhead_frac"] == 0.0
    dc = pv["drain_classes"]                          # drain all: per class and tick
    assert len(dc) == 5 and dc[0]["rows_per_tick"] == 10 and dc[0]["kernel_ms_per_tick"] == 0.5
    assert dc[4]["achieved_gbs"] is None and pv["config"]["inbox"] == 0
    p7 = d["pview_inbox7"]
    assert p7["config"]["parallelism"] == "rows2" and p7["config"]["inbox"] == 7
    assert "drain_classes" not in p7
    pe = pv["events"]                                 # the partial view's removes-only run
    assert "error" not in pe, pe
    assert pe["kinds"] == 4 and pe["crashed_nodes_detected"] == 2 and pe["kernel_overhead_frac"] == 0.0
    ps = d["pview_swim"]                              # SWIM + TFAIL drained, removal records
    assert "error" not in ps, ps
    assert ps["protocol"].startswith("swim=2, tfail=5") and ps["kernel_overhead_frac"] == 0.0
    assert ps["removes_of_live_frac"] == 0.0 and ps["crashed_nodes_detected"] == 2


INBOXES_WITH_PMC = [0, 7]       # committed profiles/pmc_*_pview*.json (0: drain all, 7: inbox 7)


def test_counter_fields_only_for_their_window():
    """Committed PMC summaries cover ticks 6-25 (the driver's --steps 20 --warmup 5): a run over
    that window prints them, any other window prints null with the window they belong to and
    no VALU fraction."""
    import bench
    for inbox in INBOXES_WITH_PMC:
        t, note = bench._pview_traffic(bench.PV_NODES, 1, [6, 25], inbox)
        assert t is not None and note is None
        t, note = bench._pview_traffic(bench.PV_NODES, 1, [6, 45], inbox)
        assert t is None and "ticks 6-25" in note and "ticks 6-45" in note
        v = bench._pview_valu(bench.PV_NODES, 1, 5.0, [6, 25], inbox)
        assert v["frac_of_2cycle_issue"] > 0 and v["window_ticks"] == [6, 25]
        v = bench._pview_valu(bench.PV_NODES, 1, 5.0, [6, 35], inbox)
        assert set(v) == {"note"}
    r = {"bytes_per_tick": 4.2e10, "kern_ms": 6.5, "rounds": 1, "el": 1.0, "merges": 1,
         "xgmi_tick": 0.0, "layout": "columns", "tiles": 8, "csr_ms": 0.1}
    out = bench.summarize_full(r, bench.N_NODES, 20, 1, 5)
    assert out["roofline"]["traffic"] is not None
    out = bench.summarize_full(r, bench.N_NODES, 40, 1, 5)
    assert out["roofline"]["traffic"] is None and "ticks 6-45" in out["roofline"]["traffic_note"]
