// gossip_protocol_amd/csrc/pview_engine.cpp -- host side of the PARTIAL-VIEW engine (C ABI).
//
// One GPU: per tick, stream-ordered and without host synchronisation,
//   exclusive_scan(deg) -> off, scatter(out_dst) -> csr, memset(deg), pview_tick_kernel.
// Row shards (G > 1, BASELINE config 5 on 2/4/8 GPUs): shard g owns the views of nodes
// [floor(g n / G), floor((g + 1) n / G)).  Before tick t merges, every sender view that a
// message of tick t - 1 carries to another shard moves there (rowx_kernels.hpp):
//   pack + gather     pairs (sender, destination shard) and message records, per shard h
//   counts            all-gather of the 2G pair / record counts of every shard, read by the
//                     host (the one synchronisation per tick: RCCL needs element counts)
//   rows + records    RCCL send/recv between every pair of shards inside one group call
//                     (one process per GPU), or device copies for an in-process group
//   csr               local messages + received records -> receiver CSR of the local rows
// then the same tick kernel runs on the local rows, reading remote sender views from the
// received rows.  Results are identical to the one-GPU engine for every G.
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "common.hpp"
#include "join_kernels.hpp"
#include "philox.hpp"
#include "policy.hpp"
#include "pview_kernels.hpp"
#include "rowx_host.hpp"
#include "rowx_kernels.hpp"
#include "scale_kernels.hpp"


namespace {

struct PvShard {
    int32_t g = 0, row0 = 0, rows = 0;
    gsp::DevBuf<uint64_t> table[2];
    gsp::DevBuf<int32_t> len[2], own_hb, fail_tick, out_dst, out_pos, deg, off, fill, csr_src, err,
        tile_sum, rc_info, rc_src, rc_slot, kcount, order, start_tick, ping, joiners, join_ok,
        rows_run,                // tests (GSP_TEST_PV_COUNT_ROWS=1): rows run per tick
        long_list;               // drain-all: the rows sent > kPvMaxInbox messages, by class
    gsp::DevBuf<uint32_t> scratch;     // drain-all: the HBM drain kernel's tuple buffers
    gsp::DevBuf<uint64_t> intro_buf;   // row layout, shards != 0: node 0's view of the last tick
    gsp::DevBuf<unsigned long long> dig, prof, rowdig;
    gsp::EvRing ev;
    gsp::RowxBufs x;             // row exchange (G > 1)

    void release() {
        for (int b = 0; b < 2; ++b) { table[b].release(); len[b].release(); }
        for (auto *b : {&own_hb, &fail_tick, &out_dst, &out_pos, &deg, &off, &fill, &csr_src, &err,
                        &tile_sum, &rc_info, &rc_src, &rc_slot, &kcount, &order, &start_tick, &ping,
                        &joiners, &join_ok, &rows_run, &long_list})
            b->release();
        scratch.release();
        intro_buf.release();
        x.release();
        dig.release();
        prof.release();
        rowdig.release();
        ev.release();
    }
};

}  // namespace

struct gsp_pview {
    gsp_pview_params p{};
    int device = 0;
    hipStream_t st = nullptr;
    int32_t shards = 1;          // G: row shards of the job
    int32_t rank = 0;            // first shard held by this engine
    bool rowmode = false;        // exchange path (G > 1, or any RCCL communicator)
    ncclComm_t comm = nullptr;
    int64_t pair_cap = 0, msg_cap = 0;
    int32_t tick = 0;
    bool timing = true;
    int32_t split = 1;           // GSP_TEST_PV_SPLIT=0: every row in the one 256-lane kernel; else
                                 // rows bucketed by k into four kernels (pview_kernels.hip)
    bool pos_scatter = false;    // one shard, no join schedule: the receiver CSR is scattered from
                                 // the positions the send kernel's deg atomics returned (the
                                 // JOINREP append and the row exchange keep the fill counters)
    int32_t cus = 0;             // compute units (drain grid)
    int32_t *h_kcount = nullptr; // pinned [8]: the bucket sizes, the split kernels' grids
    hipEvent_t kcount_ev = nullptr;
    hipStream_t drain_st = nullptr;     // drain all, split form: the drain classes' stream
    hipEvent_t drain_fork = nullptr, drain_join = nullptr;   // (GSP_TEST_PV_DRAIN_STREAM=1 / 2 only)
    int32_t drain_side = 0;      // 1 every drain class on drain_st, 2 the hub kernel only
    int32_t max_segment = gsp::kPvMaxSegment;
    bool sort_rows = true;       // run rows k-descending (GSP_TEST_PV_SORT=0 turns it off)
    bool drain = false;          // inbox 0: every message merged (pview_drain.hip)
    int64_t scratch_cap = 0;     // HBM drain kernel: tuples per buffer (two per workgroup)
    int32_t drain_lds = gsp::kDrainLdsMax;   // drain kernels: LDS tuples (GSP_TEST_PV_DRAIN_LDS lowers it)
    int32_t drain_wide = 0;      // tests: GSP_TEST_PV_DRAIN_WIDE=w runs the rows of classes < w in class w
    int32_t *h_err = nullptr;    // pinned mirror of the shards' capacity flags (async copies)
    int32_t *h_dhead = nullptr;  // drain all: pinned copy of a shard's long_list head (class sizes)
    bool nowait = false;         // row shards: no host wait for the bucket sizes (PviewTickArgs.nowait;
                                 // GSP_TEST_PV_NOWAIT=0/1 turns it off / on for tests)
    int32_t *h_dring = nullptr;  // nowait + drain all: pinned [max_ticks + 1][local shards][kDrainHead]
    std::vector<std::pair<int32_t, int32_t>> dring_pending;   // (tick, local shard) heads to add
    // drain all: per class, rows and messages run and kernel ms (gsp_pview_drain_stats)
    // class c runs from [c] to [c + 1]; the hub kernel on its own stream from [kDrainClasses + 1]
    using DrainEvents = std::array<hipEvent_t, gsp::kDrainClasses + 2>;
    std::vector<DrainEvents> dpending;
    int64_t drain_rows[gsp::kDrainClasses] = {}, drain_msgs[gsp::kDrainClasses] = {};
    double drain_ms[gsp::kDrainClasses] = {};
    std::vector<PvShard> local;
    std::vector<int32_t> h_fail, h_start;
    bool joins = false;          // a join schedule is set (some node starts after tick 0)
    gsp::JoinPlan plan;
    gsp::RowxState rowx;         // row exchange: count ring, posted sizes (rowx_host.hpp)
    struct Timed { hipEvent_t a, b, c; };
    std::vector<Timed> pending;
    std::vector<hipEvent_t> free_events;
    gsp_scale_perf perf{};

    hipEvent_t event() {
        if (!free_events.empty()) {
            hipEvent_t e = free_events.back();
            free_events.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }

    gsp::PviewTickArgs args(PvShard &sh, int32_t t) const {
        gsp::PviewTickArgs a{};
        a.prev = sh.table[(t + 1) & 1].p;
        a.cur = sh.table[t & 1].p;
        a.remote = rowmode ? sh.x.recv_rows.p : nullptr;
        a.n = p.n;
        a.view = p.view;
        a.inbox = p.inbox ? p.inbox : gsp::kPvMaxInbox;
        a.fanout = p.fanout;
        a.tick = t;
        a.tremove = p.tremove;
        a.h0 = p.h0;
        a.row0 = sh.row0;
        a.rows = sh.rows;
        a.seed = p.seed;
        a.fail_tick = sh.fail_tick.p;
        a.start_tick = joins ? sh.start_tick.p : nullptr;
        a.drop_pct = gsp::drop_at(p.policy, p.drop_pct, t);
        a.drop_prev = gsp::drop_at(p.policy, p.drop_pct, t - 1);
        a.tfail = p.tfail;
        a.swim = p.swim;
        a.ping = sh.ping.p;
        a.intro = (rowmode && sh.row0 != 0) ? sh.intro_buf.p : sh.table[(t + 1) & 1].p;
        a.intro_list = p.policy.intro_list;
        a.own_hb = sh.own_hb.p;
        a.len_cur = sh.len[t & 1].p;
        a.rc_info = sh.rc_info.p;
        a.rc_src = sh.rc_src.p;
        a.rc_slot = sh.rc_slot.p;
        a.out_dst = sh.out_dst.p;
        a.out_pos = sh.out_pos.p;
        a.rowdig = sh.rowdig.p;
        a.deg = sh.deg.p;
        a.dig = sh.dig.p + size_t(t) * gsp::kPvDigSlots * gsp::kPvFields;
        a.err = local[0].err.p;        // one flag for every shard held here
        a.max_segment = max_segment;
        a.kcount = sort_rows ? sh.kcount.p : nullptr;
        a.order = sort_rows ? sh.order.p : nullptr;
        a.prof = sh.prof.p;
        a.split = split;
        a.kcount_host = h_kcount;
        a.kcount_event = kcount_ev;
        a.drain_st = drain_st;
        a.drain_fork = drain_fork;
        a.drain_join = drain_join;
        a.drain_side = drain_side;
        a.rows_run = sh.rows_run.p ? sh.rows_run.p + t : nullptr;
        a.evict_rot = p.evict_order;
        a.ev = sh.ev.args();
        a.nowait = nowait ? 1 : 0;
        if (drain) {
            a.drain = 1;
            a.long_list = sh.long_list.p;
            a.csr_off = sh.off.p;
            a.csr_src = sh.csr_src.p;
            a.csr_slot = rowmode ? sh.x.csr_slot.p : nullptr;
            a.scratch = local[0].scratch.p;
            a.scratch_cap = scratch_cap;
            a.cus = cus;
            a.drain_lds = drain_lds;
            a.drain_wide = drain_wide;
            a.drain_rows = h_dhead;
            if (nowait && h_dring)
                a.dhead_async = h_dring + (size_t(t) * local.size() + size_t(&sh - local.data())) * gsp::kDrainHead;
        }
        return a;
    }

    gsp::PviewReceiptArgs receipt(PvShard &sh) const {
        gsp::PviewReceiptArgs a{};
        a.off = sh.off.p;
        a.csr_src = sh.csr_src.p;
        a.csr_slot = rowmode ? sh.x.csr_slot.p : nullptr;
        a.rows = sh.rows;
        a.row0 = sh.row0;
        a.inbox = p.inbox ? p.inbox : gsp::kPvMaxInbox;
        a.tick = tick + 1;
        a.max_segment = max_segment;
        a.rc_info = sh.rc_info.p;
        a.rc_src = sh.rc_src.p;
        a.rc_slot = sh.rc_slot.p;
        a.kcount = sort_rows ? sh.kcount.p : nullptr;
        a.order = sort_rows ? sh.order.p : nullptr;
        a.err = local[0].err.p;
        a.drain = drain ? 1 : 0;
        a.long_list = drain ? sh.long_list.p : nullptr;
        a.view = p.view;
        a.drain_lds = drain_lds;
        a.drain_wide = drain_wide;
        return a;
    }

    PvShard *holder(int32_t r) {
        for (PvShard &sh : local)
            if (r >= sh.row0 && r < sh.row0 + sh.rows) return &sh;
        return nullptr;
    }
};

namespace {

int pview_validate(const gsp_pview_params *p) {
    GSP_REQUIRE(p, GSP_ERR_INVALID, "pview params NULL");
    GSP_REQUIRE(p->n >= 2 && p->n < (1 << 21), GSP_ERR_INVALID, "n=%d outside [2, 2^21 - 1]", p->n);
    GSP_REQUIRE(p->view >= 1 && p->view <= gsp::kPvMaxView, GSP_ERR_INVALID, "view=%d outside [1, %d]",
                p->view, gsp::kPvMaxView);
    GSP_REQUIRE(p->inbox >= 0 && p->inbox <= gsp::kPvMaxInbox, GSP_ERR_INVALID,
                "inbox=%d outside [0, %d] (0: every message merged)", p->inbox, gsp::kPvMaxInbox);
    // drain all: the hub kernel's HBM buffers hold any receiver's list plus one message's runs
    // (a power of two >= n + 3 kPvMaxView tuples, at most 2^21)
    GSP_REQUIRE(p->inbox > 0 || p->n <= (1 << 21) - 3 * gsp::kPvMaxView, GSP_ERR_INVALID,
                "inbox=0 (drain all) needs n <= %d", (1 << 21) - 3 * gsp::kPvMaxView);
    GSP_REQUIRE(p->fanout >= 1 && p->fanout <= 16, GSP_ERR_INVALID, "fanout=%d outside [1,16]",
                p->fanout);
    GSP_REQUIRE(p->tremove >= 1 && p->tremove <= 31, GSP_ERR_INVALID, "tremove=%d outside [1,31]",
                p->tremove);
    GSP_REQUIRE(p->h0 >= 1 && p->h0 < 2047, GSP_ERR_INVALID, "h0=%d", p->h0);
    GSP_REQUIRE(p->drop_pct >= 0 && p->drop_pct <= 100, GSP_ERR_INVALID, "drop_pct=%d", p->drop_pct);
    GSP_REQUIRE(p->fail_mode >= 0 && p->fail_mode <= 2, GSP_ERR_INVALID, "fail_mode=%d", p->fail_mode);
    GSP_REQUIRE(p->max_ticks >= 1 && int64_t(p->h0) + p->max_ticks <= 2047, GSP_ERR_RANGE,
                "h0 + max_ticks exceeds the 11-bit packed heartbeat");
    GSP_REQUIRE(p->tfail == 0 || (p->tfail >= 1 && p->tfail < p->tremove), GSP_ERR_INVALID,
                "tfail=%d: 0 (off) or 1..tremove-1", p->tfail);
    GSP_REQUIRE(p->swim >= 0 && p->swim <= 8, GSP_ERR_INVALID, "swim=%d: 0 (off) or 1..8 paths", p->swim);
    GSP_REQUIRE(p->events >= 0 && p->events <= 15, GSP_ERR_INVALID, "events=%d: 0 off, 1 all, or an OR of GSP_EVENTS_*", p->events);
    GSP_REQUIRE(p->event_cap >= 0, GSP_ERR_INVALID, "event_cap=%lld", (long long)p->event_cap);
    GSP_REQUIRE(p->evict_order == 0 || p->evict_order == 1, GSP_ERR_INVALID,
                "evict_order=%d: 0 (age, -hb, id) or 1 (rotated id ties)", p->evict_order);
    return gsp::validate_policy(p->policy, p->n);
}

int shard_alloc(gsp_pview *s, PvShard &sh) {
    const int32_t n = s->p.n, F = s->p.fanout, V = s->p.view, G = s->shards;
    const size_t rows = size_t(sh.rows);
    hipStream_t st = s->st;
    for (int b = 0; b < 2; ++b) {
        GSP_HIP(sh.table[b].alloc(rows * size_t(V)));
        GSP_HIP(sh.len[b].alloc(rows));
        GSP_HIP(hipMemsetAsync(sh.len[b].p, 0, rows * 4, st));
    }
    GSP_HIP(sh.own_hb.alloc(rows));
    GSP_HIP(sh.fail_tick.alloc(size_t(n)));
    GSP_HIP(sh.out_dst.alloc(rows * F));
    if (s->pos_scatter) GSP_HIP(sh.out_pos.alloc(rows * F));
    GSP_HIP(sh.deg.alloc(size_t(n)));
    GSP_HIP(sh.off.alloc(rows + 1));
    GSP_HIP(sh.fill.alloc(rows));
    GSP_HIP(sh.csr_src.alloc(size_t(n) * F));      // every message of the job, at most
    GSP_HIP(sh.err.alloc(1));
    GSP_HIP(sh.tile_sum.alloc(size_t(n) / 4096 + 1));
    GSP_HIP(sh.rc_info.alloc(rows));
    GSP_HIP(sh.rc_src.alloc(rows * 8));
    GSP_HIP(sh.rc_slot.alloc(rows * 8));
    GSP_HIP(sh.rowdig.alloc(rows * 16));
    if (s->sort_rows) {
        GSP_HIP(sh.kcount.alloc(8));
        GSP_HIP(sh.order.alloc(rows * 8));
    }
    GSP_HIP(hipMemsetAsync(sh.rowdig.p, 0, rows * 16 * 8, st));
    if (s->rowmode)
        GSP_HIP(sh.x.alloc(G, s->pair_cap, s->msg_cap, V, true, s->comm != nullptr, int64_t(n) * F, st));
    if (s->p.swim > 0) {
        GSP_HIP(sh.ping.alloc(rows));
        GSP_HIP(hipMemsetAsync(sh.ping.p, 0xFF, rows * 4, st));     // -1: no probe yet
    }
    if (s->joins) {
        GSP_HIP(sh.start_tick.alloc(size_t(n)));
        GSP_HIP(hipMemcpyAsync(sh.start_tick.p, s->h_start.data(), size_t(n) * 4, hipMemcpyHostToDevice, st));
        const size_t nj = std::max<size_t>(1, s->plan.joiners.size());
        GSP_HIP(sh.joiners.alloc(nj));
        GSP_HIP(sh.join_ok.alloc(nj));
        if (!s->plan.joiners.empty())
            GSP_HIP(hipMemcpyAsync(sh.joiners.p, s->plan.joiners.data(), s->plan.joiners.size() * 4,
                                   hipMemcpyHostToDevice, st));
        // a late joiner's (empty) view is read at its start tick from either buffer
        GSP_HIP(hipMemsetAsync(sh.table[1].p, 0xFF, rows * size_t(V) * 8, st));
        if (s->rowmode && sh.row0 != 0) GSP_HIP(sh.intro_buf.alloc(size_t(V)));
    }
    if (s->p.events) GSP_HIP(sh.ev.alloc(s->p.events, s->p.event_cap, st));
    if (s->drain) {
        GSP_HIP(sh.long_list.alloc(gsp::kDrainHead + size_t(gsp::kDrainClasses) * rows));
        GSP_HIP(hipMemsetAsync(sh.long_list.p, 0, gsp::kDrainHead * 4, st));
        // 2 x u64 per CU, one set for every shard held here: their hub kernels run one after
        // the other on the engine's stream
        if (&sh == &s->local[0]) GSP_HIP(sh.scratch.alloc(size_t(s->cus) * 4 * size_t(s->scratch_cap)));
    }
    const size_t dig = size_t(s->p.max_ticks + 1) * gsp::kPvDigSlots * gsp::kPvFields;
    GSP_HIP(sh.dig.alloc(dig));
    if (const char *cr = std::getenv("GSP_TEST_PV_COUNT_ROWS"); cr && std::atoi(cr)) {
        GSP_HIP(sh.rows_run.alloc(size_t(s->p.max_ticks + 1)));
        GSP_HIP(hipMemsetAsync(sh.rows_run.p, 0, size_t(s->p.max_ticks + 1) * 4, st));
    }
    if (const char *pf = std::getenv("GSP_PV_PROFILE"); pf && std::atoi(pf)) {
        GSP_HIP(sh.prof.alloc(64 * 16 * gsp::kPvProfPhases));   // k slots 8-15: the drain kernel
        GSP_HIP(hipMemsetAsync(sh.prof.p, 0, 64 * 16 * gsp::kPvProfPhases * 8, st));
    }
    GSP_HIP(hipMemsetAsync(sh.dig.p, 0, dig * 8, st));
    GSP_HIP(hipMemsetAsync(sh.own_hb.p, 0, rows * 4, st));
    GSP_HIP(hipMemsetAsync(sh.deg.p, 0, size_t(n) * 4, st));
    GSP_HIP(hipMemsetAsync(sh.err.p, 0, 4, st));
    GSP_HIP(hipMemcpyAsync(sh.fail_tick.p, s->h_fail.data(), size_t(n) * 4, hipMemcpyHostToDevice, st));
    return GSP_OK;
}

// Move the sender views of tick t_sent's cross-shard messages to their destination shards and
// build every local shard's receiver CSR for tick t_sent + 1 (rowx_host.cpp).
int exchange_and_csr(gsp_pview *s, int32_t t_sent) {
    gsp::RowxJob job{s->p.n, s->shards, s->p.fanout, s->p.view, true, s->pair_cap, s->msg_cap,
                     s->comm, s->st, t_sent + 1, &s->rowx};
    // a joiner's sends ramp up to F over its first ticks (its view grows): the joiners of the
    // last three send ticks count as new senders
    job.new_senders = s->joins ? s->plan.count(t_sent) + s->plan.count(t_sent - 1) + s->plan.count(t_sent - 2) : 0;
    job.drop_now = gsp::drop_at(s->p.policy, s->p.drop_pct, t_sent);
    job.drop_before = gsp::drop_at(s->p.policy, s->p.drop_pct, t_sent - 1);
    std::vector<gsp::RowxShard> v;
    for (PvShard &sh : s->local)
        v.push_back(gsp::RowxShard{sh.g, sh.row0, sh.rows, sh.out_dst.p, sh.table[t_sent & 1].p,
                                   sh.deg.p, sh.off.p, sh.fill.p, sh.csr_src.p, sh.tile_sum.p,
                                   s->local[0].err.p, &sh.x});
    return gsp::rowx_exchange(job, v, &s->perf.xgmi_bytes);
}

// The capacity flag as last mirrored to the host: a receiver sent more than max_segment
// messages at tick t sets the flag to t, and the tick kernels of t and every later tick run no
// row, so the job's state stays that of tick t - 1.  A drain-all hub row past its HBM buffers
// (tick t | kDrainErrBit) is found while tick t's rows run: rows already done hold tick t, the
// others are skipped, so the views after that error are undefined (the job stops all the same).
// Every shard held by this engine reads one flag (shard 0's), so an in-process group stops as a
// whole; ranks of a communicator exchange their flags with the row-exchange counts and stop at
// the same tick.
int pview_mirrored_err(gsp_pview *s) {
    for (size_t i = 0; i < s->local.size(); ++i) {
        const int32_t e = s->h_err[i];
        GSP_REQUIRE(!(e & gsp::kRowxErrBit), GSP_ERR_CAPACITY,
                    "row exchange at tick %d: a shard's rows or records passed the region capacity "
                    "or the size posted to RCCL; the job stopped there", e & ~gsp::kRowxErrBit);
        GSP_REQUIRE(!(e & gsp::kDrainErrBit), GSP_ERR_CAPACITY,
                    "drain all at tick %d: a hub row's list passed its HBM buffers; the job stopped "
                    "there (the views of that tick are undefined)", e & ~gsp::kDrainErrBit);
        GSP_REQUIRE(e == 0, GSP_ERR_CAPACITY,
                    "a receiver was sent more than %d messages at tick %d; the job stopped there",
                    s->max_segment, e);
    }
    return GSP_OK;
}

// The JOINREPs node 0 sends at tick t to the nodes that start at t + 1 (join_kernels.hpp),
// and (row layout) node 0's view of tick t broadcast to the other shards as their payload.
int pv_join_sends(gsp_pview *s, int32_t t) {
    const int64_t cnt = s->plan.count(t + 1);
    if (!s->joins || cnt == 0) return GSP_OK;
    for (PvShard &sh : s->local) {
        gsp::JoinSendArgs j{};
        j.joiners = sh.joiners.p + s->plan.first(t + 1);
        j.count = int32_t(cnt);
        j.tick = t;
        j.drop_pct = gsp::drop_at(s->p.policy, s->p.drop_pct, t);
        j.seed = s->p.seed;
        j.fail_tick = sh.fail_tick.p;
        j.lo = sh.row0;
        j.hi = sh.row0 + sh.rows;
        j.ok = sh.join_ok.p + s->plan.first(t + 1);
        j.deg = sh.deg.p;
        unsigned long long *dig = sh.dig.p + size_t(t) * gsp::kPvDigSlots * gsp::kPvFields;
        j.sent = dig + gsp::kPvSent;
        j.dropped = dig + gsp::kPvDropped;
        GSP_HIP(gsp::launch_join_send(j, s->st));
    }
    if (!s->rowmode || s->shards == 1) return GSP_OK;
    const size_t bytes = size_t(s->p.view) * 8;
    if (s->comm) {
        PvShard &sh = s->local[0];
        void *buf = sh.row0 == 0 ? static_cast<void *>(sh.table[t & 1].p) : static_cast<void *>(sh.intro_buf.p);
        GSP_NCCL(ncclBroadcast(buf, buf, bytes, ncclUint8, 0, s->comm, s->st));
        s->perf.xgmi_bytes += sh.row0 == 0 ? double(bytes) * double(s->shards - 1) : 0.0;
        return GSP_OK;
    }
    const PvShard &root = s->local[0];
    for (PvShard &sh : s->local)
        if (sh.row0 != 0) {
            GSP_HIP(hipMemcpyAsync(sh.intro_buf.p, root.table[t & 1].p, bytes, hipMemcpyDeviceToDevice, s->st));
            s->perf.xgmi_bytes += double(bytes);
        }
    return GSP_OK;
}

int pv_join_scatter(gsp_pview *s, int32_t t) {
    const int64_t cnt = s->plan.count(t);
    if (!s->joins || cnt == 0) return GSP_OK;
    for (PvShard &sh : s->local)
        GSP_HIP(gsp::launch_join_scatter(sh.joiners.p + s->plan.first(t), sh.join_ok.p + s->plan.first(t),
                                         int32_t(cnt), sh.row0, sh.rows, sh.off.p, sh.fill.p, sh.csr_src.p,
                                         s->rowmode ? sh.x.csr_slot.p : nullptr, s->st));
    return GSP_OK;
}

int pview_collect(gsp_pview *s) {
    for (auto &t : s->pending) {
        float a = 0.f, b = 0.f;
        GSP_HIP(hipEventSynchronize(t.c));
        GSP_HIP(hipEventElapsedTime(&a, t.a, t.b));
        GSP_HIP(hipEventElapsedTime(&b, t.b, t.c));
        s->perf.csr_ms += a;
        s->perf.merge_ms += b;
        s->perf.merge_launches++;
        s->free_events.push_back(t.a);
        s->free_events.push_back(t.b);
        s->free_events.push_back(t.c);
    }
    s->pending.clear();
    for (auto &de : s->dpending) {
        GSP_HIP(hipEventSynchronize(de[gsp::kDrainClasses]));
        for (int c = 0; c < gsp::kDrainClasses; ++c) {
            float ms = 0.f;
            const size_t c0 = c == gsp::kDrainHub && s->drain_side == 2 ? size_t(gsp::kDrainClasses) + 1 : size_t(c);
            GSP_HIP(hipEventElapsedTime(&ms, de[c0], de[size_t(c) + 1]));
            s->drain_ms[c] += ms;
        }
        for (hipEvent_t e : de) s->free_events.push_back(e);
    }
    s->dpending.clear();
    for (const auto &ti : s->dring_pending) {      // the stream has been synchronised
        const int32_t *h = s->h_dring + (size_t(ti.first) * s->local.size() + size_t(ti.second)) * gsp::kDrainHead;
        for (int c = 0; c < gsp::kDrainClasses; ++c) {
            s->drain_rows[c] += h[c];
            s->drain_msgs[c] += h[8 + c];
        }
    }
    s->dring_pending.clear();
    if (s->rowmode)
        if (int rc = gsp::rowx_collect(s->rowx, &s->perf.xgmi_bytes)) return rc;
    for (size_t i = 0; i < s->local.size(); ++i)
        GSP_HIP(hipMemcpy(s->h_err + i, s->local[i].err.p, 4, hipMemcpyDeviceToHost));
    return pview_mirrored_err(s);
}

int pview_build(const gsp_pview_params *p, int device, int32_t shards, int32_t rank,
                int32_t local_shards, const void *nccl_id, gsp_pview **out) {
    GSP_REQUIRE(out, GSP_ERR_INVALID, "gsp_pview: out is NULL");
    *out = nullptr;
    if (int rc = pview_validate(p)) return rc;
    GSP_REQUIRE(shards >= 1 && shards <= 64 && shards <= p->n && rank >= 0 &&
                    rank + local_shards <= shards,
                GSP_ERR_INVALID, "gsp_pview: shards=%d rank=%d n=%d", shards, rank, p->n);
    int ndev = 0;
    GSP_HIP(hipGetDeviceCount(&ndev));
    GSP_REQUIRE(device >= 0 && device < ndev, GSP_ERR_HIP, "gsp_pview: device %d of %d", device, ndev);
    GSP_HIP(hipSetDevice(device));
    std::unique_ptr<gsp_pview> s(new gsp_pview);
    s->p = *p;
    s->device = device;
    s->shards = shards;
    s->rank = rank;
    s->rowmode = shards > 1 || nccl_id != nullptr;
    if (const char *sp = std::getenv("GSP_TEST_PV_SPLIT")) s->split = std::atoi(sp);
    if (const char *so = std::getenv("GSP_TEST_PV_SORT")) s->sort_rows = std::atoi(so) != 0;
    if (s->split && s->sort_rows) {
        GSP_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->h_kcount), 8 * 4));
        GSP_HIP(hipEventCreateWithFlags(&s->kcount_ev, hipEventDisableTiming));
        if (p->inbox == 0) GSP_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->h_dhead), gsp::kDrainHead * 4));
        // drain all: the hub kernel on a stream of its own beside the split kernels and the LDS
        // classes (few hub rows, one per CU, would leave the rest of the GPU idle); tests / A/B:
        // GSP_TEST_PV_DRAIN_STREAM=0 one stream, =1 every drain class on the side stream (slower,
        // DESIGN.md 4b)
        const char *ds = std::getenv("GSP_TEST_PV_DRAIN_STREAM");
        const int dmode = ds ? std::atoi(ds) : 2;
        if (p->inbox == 0 && dmode) {
            s->drain_side = dmode == 1 ? 1 : 2;
            GSP_HIP(hipStreamCreateWithFlags(&s->drain_st, hipStreamNonBlocking));
            GSP_HIP(hipEventCreateWithFlags(&s->drain_fork, hipEventDisableTiming));
            GSP_HIP(hipEventCreateWithFlags(&s->drain_join, hipEventDisableTiming));
        }
        s->nowait = s->rowmode;
        if (const char *nw = std::getenv("GSP_TEST_PV_NOWAIT")) s->nowait = std::atoi(nw) != 0;
        if (s->nowait && p->inbox == 0)
            GSP_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->h_dring),
                                  size_t(p->max_ticks + 1) * size_t(local_shards) * gsp::kDrainHead * 4));
    }
    GSP_HIP(hipDeviceGetAttribute(&s->cus, hipDeviceAttributeMultiprocessorCount, device));
    s->h_fail = gsp::fail_ticks(p->policy, p->n, p->seed, p->fail_mode, p->fail_tick, p->fail_ppm);
    s->h_start = gsp::start_ticks(p->policy, p->n);
    s->joins = p->policy.step_rate > 0 && *std::max_element(s->h_start.begin(), s->h_start.end()) > 0;
    s->drain = p->inbox == 0;
    if (s->drain) {
        // the HBM drain kernel (class 4 rows) runs one 1024-lane workgroup per CU, each with two
        // HBM tuple buffers: a power of two >= n + 3 kPvMaxView, so a list of distinct ids plus
        // one message's runs always fits and any row finishes in chunks (n <= 2^21 - 768; ids
        // are 21 bits): 2 x 16 MB per CU at n = 1M, in drain mode only
        s->scratch_cap = 8192;
        while (s->scratch_cap < int64_t(p->n) + 3 * gsp::kPvMaxView && s->scratch_cap < (int64_t(1) << 21))
            s->scratch_cap <<= 1;
        if (const char *dl = std::getenv("GSP_TEST_PV_DRAIN_LDS"))   // tests: reach the HBM paths
            s->drain_lds = std::max(gsp::kPvMaxView + 2, std::min(gsp::kDrainLdsMax, std::atoi(dl)));
        if (const char *dw = std::getenv("GSP_TEST_PV_DRAIN_WIDE")) s->drain_wide = std::max(0, std::min(3, std::atoi(dw)));
    }
    s->pos_scatter = !s->rowmode && !s->joins;
    if (const char *ps = std::getenv("GSP_TEST_PV_POS_SCATTER"); ps && !std::atoi(ps)) s->pos_scatter = false;
    if (s->joins) s->plan = gsp::join_plan(s->h_start, p->max_ticks + 1);
    int32_t max_rows = 0;
    for (int32_t g = 0; g < shards; ++g)
        max_rows = std::max(max_rows, gsp::rowx_row0(g + 1, p->n, shards) - gsp::rowx_row0(g, p->n, shards));
    s->pair_cap = max_rows;                       // a sender row goes to a shard at most once
    s->msg_cap = int64_t(max_rows) * p->fanout;
    // the per-row overflow field of the digest record is 16 bits: k_all - k <= 65535 (drain
    // all: no overflow, no bound -- a long row's counts go to the digest directly)
    s->max_segment = s->drain ? INT32_MAX : std::min(gsp::kPvMaxSegment, 65535 + p->inbox);
    if (const char *ms = std::getenv("GSP_TEST_MAX_SEGMENT"))   // tests only: force overflows
        s->max_segment = std::max(1, std::min(s->max_segment, std::atoi(ms)));
    GSP_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
    GSP_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->h_err), size_t(local_shards) * 4));
    std::memset(s->h_err, 0, size_t(local_shards) * 4);
    if (s->rowmode) {
        GSP_HIP(s->rowx.init(shards, nccl_id != nullptr));
    }
    if (nccl_id) {
        ncclUniqueId id;
        std::memcpy(&id, nccl_id, sizeof id);
        GSP_NCCL(ncclCommInitRank(&s->comm, shards, id, rank));
    }
    s->local.resize(size_t(local_shards));
    for (int32_t i = 0; i < local_shards; ++i) {
        PvShard &sh = s->local[size_t(i)];
        sh.g = rank + i;
        sh.row0 = gsp::rowx_row0(sh.g, p->n, shards);
        sh.rows = gsp::rowx_row0(sh.g + 1, p->n, shards) - sh.row0;
        if (int rc = shard_alloc(s.get(), sh)) return rc;
    }
    for (PvShard &sh : s->local) GSP_HIP(gsp::launch_pview_init(s->args(sh, 0), s->st));
    if (int rc = pv_join_sends(s.get(), 0)) return rc;
    GSP_HIP(hipStreamSynchronize(s->st));
    *out = s.release();
    return GSP_OK;
}

}  // namespace

extern "C" {

int gsp_pview_create(const gsp_pview_params *p, int device, gsp_pview **out) {
    return pview_build(p, device, 1, 0, 1, nullptr, out);
}

int gsp_pview_create_group(const gsp_pview_params *p, int device, int32_t shards, gsp_pview **out) {
    return pview_build(p, device, shards, 0, shards, nullptr, out);
}

int gsp_pview_create_rank(const gsp_pview_params *p, int device, int32_t rank, int32_t world,
                          const void *nccl_id, gsp_pview **out) {
    GSP_REQUIRE(nccl_id || world == 1, GSP_ERR_INVALID, "gsp_pview_create_rank: NULL nccl id");
    return pview_build(p, device, world, rank, 1, nccl_id, out);
}

int gsp_pview_layout(gsp_pview *s, int32_t *shards, int32_t *rank, int32_t *row0, int32_t *rows) {
    GSP_REQUIRE(s, GSP_ERR_INVALID, "gsp_pview_layout: NULL");
    if (shards) *shards = s->shards;
    if (rank) *rank = s->rank;
    if (row0) *row0 = s->local[0].row0;
    if (rows) {
        int32_t r = 0;
        for (PvShard &sh : s->local) r += sh.rows;
        *rows = r;
    }
    return GSP_OK;
}

int gsp_pview_destroy(gsp_pview *s) {
    if (!s) return GSP_OK;
    (void)hipSetDevice(s->device);
    if (s->st) (void)hipStreamSynchronize(s->st);
    for (auto &t : s->pending) {
        s->free_events.push_back(t.a);
        s->free_events.push_back(t.b);
        s->free_events.push_back(t.c);
    }
    for (auto &de : s->dpending)
        for (hipEvent_t e : de) s->free_events.push_back(e);
    for (hipEvent_t e : s->free_events) (void)hipEventDestroy(e);
    for (PvShard &sh : s->local) {
        if (sh.prof.p) {   // GSP_PV_PROFILE diagnostics: cycles per phase of sampled rows, by k
            constexpr int P = gsp::kPvProfPhases;
            std::vector<unsigned long long> h(64 * 16 * P);
            if (hipMemcpy(h.data(), sh.prof.p, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                unsigned long long ph[16][P] = {{0}};
                for (size_t i = 0; i < h.size(); ++i) ph[(i / P) % 16][i % P] += h[i];
                // k 0-7: the tick kernels; 8-15: the drain kernel's rows, k in [8 (b - 7), 8 (b - 6))
                // (15: k >= 64)
                for (int k = 0; k < 16; ++k) {
                    const unsigned long long rows = ph[k][P - 1];
                    if (!rows) continue;
                    unsigned long long tot = 0;
                    for (int i = 0; i < P - 1; ++i) tot += ph[k][i];
                    std::fprintf(stderr, "pview phases (shard %d) k=%d rows=%llu cycles/row=%.0f:", sh.g, k,
                                 rows, double(tot) / double(rows));
                    for (int i = 0; i < P - 1; ++i)
                        if (ph[k][i]) std::fprintf(stderr, " p%d=%.0f", i, double(ph[k][i]) / double(rows));
                    std::fprintf(stderr, "\n");
                }
            }
        }
        sh.release();
    }
    if (s->comm) (void)ncclCommDestroy(s->comm);
    s->rowx.release();
    if (s->h_err) (void)hipHostFree(s->h_err);
    if (s->h_kcount) (void)hipHostFree(s->h_kcount);
    if (s->h_dhead) (void)hipHostFree(s->h_dhead);
    if (s->h_dring) (void)hipHostFree(s->h_dring);
    if (s->kcount_ev) (void)hipEventDestroy(s->kcount_ev);
    if (s->drain_fork) (void)hipEventDestroy(s->drain_fork);
    if (s->drain_join) (void)hipEventDestroy(s->drain_join);
    if (s->drain_st) (void)hipStreamDestroy(s->drain_st);
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
    return GSP_OK;
}

int gsp_pview_step(gsp_pview *s, int32_t ticks) {
    GSP_REQUIRE(s && ticks >= 0, GSP_ERR_INVALID, "gsp_pview_step: bad argument");
    GSP_REQUIRE(s->tick + ticks <= s->p.max_ticks, GSP_ERR_RANGE, "gsp_pview_step: beyond max_ticks");
    GSP_HIP(hipSetDevice(s->device));
    // an earlier call's ticks overflowed: stop here -- except across ranks, whose async mirrors
    // land at different times (a rank returning here would leave the others in a collective);
    // the row exchange returns the error on every rank at the same tick instead
    if (!s->comm)
        if (int rc = pview_mirrored_err(s)) return rc;
    const int32_t n = s->p.n;
    for (int32_t i = 0; i < ticks; ++i) {
        const int32_t t = s->tick + 1;
        gsp_pview::Timed tm{};
        if (s->timing) {
            tm = {s->event(), s->event(), s->event()};
            GSP_HIP(hipEventRecord(tm.a, s->st));
        }
        if (s->rowmode) {
            if (int rc = exchange_and_csr(s, t - 1)) return rc;
        } else {
            PvShard &sh = s->local[0];
            GSP_HIP(gsp::launch_exclusive_scan(sh.deg.p, sh.off.p, n, sh.tile_sum.p, s->st));
            if (s->pos_scatter) {     // each message's slot in its receiver's segment came back
                                      // from the send kernel's deg atomic: no atomics here
                GSP_HIP(gsp::launch_pview_scatter(sh.out_dst.p, sh.out_pos.p, int64_t(n) * s->p.fanout,
                                                  s->p.fanout, sh.off.p, sh.csr_src.p, s->st));
            } else {
                GSP_HIP(hipMemsetAsync(sh.fill.p, 0, size_t(n) * 4, s->st));
                GSP_HIP(gsp::launch_scatter(sh.out_dst.p, int64_t(n) * s->p.fanout, s->p.fanout, 0,
                                            sh.off.p, sh.fill.p, sh.csr_src.p, s->st));
            }
            GSP_HIP(hipMemsetAsync(sh.deg.p, 0, size_t(n) * 4, s->st));
        }
        if (int rc = pv_join_scatter(s, t)) return rc;
        for (PvShard &sh : s->local) {
            if (s->sort_rows) GSP_HIP(hipMemsetAsync(sh.kcount.p, 0, 8 * 4, s->st));
            if (s->drain) GSP_HIP(hipMemsetAsync(sh.long_list.p, 0, gsp::kDrainHead * 4, s->st));
            GSP_HIP(gsp::launch_pview_receipt(s->receipt(sh), s->st));
        }
        // ranks: the receipt kernels' capacity flags, MAX over the ranks before any tick kernel
        // of t reads them -- every rank's rows of t run, or none does, and every rank's flag
        // (hence its sync) names the same tick
        if (s->comm)
            GSP_NCCL(ncclAllReduce(s->local[0].err.p, s->local[0].err.p, 1, ncclInt32, ncclMax, s->comm, s->st));
        if (s->timing) GSP_HIP(hipEventRecord(tm.b, s->st));
        for (PvShard &sh : s->local) {
            gsp::PviewTickArgs ta = s->args(sh, t);
            gsp_pview::DrainEvents de{};
            if (s->drain && s->timing) {
                for (hipEvent_t &e : de) e = s->event();
                ta.drain_ev = de.data();
            }
            GSP_HIP(gsp::launch_pview_tick(ta, s->st));
            if (ta.drain_ev) s->dpending.push_back(de);
            if (s->drain && ta.nowait && ta.dhead_async)   // copied without a wait: read after a sync
                s->dring_pending.emplace_back(t, int32_t(&sh - s->local.data()));
            else if (s->drain && s->h_dhead)     // the class sizes this launch read back
                for (int c = 0; c < gsp::kDrainClasses; ++c) {
                    s->drain_rows[c] += s->h_dhead[c];
                    s->drain_msgs[c] += s->h_dhead[8 + c];
                }
        }
        if (s->timing) {
            GSP_HIP(hipEventRecord(tm.c, s->st));
            s->pending.push_back(tm);
        }
        if (int rc = pv_join_sends(s, t)) return rc;
        s->tick = t;
        s->perf.ticks++;
    }
    for (size_t i = 0; i < s->local.size(); ++i)     // read by the next call, never waited on
        GSP_HIP(hipMemcpyAsync(s->h_err + i, s->local[i].err.p, 4, hipMemcpyDeviceToHost, s->st));
    return GSP_OK;
}

int gsp_pview_sync(gsp_pview *s) {
    GSP_REQUIRE(s, GSP_ERR_INVALID, "gsp_pview_sync: NULL");
    GSP_HIP(hipSetDevice(s->device));
    GSP_HIP(hipStreamSynchronize(s->st));
    return pview_collect(s);
}

int gsp_pview_digest_get(gsp_pview *s, int32_t t, gsp_pview_digest *out) {
    GSP_REQUIRE(s && out && t >= 0 && t <= s->tick, GSP_ERR_INVALID, "gsp_pview_digest_get: tick %d", t);
    if (int rc = gsp_pview_sync(s)) return rc;
    std::vector<unsigned long long> h(size_t(gsp::kPvDigSlots) * gsp::kPvFields);
    unsigned long long f[gsp::kPvFields] = {0};
    for (PvShard &sh : s->local) {
        GSP_HIP(hipMemcpy(h.data(), sh.dig.p + size_t(t) * h.size(), h.size() * 8, hipMemcpyDeviceToHost));
        for (int sl = 0; sl < gsp::kPvDigSlots; ++sl)
            for (int k = 0; k < gsp::kPvFields; ++k) f[k] += h[size_t(sl) * gsp::kPvFields + k];
    }
    out->tick = t;
    out->node_rounds = int64_t(f[gsp::kPvRounds]);
    out->merges = int64_t(f[gsp::kPvMerges]);
    out->sent = int64_t(f[gsp::kPvSent]);
    out->dropped = int64_t(f[gsp::kPvDropped]);
    out->delivered = int64_t(f[gsp::kPvDelivered]);
    out->overflow = int64_t(f[gsp::kPvOverflow]);
    out->joins = int64_t(f[gsp::kPvJoins]);
    out->removes = int64_t(f[gsp::kPvRemoves]);
    out->evicts = int64_t(f[gsp::kPvEvicts]);
    out->event_hash = f[gsp::kPvHash];
    return GSP_OK;
}

int gsp_pview_row(gsp_pview *s, int32_t r, uint64_t *buf, int32_t cap, int32_t *len) {
    GSP_REQUIRE(s && buf && len && r >= 0 && r < s->p.n && cap >= s->p.view, GSP_ERR_INVALID,
                "gsp_pview_row: bad argument");
    PvShard *sh = s->holder(r);
    GSP_REQUIRE(sh, GSP_ERR_INVALID, "gsp_pview_row: row %d is not held by this rank", r);
    if (int rc = gsp_pview_sync(s)) return rc;
    const int32_t last = std::min(s->tick, s->h_fail[size_t(r)]);
    const int32_t lr = r - sh->row0;
    GSP_HIP(hipMemcpy(buf, sh->table[last & 1].p + size_t(lr) * s->p.view, size_t(s->p.view) * 8,
                      hipMemcpyDeviceToHost));
    GSP_HIP(hipMemcpy(len, sh->len[last & 1].p + lr, 4, hipMemcpyDeviceToHost));
    return GSP_OK;
}

int gsp_pview_own_hb(gsp_pview *s, int32_t r, int32_t *hb) {
    GSP_REQUIRE(s && hb && r >= 0 && r < s->p.n, GSP_ERR_INVALID, "gsp_pview_own_hb: bad row");
    PvShard *sh = s->holder(r);
    GSP_REQUIRE(sh, GSP_ERR_INVALID, "gsp_pview_own_hb: row %d is not held by this rank", r);
    if (int rc = gsp_pview_sync(s)) return rc;
    GSP_HIP(hipMemcpy(hb, sh->own_hb.p + (r - sh->row0), 4, hipMemcpyDeviceToHost));
    return GSP_OK;
}

int gsp_pview_messages(gsp_pview *s, int32_t *dst, int64_t cap, int64_t *n) {
    GSP_REQUIRE(s && n, GSP_ERR_INVALID, "gsp_pview_messages: NULL");
    if (int rc = gsp_pview_sync(s)) return rc;
    int64_t total = 0;
    for (PvShard &sh : s->local) {
        const int64_t slots = int64_t(sh.rows) * s->p.fanout;
        if (dst && total < cap)
            GSP_HIP(hipMemcpy(dst + total, sh.out_dst.p, size_t(std::min(cap - total, slots)) * 4,
                              hipMemcpyDeviceToHost));
        total += slots;
    }
    *n = total;
    return GSP_OK;
}

// Same contract as gsp_scale_drain_events (gossip.h): the join / remove / evict records of every
// tick since the last drain, shard by shard, in device append order.
int gsp_pview_drain_events(gsp_pview *s, uint64_t *buf, int64_t cap, int64_t *n, int64_t *lost) {
    GSP_REQUIRE(s && n && cap >= 0 && (buf || cap == 0), GSP_ERR_INVALID, "gsp_pview_drain_events: bad argument");
    GSP_REQUIRE(s->p.events, GSP_ERR_INVALID, "gsp_pview_drain_events: the engine records no events "
                "(gsp_pview_params.events = 0)");
    if (int rc = gsp_pview_sync(s)) return rc;
    int64_t total = 0, dropped = 0;
    for (PvShard &sh : s->local) GSP_HIP(sh.ev.drain(buf, cap, &total, &dropped));
    *n = total;
    if (lost) *lost = dropped;
    return GSP_OK;
}

int gsp_pview_rows_run(gsp_pview *s, int32_t t, int64_t *rows) {
    GSP_REQUIRE(s && rows && t >= 1 && t <= s->tick, GSP_ERR_INVALID, "gsp_pview_rows_run: tick %d", t);
    GSP_REQUIRE(s->local[0].rows_run.p, GSP_ERR_INVALID,
                "gsp_pview_rows_run: the engine counts no rows (set GSP_TEST_PV_COUNT_ROWS=1 before create)");
    if (int rc = gsp_pview_sync(s)) return rc;
    int64_t total = 0;
    for (PvShard &sh : s->local) {
        int32_t c = 0;
        GSP_HIP(hipMemcpy(&c, sh.rows_run.p + t, 4, hipMemcpyDeviceToHost));
        total += c;
    }
    *rows = total;
    return GSP_OK;
}

int gsp_pview_drain_stats(gsp_pview *s, int32_t classes, int64_t *rows, int64_t *messages, double *ms) {
    GSP_REQUIRE(s && classes >= 0, GSP_ERR_INVALID, "gsp_pview_drain_stats: bad argument");
    if (int rc = gsp_pview_sync(s)) return rc;
    for (int32_t c = 0; c < classes; ++c) {
        const bool in = c < gsp::kDrainClasses;
        if (rows) rows[c] = in ? s->drain_rows[c] : 0;
        if (messages) messages[c] = in ? s->drain_msgs[c] : 0;
        if (ms) ms[c] = in ? s->drain_ms[c] : 0.0;
    }
    return GSP_OK;
}

int gsp_pview_perf_get(gsp_pview *s, gsp_scale_perf *out) {
    GSP_REQUIRE(s && out, GSP_ERR_INVALID, "gsp_pview_perf_get: NULL");
    if (int rc = gsp_pview_sync(s)) return rc;
    gsp_pview_digest d{};
    if (s->tick > 0)
        if (int rc = gsp_pview_digest_get(s, s->tick, &d)) return rc;
    // own view read + write, one sender view per merged message, 8-byte entries
    s->perf.bytes_per_tick = double(2 * d.node_rounds + d.delivered) * double(s->p.view) * 8.0 +
                             double(d.delivered + d.overflow) * 4.0;
    *out = s->perf;
    return GSP_OK;
}

}  // extern "C"
