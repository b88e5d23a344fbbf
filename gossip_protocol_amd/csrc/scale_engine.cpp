// gossip_protocol_amd/csrc/scale_engine.cpp -- host side of the SCALE engine (C ABI).
//
// One GPU (fused): one tick = four stream-ordered launches, no host synchronisation:
//   exclusive_scan(deg) -> off   receiver CSR offsets from last tick's destination counts
//   scatter(out_dst)   -> csr    sender ids per receiver (order fixed later by the kernel)
//   memset(deg)                  re-armed for this tick's sends
//   scale_tick_kernel            merge + ops + events + send, one workgroup per row
// Column shards (G > 1): shard g owns columns [g*W, (g+1)*W) of EVERY row, so the merge is
// entirely local; the only exchange per tick is
//   all-gather of the per-row member counts of every slice     (n * 4 B per shard)
//   all-reduce MAX of the resolved peer choices                (n * fanout * 4 B)
// over RCCL (one process per GPU) or, for a group of shards inside one process, device
// copies on the group's stream (used to test the sharded path on one GPU).
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "common.hpp"
#include "join_kernels.hpp"
#include "philox.hpp"
#include "policy.hpp"
#include "rowx_host.hpp"
#include "scale_kernels.hpp"

namespace {

struct Shard {
    int32_t g = 0;
    int32_t col0 = 0;
    int32_t row0 = 0, rows = 0;    // row layout: rows [row0, row0 + rows); else all n rows
    gsp::RowxBufs x;               // row layout exchange buffers
    gsp::DevBuf<uint16_t> table[2];
    gsp::DevBuf<int32_t> own_hb, fail_tick, cnt_total[2], cnt_slice, cnt_all, out_dst, picks,
        ping, deg, off, fill, csr_src, err, tile_sum, start_tick, joiners, join_ok,
        long_list;                 // [2][1 + rows] by tick parity: rows with k > kMaxSegment
                                   // (a CSR owner's: shard 0 of a shared group, else each)
    gsp::DevBuf<uint16_t> intro_buf;   // row layout, shards != 0: node 0's row of the last tick
    gsp::DevBuf<uint8_t> bitmap;
    gsp::DevBuf<unsigned long long> dig;
    gsp::EvRing ev;

    void release() {
        for (int b = 0; b < 2; ++b) { table[b].release(); cnt_total[b].release(); }
        for (auto *x : {&own_hb, &fail_tick, &cnt_slice, &cnt_all, &out_dst, &picks, &ping, &deg, &off,
                        &fill, &csr_src, &err, &tile_sum, &start_tick, &joiners, &join_ok, &long_list})
            x->release();
        intro_buf.release();
        bitmap.release();
        dig.release();
        ev.release();
        x.release();
    }
};

}  // namespace

struct gsp_scale {
    gsp_scale_params p{};
    int device = 0;
    hipStream_t st = nullptr;
    int32_t shards = 1;        // G: column shards in the whole job
    int32_t rank = 0;          // first shard index held by this engine
    bool sliced = false;       // column layout (G > 1)
    bool shared = false;       // column layout, every shard in this process on one device (an
                               // in-process group): the shards share shard 0's CSR, counts,
                               // picks and sends, so the tick has no exchange at all -- G
                               // column tiles of one GPU's job (DESIGN.md "Column tiles")
    bool rowmode = false;      // row layout (G > 1): sender rows move between shards
    int64_t pair_cap = 0, msg_cap = 0;
    gsp::RowxState rowx;       // row layout: the exchange's count ring and posted sizes
    int32_t *h_err = nullptr;  // pinned mirror of the shards' capacity flags, refreshed by an
                               // async copy at the end of every gsp_scale_step call
    int32_t max_segment = INT32_MAX;     // segments past kMaxSegment take the HBM sort
    ncclComm_t comm = nullptr; // one shard per process when set
    int64_t width = 0;         // n rounded up to 2048 * G
    int64_t stride = 0;        // columns per shard
    int32_t tick = 0;
    bool timing = true;
    int policy = 5;            // bit 0 nt own row, bit 1 nt sender rows, bit 2 pipelined loads
    int merge = 1;             // 1 packed 16-bit merge, 0 per-entry form
    int32_t lds_pad = 0;       // GSP_TEST_SCALE_LDS_PAD: extra LDS per tick-kernel workgroup
    std::vector<Shard> local;  // shards held by this engine (1, or G for an in-process group)
    gsp::DevBuf<gsp::ScaleTickArgs> long_tpl;   // [local][2]: every tile's args by tick parity
                                                // (scale_long_kernel)
    std::vector<int32_t> h_fail, h_start;
    bool joins = false;        // a join schedule is set (some node starts after tick 0)
    gsp::JoinPlan plan;        // the joiners of every start tick
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

    gsp::ScaleTickArgs args(Shard &sh, int32_t t) const {
        gsp::ScaleTickArgs a{};
        a.prev = sh.table[(t + 1) & 1].p;
        a.cur = sh.table[t & 1].p;
        a.remote = rowmode ? reinterpret_cast<const uint16_t *>(sh.x.recv_rows.p) : nullptr;
        a.stride = stride;
        a.n = p.n;
        a.col0 = sh.col0;
        a.row0 = sh.row0;
        a.rows = sh.rows;
        a.tick = t;
        a.tremove = p.tremove;
        a.fanout = p.fanout;
        a.h0 = p.h0;
        a.nt_own = policy & 1;
        a.nt_src = (policy >> 1) & 1;
        a.pipe = (policy >> 2) & 1;
        a.lds_pad = lds_pad;
        a.tfail = p.tfail;
        a.swim = p.swim;
        a.count_rounds = rowmode || sh.g == 0;
        a.seed = p.seed;
        a.fail_tick = sh.fail_tick.p;
        a.start_tick = joins ? sh.start_tick.p : nullptr;
        a.drop_pct = gsp::drop_at(p.policy, p.drop_pct, t);
        a.drop_prev = gsp::drop_at(p.policy, p.drop_pct, t - 1);
        // node 0's row of tick t - 1 (the JOINREP payload): the local row 0, or the copy the
        // row layout's shard 0 broadcast
        a.intro = (rowmode && sh.row0 != 0) ? sh.intro_buf.p : sh.table[(t + 1) & 1].p;
        a.intro_list = p.policy.intro_list;
        const Shard &s0 = local[0];
        // shared: cnt_all[tick parity][G][n], so this tick's slice counts never overwrite the
        // tick-(t - 1) counts another shard's JOINREP still reads
        const size_t gn = size_t(shards) * size_t(p.n);
        a.intro_cnt = sliced ? (shared ? s0.cnt_all.p + size_t((t + 1) & 1) * gn : sh.cnt_all.p) : nullptr;
        a.shards = shards;
        a.shard = sh.g;
        a.own_hb = sh.own_hb.p;
        a.cnt_prev = (shared ? s0 : sh).cnt_total[(t + 1) & 1].p;
        a.cnt_cur = shared ? s0.cnt_all.p + size_t(t & 1) * gn + size_t(sh.g) * size_t(p.n)
                  : sliced ? sh.cnt_slice.p : sh.cnt_total[t & 1].p;
        a.off = (shared ? s0 : sh).off.p;
        a.csr_src = (shared ? s0 : sh).csr_src.p;
        a.csr_slot = rowmode ? sh.x.csr_slot.p : nullptr;
        a.out_dst = sh.out_dst.p;
        a.deg = sh.deg.p;
        a.ping = (shared ? s0 : sh).ping.p;
        a.bitmap = shared ? s0.bitmap.p + size_t(sh.g - rank) * size_t(p.n) * size_t(stride / 8) : sh.bitmap.p;
        a.dig = sh.dig.p + size_t(t) * gsp::kDigSlots * gsp::kDigFields;
        a.err = local[0].err.p;        // one flag for every shard held here
        a.max_segment = max_segment;
        a.ev = sh.ev.args();
        // the rows this tile's CSR defers (k > kMaxSegment): appended by the CSR's owner only
        a.long_list = &sh == &owner(sh) ? long_list(sh, t) : nullptr;
        return a;
    }

    // the shard whose receiver CSR a shard reads (shared column tiles: shard 0's)
    const Shard &owner(const Shard &sh) const { return shared ? local[0] : sh; }
    int32_t *long_list(const Shard &sh, int32_t t) const {
        const Shard &o = owner(sh);
        return o.long_list.p + size_t(t & 1) * size_t(1 + o.rows);
    }

    gsp::ScaleResolveArgs resolve_args(Shard &sh, int32_t t) const {
        gsp::ScaleResolveArgs r{};
        r.n = p.n;
        r.fanout = p.fanout;
        r.tick = t;
        r.shard = sh.g;
        r.shards = shards;
        r.count_rounds = sh.g == 0;
        r.stride = stride;
        r.seed = p.seed;
        r.fail_tick = sh.fail_tick.p;
        r.start_tick = joins ? sh.start_tick.p : nullptr;
        r.drop_pct = gsp::drop_at(p.policy, p.drop_pct, t);
        r.cnt_all = shared ? local[0].cnt_all.p + size_t(t & 1) * size_t(shards) * size_t(p.n) : sh.cnt_all.p;
        r.cnt_total = sh.cnt_total[t & 1].p;
        r.bitmap = sh.bitmap.p;
        r.picks = sh.picks.p;
        r.tiled = shared ? 1 : 0;       // one launch resolves the ranks of every local shard
        r.tile_lo = rank;
        r.tile_cnt = int32_t(local.size());
        r.tile_bytes = int64_t(p.n) * (stride / 8);
        r.swim = p.swim;
        r.ping = sh.ping.p;
        r.out_dst = sh.out_dst.p;
        r.deg = sh.deg.p;
        r.dig = sh.dig.p + size_t(t) * gsp::kDigSlots * gsp::kDigFields;
        return r;
    }
};

namespace gsp {

// Failure schedule: the same Philox draws as the oracle (policy.hpp; DESIGN.md "Scale mode").
std::vector<int32_t> scale_fail_ticks(const gsp_scale_params &p) {
    return fail_ticks(p.policy, p.n, p.seed, p.fail_mode, p.fail_tick, p.fail_ppm);
}

int validate_scale_params(const gsp_scale_params *p) {
    GSP_REQUIRE(p, GSP_ERR_INVALID, "scale params NULL");
    GSP_REQUIRE(p->n >= 2 && p->n <= (1 << 21), GSP_ERR_INVALID, "n=%d outside [2, 2^21]", p->n);
    GSP_REQUIRE(p->fanout >= 1 && p->fanout <= 16, GSP_ERR_INVALID, "fanout=%d outside [1,16]",
                p->fanout);
    GSP_REQUIRE(p->tremove >= 1 && p->tremove <= 31, GSP_ERR_INVALID,
                "tremove=%d outside [1,31] (ts is stored mod 32)", p->tremove);
    GSP_REQUIRE(p->h0 >= 1 && p->h0 < 2047, GSP_ERR_INVALID, "h0=%d outside [1,2046]", p->h0);
    GSP_REQUIRE(p->drop_pct >= 0 && p->drop_pct <= 100, GSP_ERR_INVALID, "drop_pct=%d", p->drop_pct);
    GSP_REQUIRE(p->fail_mode >= 0 && p->fail_mode <= 2, GSP_ERR_INVALID, "fail_mode=%d", p->fail_mode);
    GSP_REQUIRE(p->tfail == 0 || (p->tfail >= 1 && p->tfail < p->tremove), GSP_ERR_INVALID,
                "tfail=%d: 0 (off) or 1..tremove-1", p->tfail);
    GSP_REQUIRE(p->swim >= 0 && p->swim <= 8, GSP_ERR_INVALID, "swim=%d: 0 (off) or 1..8 paths",
                p->swim);
    GSP_REQUIRE(p->max_ticks >= 1 && int64_t(p->h0) + p->max_ticks <= 2047, GSP_ERR_RANGE,
                "h0 + max_ticks = %d exceeds the 11-bit packed heartbeat (2047)",
                p->h0 + p->max_ticks);
    GSP_REQUIRE(p->events >= 0 && p->events <= 15, GSP_ERR_INVALID, "events=%d: 0 off, 1 all, or an OR of GSP_EVENTS_*", p->events);
    GSP_REQUIRE(p->event_cap >= 0, GSP_ERR_INVALID, "event_cap=%lld", (long long)p->event_cap);
    return validate_policy(p->policy, p->n);
}

}  // namespace gsp

namespace {

int shard_alloc(gsp_scale *s, Shard &sh) {
    const int32_t n = s->p.n;
    const size_t rows = size_t(sh.rows);
    const size_t tab = rows * size_t(s->stride);
    hipStream_t st = s->st;
    // tests / A/B (GSP_TEST_SCALE_CONTIG=1): the tables in physically contiguous memory
    const char *contig = std::getenv("GSP_TEST_SCALE_CONTIG");
    for (int b = 0; b < 2; ++b) {
        if (contig && std::atoi(contig)) GSP_HIP(sh.table[b].alloc_contiguous(tab));
        else GSP_HIP(sh.table[b].alloc(tab));
        GSP_HIP(sh.cnt_total[b].alloc(size_t(n)));
        GSP_HIP(hipMemsetAsync(sh.cnt_total[b].p, 0, size_t(n) * 4, st));
    }
    GSP_HIP(sh.own_hb.alloc(rows));
    GSP_HIP(sh.fail_tick.alloc(size_t(n)));
    GSP_HIP(sh.out_dst.alloc(rows * s->p.fanout));
    if (s->p.swim > 0) {
        GSP_HIP(sh.ping.alloc(rows));
        GSP_HIP(hipMemsetAsync(sh.ping.p, 0xFF, rows * 4, st));   // -1: no probe yet
    }
    GSP_HIP(sh.deg.alloc(size_t(n)));
    GSP_HIP(sh.off.alloc(rows + 1));
    GSP_HIP(sh.fill.alloc(rows));
    GSP_HIP(sh.csr_src.alloc(size_t(n) * s->p.fanout));
    GSP_HIP(sh.err.alloc(1));
    GSP_HIP(sh.tile_sum.alloc(size_t(n) / 4096 + 1));
    if (!s->shared || &sh == &s->local[0]) {
        GSP_HIP(sh.long_list.alloc(2 * (rows + 1)));
        GSP_HIP(hipMemsetAsync(sh.long_list.p, 0, 2 * (rows + 1) * 4, st));
    }
    if (s->sliced && (!s->shared || &sh == &s->local[0])) {
        GSP_HIP(sh.cnt_slice.alloc(size_t(n)));
        GSP_HIP(sh.cnt_all.alloc(size_t(n) * s->shards * (s->shared ? 2 : 1)));
        // + 1: the capacity flag rides the all-reduce MAX of the picks (exchange_picks)
        GSP_HIP(sh.picks.alloc(size_t(n) * (s->p.fanout + (s->p.swim > 0 ? 1 : 0)) + 1));
        // shared: every local shard's bitmap, one region each (the resolve reads them all)
        GSP_HIP(sh.bitmap.alloc(size_t(n) * size_t(s->stride / 8) * (s->shared ? s->local.size() : 1)));
    }
    if (s->rowmode)
        GSP_HIP(sh.x.alloc(s->shards, s->pair_cap, s->msg_cap, int32_t(s->stride / 4), false,
                           s->comm != nullptr, int64_t(n) * s->p.fanout, st));
    const size_t dig = size_t(s->p.max_ticks + 1) * gsp::kDigSlots * gsp::kDigFields;
    GSP_HIP(sh.dig.alloc(dig));
    GSP_HIP(hipMemsetAsync(sh.dig.p, 0, dig * sizeof(unsigned long long), st));
    if (s->p.events) GSP_HIP(sh.ev.alloc(s->p.events, s->p.event_cap, st));
    if (s->joins) {
        GSP_HIP(sh.start_tick.alloc(size_t(n)));
        GSP_HIP(hipMemcpyAsync(sh.start_tick.p, s->h_start.data(), size_t(n) * 4, hipMemcpyHostToDevice, st));
        const size_t nj = std::max<size_t>(1, s->plan.joiners.size());
        GSP_HIP(sh.joiners.alloc(nj));
        GSP_HIP(sh.join_ok.alloc(nj));
        if (!s->plan.joiners.empty())
            GSP_HIP(hipMemcpyAsync(sh.joiners.p, s->plan.joiners.data(), s->plan.joiners.size() * 4,
                                   hipMemcpyHostToDevice, st));
        // a late joiner's row is read (empty) at its start tick from either buffer, and the
        // init kernel skips the rows that have not started
        for (int b = 0; b < 2; ++b) GSP_HIP(hipMemsetAsync(sh.table[b].p, 0, tab * sizeof(uint16_t), st));
        if (s->rowmode && sh.row0 != 0) GSP_HIP(sh.intro_buf.alloc(size_t(s->stride)));
    }
    GSP_HIP(hipMemsetAsync(sh.own_hb.p, 0, rows * 4, st));
    GSP_HIP(hipMemsetAsync(sh.deg.p, 0, size_t(n) * 4, st));
    GSP_HIP(hipMemsetAsync(sh.err.p, 0, 4, st));
    GSP_HIP(hipMemcpyAsync(sh.fail_tick.p, s->h_fail.data(), size_t(n) * 4, hipMemcpyHostToDevice, st));
    return GSP_OK;
}

// all-gather of every shard's per-row slice counts into every shard's cnt_all[G][n]
int exchange_counts(gsp_scale *s, int32_t t) {
    const size_t n = size_t(s->p.n);
    if (s->shared) {                      // the local shards wrote shard 0's cnt_all directly
        if (!s->comm) return GSP_OK;
        // in place: this rank's block of local-shard rows -> every rank's cnt_all[t & 1]
        const size_t L = s->local.size();
        int32_t *all = s->local[0].cnt_all.p + size_t(t & 1) * size_t(s->shards) * n;
        GSP_NCCL(ncclAllGather(all + size_t(s->rank) * n, all, L * n, ncclInt32, s->comm, s->st));
        return GSP_OK;
    }
    if (s->comm) {
        Shard &sh = s->local[0];
        GSP_NCCL(ncclAllGather(sh.cnt_slice.p, sh.cnt_all.p, n, ncclInt32, s->comm, s->st));
        return GSP_OK;
    }
    for (Shard &dst : s->local)
        for (Shard &src : s->local)
            GSP_HIP(hipMemcpyAsync(dst.cnt_all.p + size_t(src.g) * n, src.cnt_slice.p, n * 4,
                                   hipMemcpyDeviceToDevice, s->st));
    return GSP_OK;
}

// all-reduce MAX of the resolved picks (each pick is resolved by exactly one shard)
int exchange_picks(gsp_scale *s) {
    const size_t cnt = size_t(s->p.n) * (s->p.fanout + (s->p.swim > 0 ? 1 : 0));
    if (s->comm) {
        // the capacity flag (0, or the tick that overflowed) rides along in slot cnt, so every
        // rank's next tick kernels stop together and every rank's sync reports it
        Shard &sh = s->local[0];
        GSP_HIP(hipMemcpyAsync(sh.picks.p + cnt, sh.err.p, 4, hipMemcpyDeviceToDevice, s->st));
        GSP_NCCL(ncclAllReduce(sh.picks.p, sh.picks.p, cnt + 1, ncclInt32, ncclMax, s->comm, s->st));
        GSP_HIP(hipMemcpyAsync(sh.err.p, sh.picks.p + cnt, 4, hipMemcpyDeviceToDevice, s->st));
        return GSP_OK;
    }
    Shard &root = s->local[0];
    for (size_t i = 1; i < s->local.size(); ++i)
        GSP_HIP(gsp::launch_max_into(root.picks.p, s->local[i].picks.p, int64_t(cnt), s->st));
    for (size_t i = 1; i < s->local.size(); ++i)
        GSP_HIP(hipMemcpyAsync(s->local[i].picks.p, root.picks.p, cnt * 4, hipMemcpyDeviceToDevice,
                               s->st));
    return GSP_OK;
}

// message generation for tick t (columns: after the slices are merged)
int resolve_sends(gsp_scale *s, int32_t t) {
    const double G = double(s->shards), n = double(s->p.n);
    if (s->shared) {                     // one resolve over every local shard's ranks, one finalize
        if (s->comm) {                   // ... between the ranks' count and pick collectives
            const double W = G / double(s->local.size());
            s->perf.xgmi_bytes += (W - 1.0) * (n * 4.0 * double(s->local.size()) +
                                               2.0 * n * (s->p.fanout + (s->p.swim > 0 ? 1 : 0)) * 4.0 / W);
            if (int rc = exchange_counts(s, t)) return rc;
        }
        GSP_HIP(gsp::launch_scale_resolve(s->resolve_args(s->local[0], t), s->st));
        if (s->comm)
            if (int rc = exchange_picks(s)) return rc;
        GSP_HIP(gsp::launch_scale_finalize(s->resolve_args(s->local[0], t), s->st));
        return GSP_OK;
    }
    // egress per shard of ring collectives: all-gather (G-1)/G of G*n*4 B, all-reduce
    // 2 (G-1)/G of n*f*4 B
    s->perf.xgmi_bytes += double(s->local.size()) * (G - 1.0) *
                          (n * 4.0 + 2.0 * n * (s->p.fanout + (s->p.swim > 0 ? 1 : 0)) * 4.0 / G);
    if (int rc = exchange_counts(s, t)) return rc;
    for (Shard &sh : s->local) GSP_HIP(gsp::launch_scale_resolve(s->resolve_args(sh, t), s->st));
    if (int rc = exchange_picks(s)) return rc;
    for (Shard &sh : s->local) GSP_HIP(gsp::launch_scale_finalize(s->resolve_args(sh, t), s->st));
    return GSP_OK;
}

// Row layout: every shard's member counts of tick t (cnt_total[t & 1], own rows only) reach
// every shard -- the merges digest of tick t + 1 reads them for remote senders.
int exchange_row_counts(gsp_scale *s, int32_t t) {
    if (s->comm) {
        Shard &sh = s->local[0];
        int32_t *cnt = sh.cnt_total[t & 1].p;
        GSP_NCCL(ncclGroupStart());
        for (int32_t g = 0; g < s->shards; ++g) {
            const int32_t r0 = gsp::rowx_row0(g, s->p.n, s->shards);
            const int32_t nr = gsp::rowx_row0(g + 1, s->p.n, s->shards) - r0;
            GSP_NCCL(ncclBroadcast(cnt + r0, cnt + r0, size_t(nr), ncclInt32, g, s->comm, s->st));
        }
        GSP_NCCL(ncclGroupEnd());
        s->perf.xgmi_bytes += double(sh.rows) * 4.0 * double(s->shards - 1);
        return GSP_OK;
    }
    for (Shard &src : s->local)
        for (Shard &dst : s->local) {
            if (&src == &dst) continue;
            GSP_HIP(hipMemcpyAsync(dst.cnt_total[t & 1].p + src.row0, src.cnt_total[t & 1].p + src.row0,
                                   size_t(src.rows) * 4, hipMemcpyDeviceToDevice, s->st));
            s->perf.xgmi_bytes += double(src.rows) * 4.0;
        }
    return GSP_OK;
}

// Row layout: the sender rows of tick t_sent's cross-shard messages move to their receivers'
// shards (rowx_host.cpp); every shard gets the receiver CSR of tick t_sent + 1.
int exchange_rows(gsp_scale *s, int32_t t_sent) {
    gsp::RowxJob job{s->p.n, s->shards, s->p.fanout, int32_t(s->stride / 4), false, s->pair_cap,
                     s->msg_cap, s->comm, s->st, t_sent + 1, &s->rowx};
    // a joiner's sends ramp up to F over its first ticks (its view grows): the joiners of the
    // last three send ticks count as new senders
    job.new_senders = s->joins ? s->plan.count(t_sent) + s->plan.count(t_sent - 1) + s->plan.count(t_sent - 2) : 0;
    job.drop_now = gsp::drop_at(s->p.policy, s->p.drop_pct, t_sent);
    job.drop_before = gsp::drop_at(s->p.policy, s->p.drop_pct, t_sent - 1);
    std::vector<gsp::RowxShard> v;
    for (Shard &sh : s->local)
        v.push_back(gsp::RowxShard{sh.g, sh.row0, sh.rows, sh.out_dst.p,
                                   reinterpret_cast<const uint64_t *>(sh.table[t_sent & 1].p),
                                   sh.deg.p, sh.off.p, sh.fill.p, sh.csr_src.p, sh.tile_sum.p,
                                   s->local[0].err.p, &sh.x});
    return gsp::rowx_exchange(job, v, &s->perf.xgmi_bytes);
}

// The capacity flag as last mirrored to the host (no synchronisation): a receiver with more
// than max_segment messages sets the flag to the tick, and every later tick kernel returns at
// once, so the job's state stays that of the tick before the overflow.  Every shard held by
// this engine reads one flag (shard 0's); with a communicator the flag is exchanged each tick
// (columns: inside the picks all-reduce, and every rank holds the same receiver segments; rows:
// all-reduced ahead of the tick kernels, and again with the exchange counts), so all ranks
// stop at the same tick and report it from their own flag.  Without a test's bound
// (GSP_TEST_MAX_SEGMENT) no segment overflows: segments past kMaxSegment are sorted in HBM.
int mirrored_err(gsp_scale *s) {
    for (size_t i = 0; i < s->local.size(); ++i)
    {
        const int32_t e = s->h_err[i];
        GSP_REQUIRE(!(e & gsp::kRowxErrBit), GSP_ERR_CAPACITY,
                    "row exchange at tick %d: a shard's rows or records passed the region capacity "
                    "or the size posted to RCCL; ticks after it did not run", e & ~gsp::kRowxErrBit);
        GSP_REQUIRE(e == 0, GSP_ERR_CAPACITY,
                    "a receiver got more than %d messages at tick %d; ticks after it did not run",
                    s->max_segment, e);
    }
    return GSP_OK;
}

int check_err(gsp_scale *s) {
    for (size_t i = 0; i < s->local.size(); ++i)
        GSP_HIP(hipMemcpyAsync(s->h_err + i, s->local[i].err.p, 4, hipMemcpyDeviceToHost, s->st));
    GSP_HIP(hipStreamSynchronize(s->st));
    return mirrored_err(s);
}

// The JOINREPs node 0 sends at tick t to the nodes that start at t + 1 (join_kernels.hpp):
// deg of the receivers (next tick's CSR) and the digest's sent / dropped of tick t; the row
// layout also broadcasts node 0's row of tick t to the other shards (the JOINREP payload).
int join_sends(gsp_scale *s, int32_t t) {
    const int64_t cnt = s->plan.count(t + 1);
    if (!s->joins || cnt == 0) return GSP_OK;
    for (Shard &sh : s->local) {
        if (s->shared && &sh != &s->local[0]) continue;   // one CSR (shard 0's deg)
        gsp::JoinSendArgs j{};
        j.joiners = sh.joiners.p + s->plan.first(t + 1);
        j.count = int32_t(cnt);
        j.tick = t;
        j.drop_pct = gsp::drop_at(s->p.policy, s->p.drop_pct, t);
        j.seed = s->p.seed;
        j.fail_tick = sh.fail_tick.p;
        j.lo = s->rowmode ? sh.row0 : 0;
        j.hi = s->rowmode ? sh.row0 + sh.rows : s->p.n;
        j.ok = sh.join_ok.p + s->plan.first(t + 1);
        j.deg = sh.deg.p;
        const bool counts = s->rowmode || sh.g == 0;
        unsigned long long *dig = sh.dig.p + size_t(t) * gsp::kDigSlots * gsp::kDigFields;
        j.sent = counts ? dig + gsp::kDigSent : nullptr;
        j.dropped = counts ? dig + gsp::kDigDropped : nullptr;
        GSP_HIP(gsp::launch_join_send(j, s->st));
    }
    if (!s->rowmode || s->shards == 1) return GSP_OK;
    // node 0's row of tick t -> intro_buf of every other shard
    const size_t bytes = size_t(s->stride) * sizeof(uint16_t);
    if (s->comm) {
        Shard &sh = s->local[0];
        void *buf = sh.row0 == 0 ? static_cast<void *>(sh.table[t & 1].p) : static_cast<void *>(sh.intro_buf.p);
        GSP_NCCL(ncclBroadcast(buf, buf, bytes, ncclUint8, 0, s->comm, s->st));
        s->perf.xgmi_bytes += sh.row0 == 0 ? double(bytes) * double(s->shards - 1) : 0.0;
        return GSP_OK;
    }
    const Shard &root = s->local[0];
    for (Shard &sh : s->local)
        if (sh.row0 != 0) {
            GSP_HIP(hipMemcpyAsync(sh.intro_buf.p, root.table[t & 1].p, bytes, hipMemcpyDeviceToDevice, s->st));
            s->perf.xgmi_bytes += double(bytes);
        }
    return GSP_OK;
}

// the delivered JOINREPs of tick t into every local shard's receiver CSR (after the scan)
int join_scatter(gsp_scale *s, int32_t t) {
    const int64_t cnt = s->plan.count(t);
    if (!s->joins || cnt == 0) return GSP_OK;
    for (Shard &sh : s->local) {
        if (s->shared && &sh != &s->local[0]) continue;
        GSP_HIP(gsp::launch_join_scatter(sh.joiners.p + s->plan.first(t), sh.join_ok.p + s->plan.first(t),
                                         int32_t(cnt), s->rowmode ? sh.row0 : 0,
                                         s->rowmode ? sh.rows : s->p.n, sh.off.p, sh.fill.p, sh.csr_src.p,
                                         s->rowmode ? sh.x.csr_slot.p : nullptr, s->st));
    }
    return GSP_OK;
}

int collect_timing(gsp_scale *s) {
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
    if (s->rowmode)
        if (int rc = gsp::rowx_collect(s->rowx, &s->perf.xgmi_bytes)) return rc;
    return GSP_OK;
}

// scale_long_kernel's tile table: each tile's args at both tick parities (digest base at tick
// 0, every tile reading its CSR owner's deferred-row list).  The long kernel patches only
// tick, drop_pct, drop_prev and the digest offset per tick (scale_kernels.hip,
// scale_long_kernel); every other field is read from here, so the table is rebuilt whenever
// a field it copies can change after create (gsp_scale_set_cache_policy: nt_own / nt_src /
// pipe).  An args field that changes per tick must join the kernel's patch list instead.
int upload_long_tpl(gsp_scale *s) {
    std::vector<gsp::ScaleTickArgs> tpl;
    for (Shard &sh : s->local)
        for (int32_t par = 0; par < 2; ++par) {
            gsp::ScaleTickArgs x = s->args(sh, 2 + par);
            x.dig = sh.dig.p;
            x.long_list = s->long_list(sh, par);
            tpl.push_back(x);
        }
    if (!s->long_tpl.p) GSP_HIP(s->long_tpl.alloc(tpl.size()));
    GSP_HIP(hipStreamSynchronize(s->st));          // no queued launch still reads the old table
    GSP_HIP(hipMemcpy(s->long_tpl.p, tpl.data(), tpl.size() * sizeof(gsp::ScaleTickArgs),
                      hipMemcpyHostToDevice));
    return GSP_OK;
}

int scale_build(const gsp_scale_params *p, int device, int32_t shards, int32_t rank,
                int32_t local_shards, const void *nccl_id, int32_t layout, gsp_scale **out) {
    GSP_REQUIRE(out, GSP_ERR_INVALID, "gsp_scale: out is NULL");
    *out = nullptr;
    if (int rc = gsp::validate_scale_params(p)) return rc;
    GSP_REQUIRE(shards >= 1 && shards <= 64 && rank >= 0 && rank + local_shards <= shards,
                GSP_ERR_INVALID, "gsp_scale: shards=%d rank=%d", shards, rank);
    int ndev = 0;
    GSP_HIP(hipGetDeviceCount(&ndev));
    GSP_REQUIRE(device >= 0 && device < ndev, GSP_ERR_HIP, "gsp_scale: device %d of %d", device, ndev);
    GSP_HIP(hipSetDevice(device));
    std::unique_ptr<gsp_scale> s(new gsp_scale);
    s->p = *p;
    s->device = device;
    s->shards = shards;
    s->rank = rank;
    GSP_REQUIRE(layout == GSP_SHARD_COLUMNS || layout == GSP_SHARD_ROWS, GSP_ERR_INVALID,
                "gsp_scale: layout %d", layout);
    GSP_REQUIRE(shards <= p->n, GSP_ERR_INVALID, "gsp_scale: %d shards for %d nodes", shards, p->n);
    // a communicator always runs the sharded protocol (with one rank it exercises RCCL alone)
    const bool sharded = shards > 1 || nccl_id != nullptr;
    s->sliced = sharded && layout == GSP_SHARD_COLUMNS;
    // shared: every shard of this engine shares shard 0's CSR / counts / picks / sends -- an
    // in-process group (all shards here), or the column tiles of one rank (a communicator over
    // shards / local_shards ranks, each holding local_shards consecutive shards)
    s->shared = s->sliced && local_shards > 1 && (nccl_id != nullptr || local_shards == shards);
    GSP_REQUIRE(nccl_id == nullptr || local_shards == 1 ||
                    (layout == GSP_SHARD_COLUMNS && shards % local_shards == 0 && rank % local_shards == 0),
                GSP_ERR_INVALID, "gsp_scale: %d local tiles of %d column shards at shard %d", local_shards,
                shards, rank);
    if (const char *sx = std::getenv("GSP_TEST_SCALE_SHARED")) s->shared = s->shared && std::atoi(sx) != 0;
    s->rowmode = sharded && layout == GSP_SHARD_ROWS;
    const int64_t unit = int64_t(gsp::kChunk) * (s->sliced ? shards : 1);
    s->width = (int64_t(p->n) + unit - 1) / unit * unit;
    s->stride = s->width / (s->sliced ? shards : 1);
    if (s->rowmode) {
        // a sender row goes to a shard at most once: rows_max pairs always fit; large rows get
        // the expected share 1 - (1 - 1/G)^f with margin (a tick beyond it fails loudly)
        int32_t rows_max = 0;
        for (int32_t g = 0; g < shards; ++g)
            rows_max = std::max(rows_max, gsp::rowx_row0(g + 1, p->n, shards) - gsp::rowx_row0(g, p->n, shards));
        const double share = 1.0 - std::pow(1.0 - 1.0 / shards, double(p->fanout));
        s->pair_cap = std::min<int64_t>(rows_max, int64_t(rows_max * share * 1.1) + 1024);
        s->msg_cap = std::min<int64_t>(int64_t(rows_max) * p->fanout,
                                       int64_t(double(rows_max) * p->fanout / shards * 1.25) + 4096);
    }
    s->h_fail = gsp::scale_fail_ticks(*p);
    s->h_start = gsp::start_ticks(p->policy, p->n);
    s->joins = p->policy.step_rate > 0 && *std::max_element(s->h_start.begin(), s->h_start.end()) > 0;
    if (s->joins) s->plan = gsp::join_plan(s->h_start, p->max_ticks + 1);
    if (const char *pol = std::getenv("GSP_TEST_SCALE_POLICY")) s->policy = std::atoi(pol) & 7;
    if (const char *pad = std::getenv("GSP_TEST_SCALE_LDS_PAD")) s->lds_pad = std::max(0, std::min(65536, std::atoi(pad)));
    if (const char *m = std::getenv("GSP_TEST_SCALE_MERGE")) s->merge = std::atoi(m) ? 1 : 0;
    if (!s->sliced) {
        // the fused kernel keeps the row's presence bitmap (and the event stage) in LDS next
        // to 8.3 KB of statics
        GSP_REQUIRE(gsp::scale_lds_bytes(s->stride, false, p->events != 0) <= 48 * 1024, GSP_ERR_CAPACITY,
                    "row bitmap of %lld B%s exceeds the LDS budget (one-GPU full view n <= 393216, "
                    "327680 with events)", (long long)(s->stride / 8), p->events ? " + event stage" : "");
    }
    if (const char *ms = std::getenv("GSP_TEST_MAX_SEGMENT"))   // tests only: force overflows
        s->max_segment = std::max(1, std::atoi(ms));
    GSP_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
    GSP_HIP(hipHostMalloc(reinterpret_cast<void **>(&s->h_err), size_t(local_shards) * 4));
    std::memset(s->h_err, 0, size_t(local_shards) * 4);
    if (s->rowmode) {
        GSP_HIP(s->rowx.init(shards, nccl_id != nullptr));
    }
    if (nccl_id) {
        ncclUniqueId id;
        std::memcpy(&id, nccl_id, sizeof id);
        GSP_NCCL(ncclCommInitRank(&s->comm, shards / local_shards, id, rank / local_shards));
    }
    s->local.resize(size_t(local_shards));
    for (int32_t i = 0; i < local_shards; ++i) {
        Shard &sh = s->local[size_t(i)];
        sh.g = rank + i;
        sh.col0 = s->sliced ? int32_t(int64_t(sh.g) * s->stride) : 0;
        sh.row0 = s->rowmode ? gsp::rowx_row0(sh.g, p->n, shards) : 0;
        sh.rows = s->rowmode ? gsp::rowx_row0(sh.g + 1, p->n, shards) - sh.row0 : p->n;
        if (int rc = shard_alloc(s.get(), sh)) return rc;
    }
    if (int rc = upload_long_tpl(s.get())) return rc;
    for (Shard &sh : s->local) GSP_HIP(gsp::launch_scale_init(s->args(sh, 0), s->sliced, s->st));
    if (s->sliced)
        if (int rc = resolve_sends(s.get(), 0)) return rc;
    if (s->rowmode)
        if (int rc = exchange_row_counts(s.get(), 0)) return rc;
    if (int rc = join_sends(s.get(), 0)) return rc;
    GSP_HIP(hipStreamSynchronize(s->st));
    *out = s.release();
    return GSP_OK;
}

}  // namespace

extern "C" {

int gsp_scale_create(const gsp_scale_params *p, int device, gsp_scale **out) {
    return scale_build(p, device, 1, 0, 1, nullptr, GSP_SHARD_COLUMNS, out);
}

int gsp_scale_create_group(const gsp_scale_params *p, int device, int32_t shards, gsp_scale **out) {
    return scale_build(p, device, shards, 0, shards, nullptr, GSP_SHARD_COLUMNS, out);
}

int gsp_scale_create_group_layout(const gsp_scale_params *p, int device, int32_t shards,
                                  int32_t layout, gsp_scale **out) {
    return scale_build(p, device, shards, 0, shards, nullptr, layout, out);
}

int gsp_scale_create_rank_layout(const gsp_scale_params *p, int device, int32_t rank,
                                 int32_t world, const void *nccl_id, int32_t layout, gsp_scale **out) {
    GSP_REQUIRE(nccl_id || world == 1, GSP_ERR_INVALID, "gsp_scale_create_rank_layout: NULL nccl id");
    return scale_build(p, device, world, rank, 1, nccl_id, layout, out);
}

int gsp_scale_create_rank_tiled(const gsp_scale_params *p, int device, int32_t rank, int32_t world,
                                int32_t tiles, const void *nccl_id, gsp_scale **out) {
    GSP_REQUIRE(nccl_id, GSP_ERR_INVALID, "gsp_scale_create_rank_tiled: NULL nccl id");
    GSP_REQUIRE(tiles >= 1 && world >= 1 && int64_t(world) * tiles <= 64, GSP_ERR_INVALID,
                "gsp_scale_create_rank_tiled: world=%d tiles=%d", world, tiles);
    return scale_build(p, device, world * tiles, rank * tiles, tiles, nccl_id, GSP_SHARD_COLUMNS, out);
}

int gsp_scale_nccl_id(void *out, size_t cap) {
    GSP_REQUIRE(out && cap >= sizeof(ncclUniqueId), GSP_ERR_INVALID,
                "gsp_scale_nccl_id: need %zu bytes", sizeof(ncclUniqueId));
    ncclUniqueId id;
    GSP_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof id);
    return GSP_OK;
}

int gsp_scale_create_rank(const gsp_scale_params *p, int device, int32_t rank, int32_t world,
                          const void *nccl_id, gsp_scale **out) {
    GSP_REQUIRE(nccl_id || world == 1, GSP_ERR_INVALID, "gsp_scale_create_rank: NULL nccl id");
    return scale_build(p, device, world, rank, 1, nccl_id, GSP_SHARD_COLUMNS, out);
}

int gsp_scale_destroy(gsp_scale *s) {
    if (!s) return GSP_OK;
    (void)hipSetDevice(s->device);
    if (s->st) (void)hipStreamSynchronize(s->st);
    for (auto &t : s->pending) {
        s->free_events.push_back(t.a);
        s->free_events.push_back(t.b);
        s->free_events.push_back(t.c);
    }
    for (hipEvent_t e : s->free_events) (void)hipEventDestroy(e);
    for (Shard &sh : s->local) sh.release();
    s->long_tpl.release();
    if (s->comm) (void)ncclCommDestroy(s->comm);
    s->rowx.release();
    if (s->h_err) (void)hipHostFree(s->h_err);
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
    return GSP_OK;
}

int gsp_scale_step(gsp_scale *s, int32_t ticks) {
    GSP_REQUIRE(s && ticks >= 0, GSP_ERR_INVALID, "gsp_scale_step: bad argument");
    GSP_REQUIRE(s->tick + ticks <= s->p.max_ticks, GSP_ERR_RANGE,
                "gsp_scale_step: tick %d beyond max_ticks %d", s->tick + ticks, s->p.max_ticks);
    GSP_HIP(hipSetDevice(s->device));
    // an earlier call's ticks overflowed: one process stops here at once; ranks of a
    // communicator do not (the async mirror lands at different times on different ranks, and a
    // rank that returned would leave the others in a collective) -- their kernels already run
    // no row, the row exchange returns the error on every rank at the same tick, and sync
    // reports it
    if (!s->comm)
        if (int rc = mirrored_err(s)) return rc;
    const int32_t n = s->p.n;
    const int64_t slots = int64_t(n) * s->p.fanout;
    for (int32_t i = 0; i < ticks; ++i) {
        const int32_t t = s->tick + 1;
        gsp_scale::Timed tm{};
        if (s->timing) {
            tm = {s->event(), s->event(), s->event()};
            GSP_HIP(hipEventRecord(tm.a, s->st));
        }
        if (s->rowmode) {
            if (int rc = exchange_rows(s, t - 1)) return rc;
            // ranks (row shards): a segment past a test's bound stops every rank's tick t, not
            // only the holder's -- the flag is checked ahead of the tick kernel and all-reduced
            // (ADVICE r03); unbounded otherwise (long segments are sorted in HBM)
            if (s->comm && s->max_segment < INT32_MAX) {
                Shard &sh = s->local[0];
                GSP_HIP(gsp::launch_segment_check(sh.off.p, sh.rows, s->max_segment, sh.err.p, t, s->st));
                GSP_NCCL(ncclAllReduce(sh.err.p, sh.err.p, 1, ncclInt32, ncclMax, s->comm, s->st));
            }
        } else {
            for (Shard &sh : s->local) {
                if (s->shared && &sh != &s->local[0]) continue;   // one CSR for every shard
                GSP_HIP(gsp::launch_exclusive_scan(sh.deg.p, sh.off.p, n, sh.tile_sum.p, s->st));
                GSP_HIP(hipMemsetAsync(sh.fill.p, 0, size_t(n) * 4, s->st));
                GSP_HIP(gsp::launch_scatter(sh.out_dst.p, slots, s->p.fanout, 0, sh.off.p, sh.fill.p,
                                            sh.csr_src.p, s->st));
                GSP_HIP(hipMemsetAsync(sh.deg.p, 0, size_t(n) * 4, s->st));
            }
        }
        if (int rc = join_scatter(s, t)) return rc;
        if (s->timing) GSP_HIP(hipEventRecord(tm.b, s->st));
        for (Shard &sh : s->local)
            GSP_HIP(gsp::launch_scale_tick(s->args(sh, t), s->sliced, s->merge, s->st));
        // the rows with more than kMaxSegment messages the launches above deferred (usually
        // none: one short launch per tick)
        GSP_HIP(gsp::launch_scale_long(s->args(s->local[0], t), s->long_tpl.p, int32_t(s->local.size()),
                                       s->sliced, s->st));
        if (s->timing) {
            GSP_HIP(hipEventRecord(tm.c, s->st));
            s->pending.push_back(tm);
        }
        if (s->sliced)
            if (int rc = resolve_sends(s, t)) return rc;
        if (s->rowmode)
            if (int rc = exchange_row_counts(s, t)) return rc;
        if (int rc = join_sends(s, t)) return rc;
        s->tick = t;
        s->perf.ticks++;
    }
    for (size_t i = 0; i < s->local.size(); ++i)     // read by the next call, never waited on
        GSP_HIP(hipMemcpyAsync(s->h_err + i, s->local[i].err.p, 4, hipMemcpyDeviceToHost, s->st));
    return GSP_OK;
}

int gsp_scale_sync(gsp_scale *s) {
    GSP_REQUIRE(s, GSP_ERR_INVALID, "gsp_scale_sync: NULL");
    GSP_HIP(hipSetDevice(s->device));
    GSP_HIP(hipStreamSynchronize(s->st));
    if (int rc = collect_timing(s)) return rc;
    return check_err(s);
}

int gsp_scale_tick(gsp_scale *s, int32_t *tick) {
    GSP_REQUIRE(s && tick, GSP_ERR_INVALID, "gsp_scale_tick: NULL");
    *tick = s->tick;
    return GSP_OK;
}

// Digest of this engine's shards.  Per-column quantities (joins, removes, hash) are summed
// over the shards held here; per-row quantities are counted by shard 0 only.  In the
// one-process-per-GPU case the job's digest is the sum of every rank's digest.
int gsp_scale_digest_get(gsp_scale *s, int32_t t, gsp_scale_digest *out) {
    GSP_REQUIRE(s && out, GSP_ERR_INVALID, "gsp_scale_digest_get: NULL");
    GSP_REQUIRE(t >= 0 && t <= s->tick, GSP_ERR_INVALID, "gsp_scale_digest_get: tick %d", t);
    if (int rc = gsp_scale_sync(s)) return rc;
    unsigned long long f[gsp::kDigFields] = {0};
    std::vector<unsigned long long> h(size_t(gsp::kDigSlots) * gsp::kDigFields);
    for (Shard &sh : s->local) {
        GSP_HIP(hipMemcpy(h.data(), sh.dig.p + size_t(t) * h.size(), h.size() * 8,
                          hipMemcpyDeviceToHost));
        for (int sl = 0; sl < gsp::kDigSlots; ++sl)
            for (int k = 0; k < gsp::kDigFields; ++k) f[k] += h[size_t(sl) * gsp::kDigFields + k];
    }
    out->tick = t;
    out->node_rounds = int64_t(f[gsp::kDigRounds]);
    out->merges = int64_t(f[gsp::kDigMerges]);
    out->sent = int64_t(f[gsp::kDigSent]);
    out->dropped = int64_t(f[gsp::kDigDropped]);
    out->delivered = int64_t(f[gsp::kDigDelivered]);
    out->joins = int64_t(f[gsp::kDigJoins]);
    out->removes = int64_t(f[gsp::kDigRemoves]);
    out->event_hash = f[gsp::kDigHash];
    return GSP_OK;
}

// Row r of the current table as seen by this engine: every column held by its shards
// (the whole row on one GPU or in an in-process group; zeros outside this rank's slice).
int gsp_scale_row(gsp_scale *s, int32_t r, uint16_t *buf, int32_t cap) {
    GSP_REQUIRE(s && buf && r >= 0 && r < s->p.n, GSP_ERR_INVALID, "gsp_scale_row: row %d", r);
    GSP_REQUIRE(cap >= s->p.n, GSP_ERR_INVALID, "gsp_scale_row: cap %d < n %d", cap, s->p.n);
    if (int rc = gsp_scale_sync(s)) return rc;
    std::memset(buf, 0, size_t(s->p.n) * 2);
    // a crashed row stops at its fail tick: read the buffer of the last tick it ran
    const int32_t last = std::min(s->tick, s->h_fail[size_t(r)]);
    if (s->rowmode) {
        for (Shard &sh : s->local)
            if (r >= sh.row0 && r < sh.row0 + sh.rows) {
                GSP_HIP(hipMemcpy(buf, sh.table[last & 1].p + size_t(r - sh.row0) * size_t(s->stride),
                                  size_t(s->p.n) * 2, hipMemcpyDeviceToHost));
                return GSP_OK;
            }
        GSP_REQUIRE(false, GSP_ERR_INVALID, "gsp_scale_row: row %d is not held by this rank", r);
    }
    for (Shard &sh : s->local) {
        const int64_t c0 = sh.col0;
        const int64_t cnt = std::min<int64_t>(s->stride, int64_t(s->p.n) - c0);
        if (cnt <= 0) continue;
        const uint16_t *src = sh.table[last & 1].p + size_t(r) * size_t(s->stride);
        GSP_HIP(hipMemcpy(buf + c0, src, size_t(cnt) * 2, hipMemcpyDeviceToHost));
    }
    return GSP_OK;
}

int gsp_scale_own_hb(gsp_scale *s, int32_t r, int32_t *hb) {
    GSP_REQUIRE(s && hb && r >= 0 && r < s->p.n, GSP_ERR_INVALID, "gsp_scale_own_hb: bad row");
    if (int rc = gsp_scale_sync(s)) return rc;
    for (Shard &sh : s->local)
        if (r >= sh.row0 && r < sh.row0 + sh.rows) {
            GSP_HIP(hipMemcpy(hb, sh.own_hb.p + (r - sh.row0), 4, hipMemcpyDeviceToHost));
            return GSP_OK;
        }
    GSP_REQUIRE(false, GSP_ERR_INVALID, "gsp_scale_own_hb: row %d is not held by this rank", r);
    return GSP_OK;
}

int gsp_scale_messages(gsp_scale *s, int32_t *dst, int64_t cap, int64_t *n) {
    GSP_REQUIRE(s && n, GSP_ERR_INVALID, "gsp_scale_messages: NULL");
    if (int rc = gsp_scale_sync(s)) return rc;
    if (!s->rowmode) {
        const int64_t slots = int64_t(s->p.n) * s->p.fanout;
        *n = slots;
        if (dst && cap > 0)
            GSP_HIP(hipMemcpy(dst, s->local[0].out_dst.p, size_t(std::min(cap, slots)) * 4,
                              hipMemcpyDeviceToHost));
        return GSP_OK;
    }
    int64_t total = 0;          // row layout: the slots of the rows held here, in row order
    for (Shard &sh : s->local) {
        const int64_t slots = int64_t(sh.rows) * s->p.fanout;
        if (dst && total < cap)
            GSP_HIP(hipMemcpy(dst + total, sh.out_dst.p, size_t(std::min(cap - total, slots)) * 4,
                              hipMemcpyDeviceToHost));
        total += slots;
    }
    *n = total;
    return GSP_OK;
}

int gsp_scale_perf_get(gsp_scale *s, gsp_scale_perf *out) {
    GSP_REQUIRE(s && out, GSP_ERR_INVALID, "gsp_scale_perf_get: NULL");
    if (int rc = gsp_scale_sync(s)) return rc;
    gsp_scale_digest d{};
    if (s->tick > 0)
        if (int rc = gsp_scale_digest_get(s, s->tick, &d)) return rc;
    // algorithmic HBM bytes of the tick kernel(s) of this engine at the last tick: every
    // processed row reads its own row and writes it back (2 * stride * 2 B per shard), reads
    // one sender row per delivered message (stride * 2 B) and its CSR entry (4 B)
    const double rows = double(2 * d.node_rounds + d.delivered);
    s->perf.bytes_per_tick = (rows * double(s->stride) * 2.0 + double(d.delivered) * 4.0) *
                             double(s->sliced ? s->local.size() : 1);
    *out = s->perf;
    return GSP_OK;
}

int gsp_scale_set_timing(gsp_scale *s, int32_t on) {
    GSP_REQUIRE(s, GSP_ERR_INVALID, "gsp_scale_set_timing: NULL");
    s->timing = on != 0;
    return GSP_OK;
}

int gsp_scale_set_cache_policy(gsp_scale *s, int32_t policy) {
    GSP_REQUIRE(s && policy >= 0 && policy <= 7, GSP_ERR_INVALID,
                "gsp_scale_set_cache_policy: policy %d", policy);
    s->policy = policy;
    return upload_long_tpl(s);
}

int gsp_scale_set_merge(gsp_scale *s, int32_t packed) {
    GSP_REQUIRE(s, GSP_ERR_INVALID, "gsp_scale_set_merge: NULL");
    s->merge = packed ? 1 : 0;
    return GSP_OK;
}

int gsp_scale_layout(gsp_scale *s, int32_t *shards, int32_t *rank, int64_t *stride) {
    GSP_REQUIRE(s, GSP_ERR_INVALID, "gsp_scale_layout: NULL");
    if (shards) *shards = s->shards;
    if (rank) *rank = s->rank;
    if (stride) *stride = s->stride;
    return GSP_OK;
}

int gsp_scale_drain_events(gsp_scale *s, uint64_t *buf, int64_t cap, int64_t *n, int64_t *lost) {
    GSP_REQUIRE(s && n && cap >= 0 && (buf || cap == 0), GSP_ERR_INVALID, "gsp_scale_drain_events: bad argument");
    GSP_REQUIRE(s->p.events, GSP_ERR_INVALID, "gsp_scale_drain_events: the engine records no events "
                "(gsp_scale_params.events = 0)");
    if (int rc = gsp_scale_sync(s)) return rc;
    int64_t total = 0, dropped = 0;
    for (Shard &sh : s->local) GSP_HIP(sh.ev.drain(buf, cap, &total, &dropped));
    *n = total;
    if (lost) *lost = dropped;
    return GSP_OK;
}

int gsp_scale_hip_stream(gsp_scale *s, void **stream) {
    GSP_REQUIRE(s && stream, GSP_ERR_INVALID, "gsp_scale_hip_stream: NULL");
    *stream = reinterpret_cast<void *>(s->st);
    return GSP_OK;
}

}  // extern "C"
