// gossip_protocol_amd/csrc/pview_engine.cpp -- host side of the PARTIAL-VIEW engine (C ABI).
//
// Same tick structure as the full-view engine (scan -> scatter -> tick kernel), with the
// bounded view table [2][n][V] of 8-byte entries.  Row-sharded multi-GPU operation is
// provided by row_shard.cpp on top of these pieces.
#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "common.hpp"
#include "philox.hpp"
#include "pview_kernels.hpp"
#include "scale_kernels.hpp"

namespace gsp {
std::vector<int32_t> scale_fail_ticks(const gsp_scale_params &p);
}

struct gsp_pview {
    gsp_pview_params p{};
    int device = 0;
    hipStream_t st = nullptr;
    int32_t tick = 0;
    bool timing = true;
    gsp::DevBuf<uint64_t> table[2];
    gsp::DevBuf<int32_t> len[2], own_hb, fail_tick, out_dst, deg, off, fill, csr_src, err, tile_sum;
    gsp::DevBuf<unsigned long long> dig;
    std::vector<int32_t> h_fail;
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

    gsp::PviewTickArgs args(int32_t t) const {
        gsp::PviewTickArgs a{};
        a.prev = table[(t + 1) & 1].p;
        a.cur = table[t & 1].p;
        a.remote = nullptr;
        a.n = p.n;
        a.view = p.view;
        a.inbox = p.inbox;
        a.fanout = p.fanout;
        a.tick = t;
        a.tremove = p.tremove;
        a.drop_pct = p.drop_pct;
        a.h0 = p.h0;
        a.row0 = 0;
        a.rows = p.n;
        a.seed = p.seed;
        a.fail_tick = fail_tick.p;
        a.own_hb = own_hb.p;
        a.len_prev = len[(t + 1) & 1].p;
        a.len_cur = len[t & 1].p;
        a.off = off.p;
        a.csr_src = csr_src.p;
        a.csr_slot = nullptr;
        a.out_dst = out_dst.p;
        a.deg = deg.p;
        a.dig = dig.p + size_t(t) * gsp::kPvDigSlots * gsp::kPvFields;
        a.err = err.p;
        return a;
    }
};

namespace {

int pview_validate(const gsp_pview_params *p) {
    GSP_REQUIRE(p, GSP_ERR_INVALID, "pview params NULL");
    GSP_REQUIRE(p->n >= 2 && p->n < (1 << 21), GSP_ERR_INVALID, "n=%d outside [2, 2^21 - 1]", p->n);
    GSP_REQUIRE(p->view >= 1 && p->view <= gsp::kPvMaxView, GSP_ERR_INVALID, "view=%d outside [1, %d]",
                p->view, gsp::kPvMaxView);
    GSP_REQUIRE(p->inbox >= 1 && p->inbox <= gsp::kPvMaxInbox, GSP_ERR_INVALID,
                "inbox=%d outside [1, %d]", p->inbox, gsp::kPvMaxInbox);
    GSP_REQUIRE(p->fanout >= 1 && p->fanout <= 16, GSP_ERR_INVALID, "fanout=%d outside [1,16]",
                p->fanout);
    GSP_REQUIRE(p->tremove >= 1 && p->tremove <= 31, GSP_ERR_INVALID, "tremove=%d outside [1,31]",
                p->tremove);
    GSP_REQUIRE(p->h0 >= 1 && p->h0 < 2047, GSP_ERR_INVALID, "h0=%d", p->h0);
    GSP_REQUIRE(p->drop_pct >= 0 && p->drop_pct <= 100, GSP_ERR_INVALID, "drop_pct=%d", p->drop_pct);
    GSP_REQUIRE(p->fail_mode >= 0 && p->fail_mode <= 2, GSP_ERR_INVALID, "fail_mode=%d", p->fail_mode);
    GSP_REQUIRE(p->max_ticks >= 1 && int64_t(p->h0) + p->max_ticks <= 2047, GSP_ERR_RANGE,
                "h0 + max_ticks exceeds the 11-bit packed heartbeat");
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
    int32_t err = 0;
    GSP_HIP(hipMemcpy(&err, s->err.p, 4, hipMemcpyDeviceToHost));
    GSP_REQUIRE(err == 0, GSP_ERR_CAPACITY, "a receiver got more than 1024 messages in one tick");
    return GSP_OK;
}

}  // namespace

extern "C" {

int gsp_pview_create(const gsp_pview_params *p, int device, gsp_pview **out) {
    GSP_REQUIRE(out, GSP_ERR_INVALID, "gsp_pview_create: out is NULL");
    *out = nullptr;
    if (int rc = pview_validate(p)) return rc;
    int ndev = 0;
    GSP_HIP(hipGetDeviceCount(&ndev));
    GSP_REQUIRE(device >= 0 && device < ndev, GSP_ERR_HIP, "gsp_pview_create: device %d of %d",
                device, ndev);
    GSP_HIP(hipSetDevice(device));
    std::unique_ptr<gsp_pview> s(new gsp_pview);
    s->p = *p;
    s->device = device;
    gsp_scale_params fp{};
    fp.n = p->n; fp.fail_mode = p->fail_mode; fp.fail_tick = p->fail_tick;
    fp.fail_ppm = p->fail_ppm; fp.seed = p->seed;
    s->h_fail = gsp::scale_fail_ticks(fp);
    GSP_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
    const int32_t n = p->n;
    const size_t tab = size_t(n) * size_t(p->view);
    for (int b = 0; b < 2; ++b) {
        GSP_HIP(s->table[b].alloc(tab));
        GSP_HIP(s->len[b].alloc(size_t(n)));
        GSP_HIP(hipMemsetAsync(s->len[b].p, 0, size_t(n) * 4, s->st));
    }
    GSP_HIP(s->own_hb.alloc(size_t(n)));
    GSP_HIP(s->fail_tick.alloc(size_t(n)));
    GSP_HIP(s->out_dst.alloc(size_t(n) * p->fanout));
    GSP_HIP(s->deg.alloc(size_t(n)));
    GSP_HIP(s->off.alloc(size_t(n) + 1));
    GSP_HIP(s->fill.alloc(size_t(n)));
    GSP_HIP(s->csr_src.alloc(size_t(n) * p->fanout));
    GSP_HIP(s->err.alloc(1));
    GSP_HIP(s->tile_sum.alloc(size_t(n) / 4096 + 1));
    const size_t dig = size_t(p->max_ticks + 1) * gsp::kPvDigSlots * gsp::kPvFields;
    GSP_HIP(s->dig.alloc(dig));
    GSP_HIP(hipMemsetAsync(s->dig.p, 0, dig * 8, s->st));
    GSP_HIP(hipMemsetAsync(s->own_hb.p, 0, size_t(n) * 4, s->st));
    GSP_HIP(hipMemsetAsync(s->deg.p, 0, size_t(n) * 4, s->st));
    GSP_HIP(hipMemsetAsync(s->err.p, 0, 4, s->st));
    GSP_HIP(hipMemcpyAsync(s->fail_tick.p, s->h_fail.data(), size_t(n) * 4, hipMemcpyHostToDevice,
                           s->st));
    GSP_HIP(gsp::launch_pview_init(s->args(0), s->st));
    GSP_HIP(hipStreamSynchronize(s->st));
    *out = s.release();
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
    for (hipEvent_t e : s->free_events) (void)hipEventDestroy(e);
    for (int b = 0; b < 2; ++b) { s->table[b].release(); s->len[b].release(); }
    for (auto *x : {&s->own_hb, &s->fail_tick, &s->out_dst, &s->deg, &s->off, &s->fill,
                    &s->csr_src, &s->err, &s->tile_sum})
        x->release();
    s->dig.release();
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
    return GSP_OK;
}

int gsp_pview_step(gsp_pview *s, int32_t ticks) {
    GSP_REQUIRE(s && ticks >= 0, GSP_ERR_INVALID, "gsp_pview_step: bad argument");
    GSP_REQUIRE(s->tick + ticks <= s->p.max_ticks, GSP_ERR_RANGE, "gsp_pview_step: beyond max_ticks");
    GSP_HIP(hipSetDevice(s->device));
    const int32_t n = s->p.n;
    const int64_t slots = int64_t(n) * s->p.fanout;
    for (int32_t i = 0; i < ticks; ++i) {
        const int32_t t = s->tick + 1;
        gsp_pview::Timed tm{};
        if (s->timing) {
            tm = {s->event(), s->event(), s->event()};
            GSP_HIP(hipEventRecord(tm.a, s->st));
        }
        GSP_HIP(gsp::launch_exclusive_scan(s->deg.p, s->off.p, n, s->tile_sum.p, s->st));
        GSP_HIP(hipMemsetAsync(s->fill.p, 0, size_t(n) * 4, s->st));
        GSP_HIP(gsp::launch_scatter(s->out_dst.p, slots, s->p.fanout, 0, s->off.p, s->fill.p,
                                    s->csr_src.p, s->st));
        GSP_HIP(hipMemsetAsync(s->deg.p, 0, size_t(n) * 4, s->st));
        if (s->timing) GSP_HIP(hipEventRecord(tm.b, s->st));
        GSP_HIP(gsp::launch_pview_tick(s->args(t), s->st));
        if (s->timing) {
            GSP_HIP(hipEventRecord(tm.c, s->st));
            s->pending.push_back(tm);
        }
        s->tick = t;
        s->perf.ticks++;
    }
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
    GSP_HIP(hipMemcpy(h.data(), s->dig.p + size_t(t) * h.size(), h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long f[gsp::kPvFields] = {0};
    for (int sl = 0; sl < gsp::kPvDigSlots; ++sl)
        for (int k = 0; k < gsp::kPvFields; ++k) f[k] += h[size_t(sl) * gsp::kPvFields + k];
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
    if (int rc = gsp_pview_sync(s)) return rc;
    const int32_t last = std::min(s->tick, s->h_fail[size_t(r)]);
    GSP_HIP(hipMemcpy(buf, s->table[last & 1].p + size_t(r) * s->p.view, size_t(s->p.view) * 8,
                      hipMemcpyDeviceToHost));
    GSP_HIP(hipMemcpy(len, s->len[last & 1].p + r, 4, hipMemcpyDeviceToHost));
    return GSP_OK;
}

int gsp_pview_own_hb(gsp_pview *s, int32_t r, int32_t *hb) {
    GSP_REQUIRE(s && hb && r >= 0 && r < s->p.n, GSP_ERR_INVALID, "gsp_pview_own_hb: bad row");
    if (int rc = gsp_pview_sync(s)) return rc;
    GSP_HIP(hipMemcpy(hb, s->own_hb.p + r, 4, hipMemcpyDeviceToHost));
    return GSP_OK;
}

int gsp_pview_messages(gsp_pview *s, int32_t *dst, int64_t cap, int64_t *n) {
    GSP_REQUIRE(s && n, GSP_ERR_INVALID, "gsp_pview_messages: NULL");
    if (int rc = gsp_pview_sync(s)) return rc;
    const int64_t slots = int64_t(s->p.n) * s->p.fanout;
    *n = slots;
    if (dst && cap > 0)
        GSP_HIP(hipMemcpy(dst, s->out_dst.p, size_t(std::min(cap, slots)) * 4, hipMemcpyDeviceToHost));
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
