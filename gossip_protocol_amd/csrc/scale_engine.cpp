// gossip_protocol_amd/csrc/scale_engine.cpp -- host side of the SCALE engine (C ABI).
//
// One tick = four stream-ordered launches, no host synchronisation:
//   exclusive_scan(deg) -> off   receiver CSR offsets from last tick's destination counts
//   scatter(out_dst)   -> csr    sender ids per receiver (order fixed later by the kernel)
//   memset(deg)                  re-armed for this tick's sends
//   scale_tick_kernel            merge + ops + events + send, one workgroup per row
// The membership table lives in HBM as two [rows][stride] uint16 buffers (tick parity).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "common.hpp"
#include "philox.hpp"
#include "scale_kernels.hpp"

struct gsp_scale {
    gsp_scale_params p{};
    int device = 0;
    hipStream_t st = nullptr;
    int64_t stride = 0;
    int32_t rows = 0, row0 = 0;
    int32_t tick = 0;
    bool timing = true;
    gsp::DevBuf<uint16_t> table[2];
    gsp::DevBuf<int32_t> own_hb, fail_tick, cnt[2], out_dst, deg, off, fill, csr_src, err, tile_sum;
    // cache policy of the row streams (scale_kernels.hpp); 1 = non-temporal own row, the
    // fastest in the A/B of profiles/r01/r2/ab_policy.json (7.52 vs 7.89 ms per launch)
    int policy = 1;
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

    gsp::ScaleTickArgs args(int32_t t) const {
        gsp::ScaleTickArgs a{};
        a.prev = table[(t + 1) & 1].p;
        a.cur = table[t & 1].p;
        a.stride = stride;
        a.n = p.n;
        a.row0 = row0;
        a.rows = rows;
        a.tick = t;
        a.tremove = p.tremove;
        a.fanout = p.fanout;
        a.drop_pct = p.drop_pct;
        a.h0 = p.h0;
        a.seed = p.seed;
        a.fail_tick = fail_tick.p;
        a.own_hb = own_hb.p;
        a.cnt_prev = cnt[(t + 1) & 1].p;
        a.cnt_cur = cnt[t & 1].p;
        a.off = off.p;
        a.csr_src = csr_src.p;
        a.out_dst = out_dst.p;
        a.deg = deg.p;
        a.dig = dig.p + size_t(t) * gsp::kDigSlots * gsp::kDigFields;
        a.err = err.p;
        return a;
    }
};

namespace gsp {

// Failure schedule: the same Philox draws as the oracle (DESIGN.md "Scale mode").
std::vector<int32_t> scale_fail_ticks(const gsp_scale_params &p) {
    std::vector<int32_t> f(size_t(p.n), 0x7FFFFFFF);
    if (p.fail_mode == 1) {
        for (int32_t r = 0; r < p.n; ++r)
            if (draw_u31(kDomainFail, p.seed, uint32_t(p.fail_tick), uint32_t(r), 0, 0) % 1000000u <
                uint32_t(p.fail_ppm))
                f[size_t(r)] = p.fail_tick;
    } else if (p.fail_mode == 2) {
        const int64_t m = int64_t(p.n) * p.fail_ppm / 1000000;
        const uint32_t start = draw_u31(kDomainFail, p.seed, uint32_t(p.fail_tick), 0xFFFFFFFFu, 0, 0) %
                               uint32_t(p.n);
        for (int64_t i = 0; i < m; ++i) f[size_t((start + i) % uint32_t(p.n))] = p.fail_tick;
    }
    return f;
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
    GSP_REQUIRE(p->max_ticks >= 1 && int64_t(p->h0) + p->max_ticks <= 2047, GSP_ERR_RANGE,
                "h0 + max_ticks = %d exceeds the 11-bit packed heartbeat (2047)",
                p->h0 + p->max_ticks);
    return GSP_OK;
}

}  // namespace gsp

namespace {

int scale_alloc(gsp_scale *s) {
    const int32_t n = s->p.n;
    const size_t tab = size_t(s->rows) * size_t(s->stride);
    for (int b = 0; b < 2; ++b) {
        GSP_HIP(s->table[b].alloc(tab));
        GSP_HIP(s->cnt[b].alloc(size_t(n)));
        GSP_HIP(hipMemsetAsync(s->cnt[b].p, 0, size_t(n) * 4, s->st));
    }
    GSP_HIP(s->own_hb.alloc(size_t(s->rows)));
    GSP_HIP(s->fail_tick.alloc(size_t(n)));
    GSP_HIP(s->out_dst.alloc(size_t(s->rows) * s->p.fanout));
    GSP_HIP(s->deg.alloc(size_t(n)));
    GSP_HIP(s->off.alloc(size_t(n) + 1));
    GSP_HIP(s->fill.alloc(size_t(n)));
    GSP_HIP(s->csr_src.alloc(size_t(n) * s->p.fanout));
    GSP_HIP(s->err.alloc(1));
    GSP_HIP(s->tile_sum.alloc(size_t(n) / 4096 + 1));
    const size_t dig = size_t(s->p.max_ticks + 1) * gsp::kDigSlots * gsp::kDigFields;
    GSP_HIP(s->dig.alloc(dig));
    GSP_HIP(hipMemsetAsync(s->dig.p, 0, dig * sizeof(unsigned long long), s->st));
    GSP_HIP(hipMemsetAsync(s->own_hb.p, 0, size_t(s->rows) * 4, s->st));
    GSP_HIP(hipMemsetAsync(s->deg.p, 0, size_t(n) * 4, s->st));
    GSP_HIP(hipMemsetAsync(s->err.p, 0, 4, s->st));
    GSP_HIP(hipMemcpyAsync(s->fail_tick.p, s->h_fail.data(), size_t(n) * 4, hipMemcpyHostToDevice,
                           s->st));
    return GSP_OK;
}

int check_err(gsp_scale *s) {
    int32_t err = 0;
    GSP_HIP(hipMemcpyAsync(&err, s->err.p, 4, hipMemcpyDeviceToHost, s->st));
    GSP_HIP(hipStreamSynchronize(s->st));
    GSP_REQUIRE(err == 0, GSP_ERR_CAPACITY,
                "a receiver got more than %d messages in one tick", gsp::kMaxSegment);
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
    return GSP_OK;
}

}  // namespace

extern "C" {

int gsp_scale_create(const gsp_scale_params *p, int device, gsp_scale **out) {
    GSP_REQUIRE(out, GSP_ERR_INVALID, "gsp_scale_create: out is NULL");
    *out = nullptr;
    if (int rc = gsp::validate_scale_params(p)) return rc;
    int ndev = 0;
    GSP_HIP(hipGetDeviceCount(&ndev));
    GSP_REQUIRE(device >= 0 && device < ndev, GSP_ERR_HIP, "gsp_scale_create: device %d of %d",
                device, ndev);
    GSP_HIP(hipSetDevice(device));
    std::unique_ptr<gsp_scale> s(new gsp_scale);
    s->p = *p;
    s->device = device;
    s->stride = (int64_t(p->n) + gsp::kChunk - 1) / gsp::kChunk * gsp::kChunk;
    s->rows = p->n;
    s->row0 = 0;
    s->h_fail = gsp::scale_fail_ticks(*p);
    if (const char *pol = std::getenv("GSP_SCALE_POLICY")) s->policy = std::atoi(pol) & 3;
    GSP_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
    if (int rc = scale_alloc(s.get())) return rc;
    const size_t lds = gsp::scale_lds_bytes(s->stride);
    // the row's presence bitmap lives in LDS next to 8.3 KB of static scratch
    GSP_REQUIRE(lds <= 48 * 1024, GSP_ERR_CAPACITY,
                "row bitmap of %zu B exceeds the LDS budget (full view n <= 393216)", lds);
    gsp::ScaleTickArgs a = s->args(0);
    GSP_HIP(gsp::launch_scale_init(a, s->st));
    GSP_HIP(hipStreamSynchronize(s->st));
    s->tick = 0;
    *out = s.release();
    return GSP_OK;
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
    for (int b = 0; b < 2; ++b) { s->table[b].release(); s->cnt[b].release(); }
    for (auto *b : {&s->own_hb, &s->fail_tick, &s->out_dst, &s->deg, &s->off, &s->fill,
                    &s->csr_src, &s->err, &s->tile_sum})
        b->release();
    s->dig.release();
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
    return GSP_OK;
}

int gsp_scale_step(gsp_scale *s, int32_t ticks) {
    GSP_REQUIRE(s && ticks >= 0, GSP_ERR_INVALID, "gsp_scale_step: bad argument");
    GSP_REQUIRE(s->tick + ticks <= s->p.max_ticks, GSP_ERR_RANGE,
                "gsp_scale_step: tick %d beyond max_ticks %d", s->tick + ticks, s->p.max_ticks);
    GSP_HIP(hipSetDevice(s->device));
    const int32_t n = s->p.n;
    const int64_t slots = int64_t(s->rows) * s->p.fanout;
    for (int32_t i = 0; i < ticks; ++i) {
        const int32_t t = s->tick + 1;
        gsp_scale::Timed tm{};
        if (s->timing) {
            tm = {s->event(), s->event(), s->event()};
            GSP_HIP(hipEventRecord(tm.a, s->st));
        }
        GSP_HIP(gsp::launch_exclusive_scan(s->deg.p, s->off.p, n, s->tile_sum.p, s->st));
        GSP_HIP(hipMemsetAsync(s->fill.p, 0, size_t(n) * 4, s->st));
        GSP_HIP(gsp::launch_scatter(s->out_dst.p, slots, s->p.fanout, s->row0, s->off.p, s->fill.p,
                                    s->csr_src.p, s->st));
        GSP_HIP(hipMemsetAsync(s->deg.p, 0, size_t(n) * 4, s->st));
        if (s->timing) GSP_HIP(hipEventRecord(tm.b, s->st));
        GSP_HIP(gsp::launch_scale_tick(s->args(t), s->policy, s->st));
        if (s->timing) {
            GSP_HIP(hipEventRecord(tm.c, s->st));
            s->pending.push_back(tm);
        }
        s->tick = t;
        s->perf.ticks++;
    }
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

int gsp_scale_digest_get(gsp_scale *s, int32_t t, gsp_scale_digest *out) {
    GSP_REQUIRE(s && out, GSP_ERR_INVALID, "gsp_scale_digest_get: NULL");
    GSP_REQUIRE(t >= 0 && t <= s->tick, GSP_ERR_INVALID, "gsp_scale_digest_get: tick %d", t);
    if (int rc = gsp_scale_sync(s)) return rc;
    std::vector<unsigned long long> h(size_t(gsp::kDigSlots) * gsp::kDigFields);
    GSP_HIP(hipMemcpy(h.data(), s->dig.p + size_t(t) * h.size(), h.size() * 8,
                      hipMemcpyDeviceToHost));
    unsigned long long f[gsp::kDigFields] = {0};
    for (int sl = 0; sl < gsp::kDigSlots; ++sl)
        for (int k = 0; k < gsp::kDigFields; ++k) f[k] += h[size_t(sl) * gsp::kDigFields + k];
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

int gsp_scale_row(gsp_scale *s, int32_t r, uint16_t *buf, int32_t cap) {
    GSP_REQUIRE(s && buf && r >= s->row0 && r < s->row0 + s->rows, GSP_ERR_INVALID,
                "gsp_scale_row: row %d not on this engine", r);
    GSP_REQUIRE(cap >= s->p.n, GSP_ERR_INVALID, "gsp_scale_row: cap %d < n %d", cap, s->p.n);
    if (int rc = gsp_scale_sync(s)) return rc;
    // a crashed row stops at its fail tick: read the buffer of the last tick it ran
    const int32_t last = std::min(s->tick, s->h_fail[size_t(r)]);
    const uint16_t *src = s->table[last & 1].p + size_t(r - s->row0) * size_t(s->stride);
    GSP_HIP(hipMemcpy(buf, src, size_t(s->p.n) * 2, hipMemcpyDeviceToHost));
    return GSP_OK;
}

int gsp_scale_own_hb(gsp_scale *s, int32_t r, int32_t *hb) {
    GSP_REQUIRE(s && hb && r >= s->row0 && r < s->row0 + s->rows, GSP_ERR_INVALID,
                "gsp_scale_own_hb: bad row");
    if (int rc = gsp_scale_sync(s)) return rc;
    GSP_HIP(hipMemcpy(hb, s->own_hb.p + (r - s->row0), 4, hipMemcpyDeviceToHost));
    return GSP_OK;
}

int gsp_scale_messages(gsp_scale *s, int32_t *dst, int64_t cap, int64_t *n) {
    GSP_REQUIRE(s && n, GSP_ERR_INVALID, "gsp_scale_messages: NULL");
    if (int rc = gsp_scale_sync(s)) return rc;
    const int64_t slots = int64_t(s->rows) * s->p.fanout;
    *n = slots;
    if (dst && cap > 0)
        GSP_HIP(hipMemcpy(dst, s->out_dst.p, size_t(std::min(cap, slots)) * 4,
                          hipMemcpyDeviceToHost));
    return GSP_OK;
}

int gsp_scale_perf_get(gsp_scale *s, gsp_scale_perf *out) {
    GSP_REQUIRE(s && out, GSP_ERR_INVALID, "gsp_scale_perf_get: NULL");
    if (int rc = gsp_scale_sync(s)) return rc;
    gsp_scale_digest d{};
    if (s->tick > 0) {
        if (int rc = gsp_scale_digest_get(s, s->tick, &d)) return rc;
    }
    // algorithmic HBM bytes of the fused kernel at the last tick: every processed row
    // reads its own row and writes it back (2 * stride * 2 B), reads one sender row per
    // delivered message (stride * 2 B) and its CSR entry (4 B)
    s->perf.bytes_per_tick = double(2 * d.node_rounds + d.delivered) * double(s->stride) * 2.0 +
                             double(d.delivered) * 4.0;
    *out = s->perf;
    return GSP_OK;
}

int gsp_scale_set_timing(gsp_scale *s, int32_t on) {
    GSP_REQUIRE(s, GSP_ERR_INVALID, "gsp_scale_set_timing: NULL");
    s->timing = on != 0;
    return GSP_OK;
}

int gsp_scale_set_cache_policy(gsp_scale *s, int32_t policy) {
    GSP_REQUIRE(s && policy >= 0 && policy <= 3, GSP_ERR_INVALID,
                "gsp_scale_set_cache_policy: policy %d", policy);
    s->policy = policy;
    return GSP_OK;
}

int gsp_scale_hip_stream(gsp_scale *s, void **stream) {
    GSP_REQUIRE(s && stream, GSP_ERR_INVALID, "gsp_scale_hip_stream: NULL");
    *stream = reinterpret_cast<void *>(s->st);
    return GSP_OK;
}

}  // extern "C"
