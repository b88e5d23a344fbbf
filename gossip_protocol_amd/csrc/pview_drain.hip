// gossip_protocol_amd/csrc/pview_drain.hip -- the DRAIN-ALL partial view (inbox = 0).
//
// The reference drains every queued message (checkMessages, MP1Node.cpp:200-212).  With
// gsp_pview_params.inbox = 0 the partial view does too: a receiver sent k <= kPvMaxInbox
// messages runs in the tick kernels as before (they merge all k), and a receiver sent more
// (a "long" row: the receipt kernel lists it by class, pv_drain_class) runs here.
//
// The reference merges the k messages one after the other in ascending sender order into a
// list that may grow past the view (MP1Node.cpp:237-301), then applies TREMOVE (:339-348) and
// evicts down to V.  Every update of one message touches one id (the payload's ids are
// distinct, and a sender is in no payload of its own), so within a message the updates are
// independent, and across messages only each id's own updates need their order.
//
// Every update of the row becomes a TUPLE, u64: id << 32 | m << 17 | flag << 16 | val (val =
// hb << 5 | ts5): m = 0 the list (the own view at the start, flag = 1: the join count's test,
// or the list a previous chunk left), m = 1..kc message m (its payload entries, flag 0, val 0
// a no-op, and its sender, flag 1) -- built as runs of Vp = pow2(V) tuples, each sorted by id
// (views are stored sorted), merged bottom-up by merge path, and each id's run folded in
// message order: list tuple cur = val; payload cur = pv_merge (MP1Node.cpp:247-251 present,
// :282-301 absent and fresh); sender cur = pv_event (:237-243).  Then TREMOVE and eviction to
// V by two 256-bin histogram passes over the 16-bit prefix age << 11 | (2047 - hb) plus an
// id-order (or rotated-id) cut of the boundary bin; the new view is written in id order.
//
// LDS CLASSES (pview_drain_lds_kernel; rows of at most kDrainStage messages and 16,384 tuples):
// the row's tuples in one LDS buffer, merged and folded in place, 192 / 256 / 512 / 1024 lanes
// per row by size (pv_drain_class), the counts into the per-row digest record.
// HUB CLASS (pview_drain_hbm_kernel: the rest): runs sorted into 16 K-tuple blocks in LDS, the
// blocks merged in two HBM buffers per workgroup; messages are taken in chunks when they do
// not fit the buffers, the list carried between chunks as the m = 0 run; a list past the
// buffers stops the job (GSP_ERR_CAPACITY, err = tick | kDrainErrBit).
// Round 6 measured an LDS hash-table form of the LDS classes (the list as a hash table, one
// message per step, a radix select for the eviction): parity-green but 7.1 ms against the
// sort-and-fold's 4.4 ms on config 5's drain-all tick, so it was dropped.
//
// Both paths run the protocol extensions too: TFAIL (a payload holds the sender's members
// gossipable at t - 1), SWIM (the probe of t - 1 resolved before TREMOVE) and the JOINREP's
// bounded introducer list (node 0's gossipable members at the Philox ranks).
// Oracle: oracle/pview_oracle.c with inbox = 0 (the sequential fold over every message).
#include <cstdint>

#include "join_kernels.hpp"
#include "philox.hpp"
#include "pview_kernels.hpp"
#include "pview_rules.hpp"
#include "scale_kernels.hpp"
#include "wave_ops.hpp"

namespace gsp {
namespace {

constexpr int kHT = 1024;                       // threads per hub-kernel workgroup (16 waves)
constexpr int kHBlock = 16384;                  // HBM kernel: tuples sorted per LDS block
constexpr uint64_t kNone = ~0ull;               // an empty tuple: sorts last
constexpr uint32_t kNoId = 0xFFFFFFFFu;
constexpr int32_t kMaxChunk = 32767;            // messages per chunk: m is 15 bits
// sender staging word: s << 40 | kind bits | row
constexpr uint64_t kStageJoinRep = 1ull << 39;  // a JOINREP: node 0's sender entry, no payload
constexpr uint64_t kStageRemote = 1ull << 38;   // the payload row is a received (remote) row
constexpr uint64_t kStageRow = (1ull << 38) - 1;

// LDS of one workgroup: CAP tuples (LDS classes: the row's tuple buffer; hub kernel: a block of
// runs sorted in place, the segment sort keys), the senders of an LDS row, the eviction
// histogram, scan and digest words, the JOINREP payload mask.
template <int NT, int CAP>
struct alignas(16) DrainShared {
    static constexpr int kW = NT / 64;
    uint64_t buf[CAP + CAP / 16];               // skewed (SkewBuf), one pad per 16
    uint64_t stage[kDrainStage];                // LDS rows: the senders, staged (d_build)
    uint32_t hist[256];                         // eviction histogram
    uint32_t red[2][kW];                        // block scan words (two buffers, alternated)
    uint32_t sel[4];                            // selected bin, tuples still needed from it
    uint32_t tot[kW][8];                        // per-wave digest counts
    uint32_t jm[kPvMaxView / 32];               // JOINREP payload: slot p of node 0's view
};

// A workgroup barrier that orders LDS only: __syncthreads() would first wait for the wave's
// global stores (a row's output, digest atomics) to complete, which nothing here needs.
__device__ __forceinline__ void d_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// An LDS tuple buffer indexed with one pad word per 16 tuples: a lane's contiguous run of 16
// (the merge outputs, the fold's tuples) then starts 17 words after its neighbour's, so the
// 64-bit reads and writes of a wave hit distinct banks (a stride of 16 words is a 16-way
// conflict for ds_read_b64 and 32-way for ds_write_b64: MI355X_MICROARCH.md, LDS).
struct SkewBuf {
    uint64_t *p;
    __device__ __forceinline__ uint64_t &operator[](int32_t i) const { return p[i + (i >> 4)]; }
};

__device__ inline uint64_t d_tuple(uint32_t x, uint32_t m, uint32_t flag, uint32_t v) {
    return (uint64_t(x) << 32) | uint64_t((m << 17) | (flag << 16) | v);
}

// exclusive block scan over the workgroup; *total = the sum
template <int NT>
__device__ inline uint32_t d_scan(uint32_t v, uint32_t *total, uint32_t *buf) {
    const int32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if (lane == 63) buf[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int q = 0; q < NT / 64; ++q) {
        const uint32_t x = buf[q];
        before += q < wave ? x : 0u;
        all += x;
    }
    *total = all;
    return incl - v + before;
}

template <int NT>
__device__ inline uint32_t d_sum(uint32_t v, uint32_t *buf) {
    uint32_t total = 0;
    (void)d_scan<NT>(v, &total, buf);
    return total;
}

// Bitonic sort, ascending, of the P (a power of two) u64 keys at k (LDS or the workgroup's
// HBM scratch), every thread of the workgroup taking part.
template <int NT>
__device__ inline void d_bitonic(uint64_t *k, int32_t P) {
    for (int32_t size = 2; size <= P; size <<= 1)
        for (int32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (int32_t i = threadIdx.x; i < P / 2; i += NT) {
                const int32_t lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint64_t x = k[lo], y = k[hi];
                if ((x > y) == up) { k[lo] = y; k[hi] = x; }
            }
            __syncthreads();
        }
}

// the segment's (sender, row) pairs sorted by sender, in place (a JOINREP, sender
// kJoinRepSrc = -1, first: its sender is node 0); keys: P u64 of scratch
template <int NT>
__device__ void d_sort_segment(int32_t *src, int32_t *slot, int32_t k, int32_t P, int32_t row0,
                               uint64_t *keys) {
    for (int32_t i = threadIdx.x; i < P; i += NT) {
        uint64_t key = ~0ull;
        if (i < k) {
            const int32_t s = src[i];
            const int32_t sl = slot ? slot[i] : s - row0;
            key = (uint64_t(uint32_t(s + 1)) << 32) | uint64_t(uint32_t(sl));
        }
        keys[i] = key;
    }
    __syncthreads();
    d_bitonic<NT>(keys, P);
    for (int32_t i = threadIdx.x; i < k; i += NT) {
        const uint64_t key = keys[i];
        src[i] = int32_t(uint32_t(key >> 32)) - 1;
        if (slot) slot[i] = int32_t(uint32_t(key));
    }
    __syncthreads();
}

// The staging word of sender i of a segment: s << 40 | kind bits | its row (local, or the
// received row of a remote sender)
__device__ __forceinline__ uint64_t d_stage_word(const PviewTickArgs &a, int32_t s, const int32_t *slot, int32_t i) {
    if (s == kJoinRepSrc) return kStageJoinRep;
    const int32_t sl = slot ? slot[i] : s - a.row0;
    return (uint64_t(uint32_t(s)) << 40) | (sl >= 0 ? uint64_t(sl) : (kStageRemote | uint64_t(-int64_t(sl) - 1)));
}

// A JOINREP's payload with a bounded introducer list: node 0's members gossipable at t - 1
// (TFAIL), those at the Philox ranks pv_intro_mask draws -- as bits over the slots of node 0's
// view (jm[p / 32] bit p % 32).  Block-uniform; each lane looks at kPer contiguous slots.
template <int NT>
__device__ __forceinline__ void d_intro_mask(const PviewTickArgs &a, uint32_t r, uint32_t *jm, uint32_t *buf) {
    constexpr int kPer = (kPvMaxView + NT - 1) / NT;
    const int32_t tid = threadIdx.x;
    const uint32_t t = uint32_t(a.tick), tf = uint32_t(a.tfail), t5m1 = (t - 1u) & 31u;
    bool g[kPer];
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int32_t p = tid * kPer + q;
        g[q] = pv_gossiped(p < a.view ? a.intro[p] : kPvEmpty, tf, t5m1);
        c += g[q] ? 1u : 0u;
    }
    if (tid < kPvMaxView / 32) jm[tid] = 0u;
    uint32_t cnt0 = 0;
    uint32_t rank = d_scan<NT>(c, &cnt0, buf);                   // (its barrier orders the zeroing)
    const int32_t B = a.intro_list < int32_t(cnt0) ? a.intro_list : int32_t(cnt0);
    uint64_t cm[4];
    pv_intro_mask(a.seed, t - 1u, r, int32_t(cnt0), B, cm);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        if (!g[q]) continue;
        const int32_t p = tid * kPer + q;
        const uint32_t w = rank >> 6;
        const uint64_t word = w == 0 ? cm[0] : w == 1 ? cm[1] : w == 2 ? cm[2] : cm[3];
        if ((word >> (rank & 63u)) & 1ull) atomicOr(&jm[p >> 5], 1u << (p & 31));
        rank++;
    }
    __syncthreads();
}

// Diagnostics (GSP_PV_PROFILE=1): thread 0 adds the cycles of each phase of every 16th row a
// workgroup runs to prof[slot][8 + min(7, (k - 8) / 8)][phase] (pview_engine.cpp prints them).
struct DMark {
    unsigned long long *out = nullptr;
    uint64_t last = 0;
    __device__ __forceinline__ void init(unsigned long long *prof, int32_t i, int32_t k) {
        if (prof && threadIdx.x == 0 && (i & 15) == 0) {
            const int32_t b = 8 + ((k - 8) / 8 < 7 ? (k - 8) / 8 : 7);
            out = prof + ((blockIdx.x & 63u) * 16 + uint32_t(b)) * kPvProfPhases;
            atomicAdd(out + kPvProfPhases - 1, 1ull);
            last = clock64();
        }
    }
    __device__ __forceinline__ void mark(int phase) {
        if (out) {
            const uint64_t now = clock64();
            atomicAdd(out + phase, (unsigned long long)(now - last));
            last = now;
        }
    }
};

// Chunk step 2: the runs of messages [m0, m0 + kc) after the list (padded to Lp), into X;
// the senders staged in Y.  Returns this lane's count of non-empty payload entries (the
// digest's merges).
// jm: the JOINREP payload mask (d_intro_mask), or null (a JOINREP carries no payload).
template <int NT, class P>
__device__ __forceinline__ uint32_t d_build(const PviewTickArgs &a, P X, uint64_t *Y, int32_t L,
                                            int32_t Lp, int32_t m0, int32_t kc, int32_t Vp, int32_t lgV,
                                            const int32_t *src, const int32_t *slot, uint32_t r,
                                            const uint32_t *jm) {
    const int32_t tid = threadIdx.x, V = a.view;
    const uint32_t tf = uint32_t(a.tfail), t5m1 = (uint32_t(a.tick) - 1u) & 31u;
    for (int32_t i = tid; i < kc; i += NT) Y[i] = d_stage_word(a, src[m0 + i], slot, m0 + i);   // the senders
    for (int32_t i = L + tid; i < Lp; i += NT) X[i] = kNone;
    __syncthreads();
    const int32_t np = kc << lgV;                                // payload tuples
    const int32_t nt = np + ((kc + Vp - 1) >> lgV << lgV);       // + the senders' runs
    uint32_t merged = 0;
    constexpr int kB = 8;                                        // loads in flight per lane
    for (int32_t q0 = 0; q0 < nt; q0 += kB * NT) {
        uint64_t e[kB];
        uint32_t mi[kB];
        uint32_t cut = 0;                                        // bit u: slot not carried
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int32_t q = q0 + u * NT + tid;
            e[u] = kPvEmpty;
            mi[u] = 0;
            if (q < np) {
                const int32_t m = q >> lgV, pos = q & (Vp - 1);
                mi[u] = uint32_t(m);
                const uint64_t w = Y[m];
                if (pos < V && !(w & kStageJoinRep)) {
                    const int64_t row = int64_t(w & kStageRow);
                    const uint64_t *p = (w & kStageRemote) ? a.remote : a.prev;
                    e[u] = p[row * V + pos];
                } else if (pos < V && jm) {
                    e[u] = a.intro[pos];                         // the introducer list
                    cut |= ((jm[pos >> 5] >> (pos & 31)) & 1u) ? 0u : 1u << u;
                }
            } else if (q < nt && q - np < kc) {
                mi[u] = uint32_t(q - np);
                e[u] = Y[q - np];                                // the staging word
            }
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int32_t q = q0 + u * NT + tid;
            if (q >= nt) continue;
            uint64_t key = kNone;
            if (q < np) {
                // a slot the message does not carry (TFAIL: not gossipable at t - 1; a JOINREP:
                // not on the introducer list) stays in its sorted run as a no-op tuple (val 0)
                if (e[u] != kPvEmpty) {
                    const bool carried = !((cut >> u) & 1u) && pv_gossiped(e[u], tf, t5m1);
                    merged += carried ? 1u : 0u;
                    const uint32_t x = uint32_t(e[u] >> 32), v = uint32_t(e[u]) & 0xFFFFu;
                    key = d_tuple(x, mi[u] + 1u, 0u, (x == r || !carried) ? 0u : v);
                }
            } else if (q - np < kc) {
                const uint32_t s = (e[u] & kStageJoinRep) ? 0u : uint32_t(e[u] >> 40);
                key = d_tuple(s, mi[u] + 1u, 1u, 0u);
            }
            X[Lp + q] = key;
        }
    }
    __syncthreads();
    return merged;
}

// Chunk step 3 (HBM kernel): merge-path merges of the sorted runs of width w0, X <-> Y;
// returns the offset of the sorted buffer.
__device__ __forceinline__ int64_t d_merge_runs(uint64_t *base, int64_t C, int64_t xo, int32_t N, int32_t w0) {
    const int32_t tid = threadIdx.x;
    int32_t E = 2;                                               // outputs per lane and pass
    while (E < 16 && int64_t(E) * kHT < N) E <<= 1;
    for (int32_t w = w0; w < N; w <<= 1) {
        const uint64_t *X = base + xo;
        uint64_t *Y = base + (C - xo);
        const int32_t Ew = E < 2 * w ? E : 2 * w;                // divides 2w: one pair per piece
        for (int32_t d0 = tid * Ew; d0 < N; d0 += kHT * Ew) {
            const int32_t p0 = d0 & ~(2 * w - 1);
            const int32_t a1 = p0 + w < N ? p0 + w : N, b1 = p0 + 2 * w < N ? p0 + 2 * w : N;
            const int32_t na = a1 - p0, nb = b1 - a1, d = d0 - p0;
            const uint64_t *A = X + p0, *B = X + a1;
            int32_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
            while (lo < hi) {                                    // merge path: A first on ties
                const int32_t mid = (lo + hi) >> 1;
                if (A[mid] <= B[d - 1 - mid]) lo = mid + 1; else hi = mid;
            }
            int32_t i = lo, j = d - lo;
            uint64_t va = i < na ? A[i] : kNone, vb = j < nb ? B[j] : kNone;
            const int32_t n = b1 - d0 < Ew ? b1 - d0 : Ew;
            for (int32_t q = 0; q < n; ++q) {
                const bool ta = j >= nb || (i < na && va <= vb);
                Y[d0 + q] = ta ? va : vb;
                if (ta) { ++i; va = i < na ? A[i] : kNone; }
                else { ++j; vb = j < nb ? B[j] : kNone; }
            }
        }
        __syncthreads();
        xo = C - xo;
    }
    return xo;
}

// One tuple of an id's run applied to the run's state (cur: hb << 5 | ts5, 0 = absent; own:
// the list flag of an m = 0 tuple), in message order.
__device__ __forceinline__ void d_apply(uint32_t &cur, uint32_t &own, uint32_t lo, uint32_t t5, uint32_t tr) {
    const uint32_t m = lo >> 17, fl = (lo >> 16) & 1u, v = lo & 0xFFFFu;
    if (m == 0) {
        if (v) { cur = v; own = fl; }                            // the list (own view, earlier chunks)
    } else if (fl) {
        cur = pv_event(cur, t5);                                 // the sender: MP1Node.cpp:237-243
    } else {
        cur = pv_merge(cur, v, t5, tr);                          // a payload entry: :247-251, 282-301
    }
}

// Step 5's bin selection (wave 0): the first bin where the running count reaches need;
// sh.sel = {bin, tuples still needed from it}
template <class Sh>
__device__ inline void d_select(Sh &sh, uint32_t need) {
    if (threadIdx.x < 64) {
        const int32_t l = threadIdx.x;
        uint32_t h[4], s = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) { h[q] = sh.hist[4 * l + q]; s += h[q]; }
        const uint32_t incl = wave_incl_scan(s);
        const uint64_t bal = __ballot(incl >= need);
        const int32_t fl = bal ? __ffsll((unsigned long long)bal) - 1 : 63;
        if (l == fl) {
            uint32_t cum = incl - s;
            int32_t b = 0;
            for (; b < 3; ++b) {
                if (cum + h[b] >= need) break;
                cum += h[b];
            }
            sh.sel[0] = uint32_t(4 * l + b);
            sh.sel[1] = need - cum;
        }
    }
    __syncthreads();
}

__device__ inline uint32_t d_prefix(uint32_t v, uint32_t t5) {   // age << 11 | (2047 - hb)
    return (((t5 - v) & 31u) << 11) | (2047u - (v >> 5));
}

template <int NT, bool kRecord = false, class Sh>
__device__ __forceinline__ void d_row_digest(const PviewTickArgs &a, Sh &sh, int32_t lr, uint32_t r, int32_t k,
                                             uint32_t merged, uint32_t joins, uint32_t removes,
                                             uint32_t evicts, uint64_t hsum, uint32_t W);

// Steps 5-6 over the list S[0, L) (x << 32 | own << 16 | val).  pcol / pok: the SWIM probe.
template <bool kEv, int NT, bool kRecord = false, class Sh, class P>
__device__ __forceinline__ void d_finish(const PviewTickArgs &a, Sh &sh, P S, int32_t L,
                                         int32_t lr, uint32_t r, int32_t k, uint32_t merged,
                                         uint32_t pcol, bool pok, DMark &pm) {
    const int32_t tid = threadIdx.x, V = a.view;
    const uint32_t t = uint32_t(a.tick), t5 = t & 31u, tr = uint32_t(a.tremove);
    const uint64_t Sj = pv_seed(1, t, r), Sr = pv_seed(2, t, r), Se = pv_seed(3, t, r);
    const bool rot = a.evict_rot != 0;
    const uint32_t mrot = rot ? draw_u31(kDomainEvict, a.seed, t, r, 0u, 0u) % uint32_t(a.n) : 0u;
    const bool ev = kEv && a.ev.buf != nullptr;
    uint32_t joins = 0, removes = 0, surv = 0;
    uint64_t hsum = 0;
    // joins (not in the own view at the start) and TREMOVE (MP1Node.cpp:339-348)
    for (int32_t base = 0; base < L; base += NT) {               // wave-uniform trips
        const int32_t i = base + tid;
        bool jn = false, rm = false;
        uint32_t x = 0;
        if (i < L) {
            const uint64_t e = S[i];
            x = uint32_t(e >> 32);
            uint32_t v = uint32_t(e) & 0xFFFFu;
            if (x == pcol) {                                     // SWIM: the probe's answer
                v = (v & 0xFFE0u) | (pok ? t5 : ((t5 - tr) & 31u));
                S[i] = (e & ~0xFFFFull) | v;
            }
            jn = !((uint32_t(e) >> 16) & 1u);
            rm = ((t5 - v) & 31u) >= tr;
            joins += jn ? 1u : 0u;
            removes += rm ? 1u : 0u;
            surv += rm ? 0u : 1u;
            if (jn) hsum += pv_hash(uint32_t(Sj), x);
            if (rm) hsum += pv_hash(uint32_t(Sr), x);
            // the eviction's first histogram (zeroed at the row's start): a long row's list
            // nearly always holds more than V survivors
            else atomicAdd(&sh.hist[d_prefix(v, t5) >> 8], 1u);
        }
        if (ev) {
            const bool ej = jn && (a.ev.kinds & GSP_EVENTS_JOIN), er = rm && (a.ev.kinds & GSP_EVENTS_REMOVE);
            uint64_t p = wave_reserve_events(ev_stripe_count(a.ev), (ej ? 1u : 0u) + (er ? 1u : 0u));
            unsigned long long *eb = ev_stripe_buf(a.ev);
            if (ej) { if (int64_t(p) < a.ev.cap) eb[p] = event_record(1u, t, r, x); ++p; }
            if (er) { if (int64_t(p) < a.ev.cap) eb[p] = event_record(2u, t, r, x); }
        }
    }
    const uint32_t C = d_sum<NT>(surv, sh.red[0]);
    pm.mark(5);
    // the V-th survivor's prefix bin T16 and how many of that bin are kept (need2); every
    // survivor with a smaller prefix is kept
    uint32_t T16 = 0x10000u, need2 = 0;
    if (int32_t(C) > V) {
        d_select(sh, uint32_t(V));                               // the high byte (built above)
        T16 = sh.sel[0];
        need2 = sh.sel[1];
        __syncthreads();                                         // sel / hist reused
        for (int32_t i = tid; i < 256; i += NT) sh.hist[i] = 0;
        __syncthreads();
        for (int32_t i = tid; i < L; i += NT) {                  // the low byte, that bin only
            const uint32_t v = uint32_t(S[i]) & 0xFFFFu;
            if (((t5 - v) & 31u) >= tr) continue;
            const uint32_t p = d_prefix(v, t5);
            if ((p >> 8) == T16) atomicAdd(&sh.hist[p & 255u], 1u);
        }
        __syncthreads();
        d_select(sh, need2);
        T16 = (T16 << 8) | sh.sel[0];
        need2 = sh.sel[1];
    }
    pm.mark(6);
    // the kept entries in id order: contiguous pieces per lane.  The T16 bin's members are
    // kept in (rotated) id order: member rank rho (id order) -> (rho - MB) mod c2, MB = the
    // members below the rotation point
    const int32_t F = (L + NT - 1) / NT, i0 = tid * F, i1 = i0 + F < L ? i0 + F : L;
    uint32_t mc = 0, mb = 0, less = 0;                           // less: survivors below T16
    for (int32_t i = i0; i < i1; ++i) {
        const uint64_t e = S[i];
        const uint32_t v = uint32_t(e) & 0xFFFFu;
        if (((t5 - v) & 31u) >= tr) continue;
        const uint32_t p = d_prefix(v, t5);
        less += p < T16 ? 1u : 0u;
        if (p == T16) {
            mc++;
            mb += uint32_t(e >> 32) < mrot ? 1u : 0u;
        }
    }
    uint32_t c2 = 0, MB = 0;
    const uint32_t rho0 = d_scan<NT>(mc, &c2, sh.red[1]);
    MB = d_sum<NT>(mb, sh.red[0]);
    // the lane's members are ranks [rho0, rho0 + mc); rank rho is kept iff (rho - MB) mod c2 <
    // need2, i.e. rho in [MB, min(c2, MB + need2)) or in [0, MB + need2 - c2)
    auto overlap = [](uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) -> uint32_t {
        const uint32_t lo = a0 > b0 ? a0 : b0, hi = a1 < b1 ? a1 : b1;
        return hi > lo ? hi - lo : 0u;
    };
    const uint32_t kend = MB + need2 < c2 ? MB + need2 : c2, kwrap = MB + need2 > c2 ? MB + need2 - c2 : 0u;
    const uint32_t kept = less + overlap(rho0, rho0 + mc, MB, kend) + overlap(rho0, rho0 + mc, 0u, kwrap);
    uint32_t W = 0;
    const uint32_t w0 = d_scan<NT>(kept, &W, sh.red[1]);
    uint64_t *out = a.cur + int64_t(lr) * V;
    uint32_t evicts = 0;
    {
        uint32_t rho = rho0, w = w0;
        for (int32_t i = i0; i < i1; ++i) {
            const uint64_t e = S[i];
            const uint32_t x = uint32_t(e >> 32), v = uint32_t(e) & 0xFFFFu;
            if (((t5 - v) & 31u) >= tr) continue;
            const uint32_t p = d_prefix(v, t5);
            bool keep = p < T16;
            if (p == T16) {
                const uint32_t rr = rho >= MB ? rho - MB : rho + c2 - MB;
                keep = rr < need2;
                rho++;
            }
            if (keep) {
                __builtin_nontemporal_store((uint64_t(x) << 32) | uint64_t(v), out + w++);
            } else {
                evicts++;
                hsum += pv_hash(uint32_t(Se), x);
            }
        }
    }
    if (ev && (a.ev.kinds & GSP_EVENTS_EVICT)) {                 // a second pass, wave-uniform trips
        uint32_t rho = rho0;
        for (int32_t q = 0; q < F; ++q) {
            const int32_t i = i0 + q;
            bool evict = false;
            uint32_t x = 0;
            if (i < i1) {
                const uint64_t e = S[i];
                x = uint32_t(e >> 32);
                const uint32_t v = uint32_t(e) & 0xFFFFu;
                if (((t5 - v) & 31u) < tr) {
                    const uint32_t p = d_prefix(v, t5);
                    evict = p > T16;
                    if (p == T16) {
                        const uint32_t rr = rho >= MB ? rho - MB : rho + c2 - MB;
                        evict = rr >= need2;
                        rho++;
                    }
                }
            }
            uint64_t pe = wave_reserve_events(ev_stripe_count(a.ev), evict ? 1u : 0u);
            if (evict && int64_t(pe) < a.ev.cap) ev_stripe_buf(a.ev)[pe] = event_record(3u, t, r, x);
        }
    }
    for (int32_t i = int32_t(W) + tid; i < V; i += NT) __builtin_nontemporal_store(kPvEmpty, out + i);
    pm.mark(7);
    d_row_digest<NT, kRecord>(a, sh, lr, r, k, merged, joins, removes, evicts, hsum, W);
    pm.mark(8);
}

// The row's counts: straight into the tick digest (a hub row's counts overflow the per-row
// record's 8- and 16-bit fields; its record stays zero) or, kRecord (a hash-class row: k <= 64,
// at most 19,712 ids), into the per-row record pview_digest_kernel sums (wave slot 0; no
// contended global atomics) -- joins, removes, evictions, merges and the hash (16 + 16 + 32
// bits), one reduction -- and its length and own heartbeat.
template <int NT, bool kRecord, class Sh>
__device__ __forceinline__ void d_row_digest(const PviewTickArgs &a, Sh &sh, int32_t lr, uint32_t r, int32_t k,
                                             uint32_t merged, uint32_t joins, uint32_t removes,
                                             uint32_t evicts, uint64_t hsum, uint32_t W) {
    const int32_t tid = threadIdx.x;
    const uint32_t t = uint32_t(a.tick);
    {
        const uint32_t part[7] = {joins, removes, evicts, merged, uint32_t(hsum) & 0xFFFFu,
                                  (uint32_t(hsum) >> 16) & 0xFFFFu, uint32_t(hsum >> 32)};
#pragma unroll
        for (int q = 0; q < 7; ++q) {
            const uint32_t w = wave_sum32(part[q]);
            if ((tid & 63) == 0) sh.tot[tid >> 6][q] = w;
        }
    }
    d_sync_lds();                                                // (the row's stores need not wait)
    uint32_t sum[7] = {0, 0, 0, 0, 0, 0, 0};
    if (tid < 64) {                                              // wave 0: lane w reads wave w's
#pragma unroll
        for (int q = 0; q < 7; ++q) sum[q] = wave_sum32(tid < NT / 64 ? sh.tot[tid][q] : 0u);
    }
    const uint32_t jr = sum[0], rm = sum[1], evs = sum[2], mg = sum[3];
    const uint64_t h_lo = sum[4], h_mid = sum[5], h_hi = sum[6];
    const uint64_t Sj = pv_seed(1, t, r), Sr = pv_seed(2, t, r), Se = pv_seed(3, t, r);
    const uint64_t h = h_lo + (h_mid << 16) + (h_hi << 32) + uint64_t(jr) * Sj + uint64_t(rm) * Sr + uint64_t(evs) * Se;
    if constexpr (kRecord) {
        // rowdig[lr][0]: w0 = merges | delivered << 32 | round << 56, w1 = joins | removes << 16 |
        // evicts << 32, w2 = the hash; w3 is the send kernel's; wave slots 1-3 zero
        if (tid < 16 && tid != 3) {
            const uint64_t w = tid == 0 ? uint64_t(mg + uint32_t(k)) | (uint64_t(k) << 32) | (1ull << 56)
                               : tid == 1 ? uint64_t(jr) | (uint64_t(rm) << 16) | (uint64_t(evs) << 32)
                               : tid == 2 ? h : 0ull;
            a.rowdig[int64_t(lr) * 16 + tid] = w;
        }
    } else {
        if (tid == 0) {
            unsigned long long *dig = a.dig + (blockIdx.x % kPvDigSlots) * kPvFields;
            atomicAdd(dig + kPvRounds, 1ull);
            atomicAdd(dig + kPvMerges, (unsigned long long)(mg + uint32_t(k)));
            atomicAdd(dig + kPvDelivered, (unsigned long long)k);
            if (jr) atomicAdd(dig + kPvJoins, (unsigned long long)jr);
            if (rm) atomicAdd(dig + kPvRemoves, (unsigned long long)rm);
            if (evs) atomicAdd(dig + kPvEvicts, (unsigned long long)evs);
            atomicAdd(dig + kPvHash, (unsigned long long)h);
        }
        if (tid < 16 && tid != 3) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;   // w3: the send kernel's
    }
    if (tid == 0) {
        a.len_cur[lr] = int32_t(W);
        // alive at every tick since it started (pre-joined: ticks 1..t)
        const int32_t st = a.start_tick ? a.start_tick[r] : 0;
        a.own_hb[lr] = int32_t(t) - (st > 0 ? st - 1 : 0);
    }
}

// The list's first form: the own view, this node itself and zero values left out, as list
// tuples (flag 1: in the own view) at X[0, L); returns L.
template <int NT, class Sh, class P>
__device__ __forceinline__ int32_t d_own(const PviewTickArgs &a, Sh &sh, P X, int32_t lr, uint32_t r) {
    const int32_t tid = threadIdx.x, V = a.view;
    const int32_t per = V > NT ? 2 : 1;                          // V <= 256 <= 2 NT: contiguous slots
    uint64_t e[2];
    uint32_t cnt = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int32_t i = tid * per + q;
        e[q] = q < per && i < V ? a.prev[int64_t(lr) * V + i] : kPvEmpty;
        const uint32_t x = uint32_t(e[q] >> 32), v = uint32_t(e[q]) & 0xFFFFu;
        if (!(e[q] != kPvEmpty && x != r && v != 0u)) e[q] = kPvEmpty;
        cnt += e[q] != kPvEmpty ? 1u : 0u;
    }
    uint32_t tot = 0;
    uint32_t pos = d_scan<NT>(cnt, &tot, sh.red[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q)
        if (e[q] != kPvEmpty) X[pos++] = d_tuple(uint32_t(e[q] >> 32), 0u, 1u, uint32_t(e[q]) & 0xFFFFu);
    __syncthreads();
    return int32_t(tot);
}

// ---- the merge and the fold (LDS classes: the row's N <= CAP tuples in one LDS buffer) ------

// Compare-exchange of two u64 registers (ascending)
__device__ __forceinline__ void d_cx(uint64_t &x, uint64_t &y) {
    const uint64_t lo = x < y ? x : y, hi = x < y ? y : x;
    x = lo;
    y = hi;
}

// Merge levels in place: each lane finds the co-rank of its E = CAP / NT outputs, loads the E
// tuples of each input from there (two batches of independent LDS reads), keeps the E
// smallest of the 2E (a bitonic half-cleaner: a[q] against b[E-1-q]) and sorts that bitonic
// sequence in registers (log2 E stages); the workgroup waits, then the lanes write their
// outputs over the inputs (Vp >= 8: a lane's outputs lie in one pair of runs).
template <int NT, int E, class P>
__device__ __forceinline__ void d_merge_ip(P X, int32_t N, int32_t Vp) {
    static_assert((E & (E - 1)) == 0, "E is a power of two");
    const int32_t d0 = int32_t(threadIdx.x) * E;
    for (int32_t w = Vp; w < N; w <<= 1) {
        uint64_t o[E];
        int32_t n = 0;
        if (d0 < N) {
            const int32_t p0 = d0 & ~(2 * w - 1);
            const int32_t a1 = p0 + w < N ? p0 + w : N, b1 = p0 + 2 * w < N ? p0 + 2 * w : N;
            const int32_t na = a1 - p0, nb = b1 - a1, d = d0 - p0;
            int32_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
            while (lo < hi) {                                    // merge path: A first on ties
                const int32_t mid = (lo + hi) >> 1;
                if (X[p0 + mid] <= X[a1 + d - 1 - mid]) lo = mid + 1; else hi = mid;
            }
            const int32_t i = lo, j = d - lo;
            uint64_t bq[E];
#pragma unroll
            for (int q = 0; q < E; ++q) {                        // the next E of each input
                o[q] = i + q < na ? X[p0 + i + q] : kNone;
                bq[q] = j + q < nb ? X[a1 + j + q] : kNone;
            }
#pragma unroll
            for (int q = 0; q < E; ++q) {                        // the E smallest: bitonic
                const uint64_t y = bq[E - 1 - q];
                o[q] = o[q] < y ? o[q] : y;
            }
#pragma unroll
            for (int h = E / 2; h > 0; h >>= 1)                  // bitonic sort, ascending
#pragma unroll
                for (int q = 0; q < E; ++q)
                    if ((q & h) == 0) d_cx(o[q], o[q + h]);
            n = b1 - d0 < E ? b1 - d0 : E;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < E; ++q)
            if (q < n) X[d0 + q] = o[q];
        __syncthreads();
    }
}

// Hub kernel, step 3 in HBM for runs of w >= E / 2: one merge level X -> Y per pass, every lane's
// E outputs from windows of E tuples of each input loaded at once (a bitonic half-cleaner and a
// register sort, as d_merge_ip) instead of one dependent load per output (d_merge_runs);
// returns the offset of the sorted buffer.
template <int E>
__device__ __forceinline__ int64_t d_merge_runs_win(uint64_t *base, int64_t C, int64_t xo, int32_t N, int32_t w0) {
    const int32_t tid = threadIdx.x;
    for (int32_t w = w0; w < N; w <<= 1) {
        const uint64_t *X = base + xo;
        uint64_t *Y = base + (C - xo);
        for (int32_t d0 = tid * E; d0 < N; d0 += kHT * E) {    // E divides 2w: one pair per lane
            const int32_t p0 = d0 & ~(2 * w - 1);
            const int32_t a1 = p0 + w < N ? p0 + w : N, b1 = p0 + 2 * w < N ? p0 + 2 * w : N;
            const int32_t na = a1 - p0, nb = b1 - a1, d = d0 - p0;
            const uint64_t *A = X + p0, *B = X + a1;
            int32_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
            while (lo < hi) {                                    // merge path: A first on ties
                const int32_t mid = (lo + hi) >> 1;
                if (A[mid] <= B[d - 1 - mid]) lo = mid + 1; else hi = mid;
            }
            const int32_t i = lo, j = d - lo;
            uint64_t o[E], bq[E];
#pragma unroll
            for (int q = 0; q < E; ++q) {
                o[q] = i + q < na ? A[i + q] : kNone;
                bq[q] = j + q < nb ? B[j + q] : kNone;
            }
#pragma unroll
            for (int q = 0; q < E; ++q) {                        // the E smallest: bitonic
                const uint64_t y = bq[E - 1 - q];
                o[q] = o[q] < y ? o[q] : y;
            }
#pragma unroll
            for (int h = E / 2; h > 0; h >>= 1)
#pragma unroll
                for (int q = 0; q < E; ++q)
                    if ((q & h) == 0) d_cx(o[q], o[q + h]);
            const int32_t n = b1 - d0 < E ? b1 - d0 : E;
#pragma unroll
            for (int q = 0; q < E; ++q)
                if (q < n) Y[d0 + q] = o[q];
        }
        __syncthreads();
        xo = C - xo;
    }
    return xo;
}

// Each id's run folded in place, over the tuples S[sb, sb + n) of a sorted sequence of N.
// Pass 1: lane t loads its F tuples into registers (one batch of independent reads), folds the
// runs that start among them in registers -- a run that continues past them is walked on in
// S (rare; it may cross into the next block) -- and writes each run's result over the run's
// first tuple (id kept: a neighbour only reads a run head to see that its own run has ended;
// results have m = 0, the runs' other tuples m >= 1).  Pass 2: after a barrier the lane loads
// its results and, after the scan's barrier, writes them compacted in id order from S[out0].
// prev0: the id of the tuple before the block (read before anything overwrote it).  Returns
// the results written.
template <int NT, int F, class Sh, class P>
__device__ __forceinline__ int32_t d_fold_block(Sh &sh, P S, int32_t sb, int32_t n, int32_t N, uint32_t prev0,
                                                int32_t out0, uint32_t t5, uint32_t tr) {
    const int32_t i0 = sb + int32_t(threadIdx.x) * F, iend = sb + n;
    uint64_t tu[F];
#pragma unroll
    for (int q = 0; q < F; ++q) tu[q] = i0 + q < iend ? S[i0 + q] : kNone;
    const uint32_t prev = threadIdx.x == 0 ? prev0 : i0 < iend ? uint32_t(S[i0 - 1] >> 32) : kNoId;
    uint32_t cnt = 0;
    uint32_t cur = 0, own = 0;                                   // the run being folded
    int32_t at0 = -1;                                            // its first tuple (this lane's)
#pragma unroll
    for (int q = 0; q < F; ++q) {
        const uint32_t x = uint32_t(tu[q] >> 32);
        const uint32_t px = q == 0 ? prev : uint32_t(tu[q > 0 ? q - 1 : 0] >> 32);
        if (x != px) {                                           // a run starts here
            cur = 0;
            own = 0;
            at0 = x != kNoId ? q : -1;
        }
        if (at0 >= 0) d_apply(cur, own, uint32_t(tu[q]), t5, tr);   // a run of this lane
        const bool last = q + 1 == F || i0 + q + 1 == iend;     // this lane's last tuple
        const uint32_t nx = q + 1 < F ? uint32_t(tu[q + 1 < F ? q + 1 : q] >> 32) : kNoId;
        if (at0 >= 0 && (last || nx != x)) {
            if (last) {                                          // may continue past this lane
                for (int32_t j = i0 + q + 1; j < N; j += 4) {    // read four at a time
                    uint64_t u[4];
#pragma unroll
                    for (int z = 0; z < 4; ++z) u[z] = j + z < N ? S[j + z] : kNone;
                    bool stop = false;
#pragma unroll
                    for (int z = 0; z < 4; ++z) {
                        stop = stop || uint32_t(u[z] >> 32) != x;
                        if (!stop) d_apply(cur, own, uint32_t(u[z]), t5, tr);
                    }
                    if (stop) break;
                }
            }
            S[i0 + at0] = d_tuple(x, 0u, cur ? own : 0u, cur);   // cur = 0: absent
            cnt += cur ? 1u : 0u;
            at0 = -1;
        }
    }
    __syncthreads();                                             // every run folded
    uint64_t res[F];
#pragma unroll
    for (int q = 0; q < F; ++q) {
        const int32_t i = i0 + q;
        const uint64_t t = i < iend ? S[i] : kNone;
        const uint32_t lo = uint32_t(t);
        res[q] = (t != kNone && (lo >> 17) == 0u && (lo & 0xFFFFu) != 0u) ? t : 0ull;
    }
    uint32_t tot = 0;
    uint32_t at = uint32_t(out0) + d_scan<NT>(cnt, &tot, sh.red[0]);   // every result loaded
#pragma unroll
    for (int q = 0; q < F; ++q)
        if (res[q]) S[int32_t(at++)] = res[q];
    __syncthreads();
    return int32_t(tot);
}

// The fold of an LDS row: one block.  Returns the list length.
template <int NT, int F, class Sh, class P>
__device__ __forceinline__ int32_t d_fold_ip(Sh &sh, P S, int32_t N, uint32_t t5, uint32_t tr) {
    return d_fold_block<NT, F>(sh, S, 0, N, N, kNoId, 0, t5, tr);
}

// The hub kernel's fold of one block: the block's nb tuples of the sorted HBM sequence H[0, nrest)
// staged in LDS (B) and folded there as d_fold_block does -- only a run that continues past the
// block reads on in HBM -- and the results written compacted to Out[out0, ...) in HBM (behind
// the block: out0 + results <= the block's start + nb).  Returns the results written.
template <int NT, int F, class Sh>
__device__ __forceinline__ int32_t d_fold_staged(Sh &sh, SkewBuf B, const uint64_t *H, int32_t nb, int32_t nrest,
                                                 uint32_t prev0, uint64_t *Out, int32_t out0, uint32_t t5, uint32_t tr) {
    for (int32_t i = int32_t(threadIdx.x); i < nb; i += NT) B[i] = H[i];
    __syncthreads();
    const int32_t i0 = int32_t(threadIdx.x) * F;
    uint64_t tu[F];
#pragma unroll
    for (int q = 0; q < F; ++q) tu[q] = i0 + q < nb ? B[i0 + q] : kNone;
    const uint32_t prev = threadIdx.x == 0 ? prev0 : i0 < nb ? uint32_t(B[i0 - 1] >> 32) : kNoId;
    uint32_t cnt = 0;
    uint32_t cur = 0, own = 0;                                   // the run being folded
    int32_t at0 = -1;                                            // its first tuple (this lane's)
#pragma unroll
    for (int q = 0; q < F; ++q) {
        const uint32_t x = uint32_t(tu[q] >> 32);
        const uint32_t px = q == 0 ? prev : uint32_t(tu[q > 0 ? q - 1 : 0] >> 32);
        if (x != px) {                                           // a run starts here
            cur = 0;
            own = 0;
            at0 = x != kNoId ? q : -1;
        }
        if (at0 >= 0) d_apply(cur, own, uint32_t(tu[q]), t5, tr);
        const bool last = q + 1 == F || i0 + q + 1 == nb;        // this lane's last tuple
        const uint32_t nx = q + 1 < F ? uint32_t(tu[q + 1 < F ? q + 1 : q] >> 32) : kNoId;
        if (at0 >= 0 && (last || nx != x)) {
            if (last) {                                          // may continue past this lane: a hub's
                // hot ids run for up to k tuples, read four at a time (past the block: in HBM)
                for (int32_t j = i0 + q + 1; j < nrest; j += 4) {
                    uint64_t u[4];
#pragma unroll
                    for (int z = 0; z < 4; ++z) {
                        const int32_t jj = j + z;
                        u[z] = jj < nrest ? (jj < nb ? B[jj] : H[jj]) : kNone;
                    }
                    bool stop = false;
#pragma unroll
                    for (int z = 0; z < 4; ++z) {
                        stop = stop || uint32_t(u[z] >> 32) != x;
                        if (!stop) d_apply(cur, own, uint32_t(u[z]), t5, tr);
                    }
                    if (stop) break;
                }
            }
            B[i0 + at0] = d_tuple(x, 0u, cur ? own : 0u, cur);   // cur = 0: absent
            cnt += cur ? 1u : 0u;
            at0 = -1;
        }
    }
    __syncthreads();                                             // every run folded
    uint64_t res[F];
#pragma unroll
    for (int q = 0; q < F; ++q) {
        const int32_t i = i0 + q;
        const uint64_t t = i < nb ? B[i] : kNone;
        const uint32_t lo = uint32_t(t);
        res[q] = (t != kNone && (lo >> 17) == 0u && (lo & 0xFFFFu) != 0u) ? t : 0ull;
    }
    uint32_t tot = 0;
    uint32_t at = uint32_t(out0) + d_scan<NT>(cnt, &tot, sh.red[0]);
#pragma unroll
    for (int q = 0; q < F; ++q)
        if (res[q]) Out[int32_t(at++)] = res[q];
    __syncthreads();                                             // B reused by the next block
    return int32_t(tot);
}

// ---- hub kernel (class kDrainHub): two HBM tuple buffers per workgroup, messages in chunks --

template <bool kEv>
__device__ __forceinline__ void d_body_hbm(const PviewTickArgs &a, DrainShared<kHT, kHBlock> &sh, uint64_t *base,
                                           int64_t C, int32_t lr, uint32_t r, int32_t k, const int32_t *src,
                                           const int32_t *slot, const uint32_t *jm, uint32_t pcol, bool pok,
                                           DMark &pm) {
    const int32_t tid = threadIdx.x, V = a.view;
    const uint32_t t5 = uint32_t(a.tick) & 31u, tr = uint32_t(a.tremove);
    int32_t lgV = 0;
    while ((1 << lgV) < V) ++lgV;
    const int32_t Vp = 1 << lgV;
    int64_t xo = 0;
    for (int32_t i = tid; i < 256; i += kHT) sh.hist[i] = 0;     // d_finish's first histogram
    int32_t L = d_own<kHT>(a, sh, base, lr, r);
    pm.mark(1);
    uint32_t merged = 0;
    for (int32_t m0 = 0; m0 < k;) {                              // block-uniform chunks
        const int32_t Lp = (L + Vp - 1) >> lgV << lgV;
        // the most messages with Lp + kc Vp + the senders' runs <= C
        int64_t kc = (C - Lp - Vp) / Vp;
        if (kc > k - m0) kc = k - m0;
        if (kc > kMaxChunk) kc = kMaxChunk;
        while (kc > 0 && Lp + kc * Vp + (kc + Vp - 1) / Vp * Vp > C) --kc;
        if (kc < 1) {                                            // the list fills the buffer
            if (tid == 0) atomicCAS(a.err, 0, a.tick | kDrainErrBit);
            if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
            return;
        }
        uint64_t *X = base + xo, *Y = base + (C - xo);
        merged += d_build<kHT>(a, X, Y, L, Lp, m0, int32_t(kc), Vp, lgV, src, slot, r, m0 == 0 ? jm : nullptr);
        pm.mark(2);
        const int32_t N = Lp + (int32_t(kc) << lgV) + ((int32_t(kc) + Vp - 1) >> lgV << lgV);
        // runs of Vp sorted into blocks of kHBlock in LDS (in-place merges: Vp >= 8), then the
        // blocks merged in HBM
        if (Vp >= 8) {
            uint64_t *X2 = base + xo;
            const SkewBuf B{sh.buf};
            for (int32_t b0 = 0; b0 < N; b0 += kHBlock) {
                const int32_t nb = N - b0 < kHBlock ? N - b0 : kHBlock;
                for (int32_t i = tid; i < nb; i += kHT) B[i] = X2[b0 + i];
                __syncthreads();
                d_merge_ip<kHT, kHBlock / kHT>(B, nb, Vp);
                for (int32_t i = tid; i < nb; i += kHT) X2[b0 + i] = B[i];
                __syncthreads();
            }
        }
        xo = Vp >= 8 ? d_merge_runs_win<16>(base, C, xo, N, kHBlock) : d_merge_runs(base, C, xo, N, Vp);
        pm.mark(3);
        {                                                        // fold, LDS-staged blocks of 8 K tuples
            uint64_t *S2 = base + xo;
            const SkewBuf B{sh.buf};
            int32_t out = 0;
            uint32_t carry = kNoId;
            constexpr int kFB = kHT * 8;                         // 8 tuples per lane (16: spills)
            for (int32_t b0 = 0; b0 < N; b0 += kFB) {
                const int32_t nb = N - b0 < kFB ? N - b0 : kFB;
                const uint32_t last_x = uint32_t(S2[b0 + nb - 1] >> 32);   // before any compaction
                out += d_fold_staged<kHT, 8>(sh, B, S2 + b0, nb, N - b0, carry, S2, out, t5, tr);
                carry = last_x;
            }
            L = out;
        }
        pm.mark(4);
        m0 += int32_t(kc);
    }
    d_finish<kEv, kHT>(a, sh, base + xo, L, lr, r, k, merged, pcol, pok, pm);
}

template <bool kEv>
__device__ void d_row_hbm(const PviewTickArgs &a, DrainShared<kHT, kHBlock> &sh, int32_t lr, uint64_t *scratch,
                          int32_t it) {
    const int32_t tid = threadIdx.x;
    const uint32_t r = uint32_t(a.row0 + lr);
    if (a.rows_run && tid == 0) atomicAdd(a.rows_run, 1);       // tests: each row exactly once
    // crashed, not started yet, or the job stopped
    if (a.tick > a.fail_tick[r] || (a.start_tick && a.tick < a.start_tick[r]) || *a.err) {
        if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
        return;
    }
    const int64_t cap = a.scratch_cap;
    const int32_t o0 = a.csr_off[lr];
    const int32_t k = a.csr_off[lr + 1] - o0;
    int32_t *src = a.csr_src + o0;
    int32_t *slot = a.csr_slot ? a.csr_slot + o0 : nullptr;
    DMark pm;
    pm.init(a.prof, it, k);
    // 1. ascending sender order (keys in LDS, or in the HBM buffers)
    int32_t P = 1;
    while (P < k) P <<= 1;
    if (P <= kHBlock) {
        d_sort_segment<kHT>(src, slot, k, P, a.row0, sh.buf);
    } else if (P <= 2 * cap) {
        d_sort_segment<kHT>(src, slot, k, P, a.row0, scratch);
    } else {
        if (tid == 0) atomicCAS(a.err, 0, a.tick | kDrainErrBit);
        if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
        return;
    }
    uint32_t pcol;
    bool pok;
    pv_swim_probe(a, lr, r, pcol, pok);
    const bool jpay = k > 0 && a.intro_list > 0 && src[0] == kJoinRepSrc;   // block-uniform
    if (jpay) d_intro_mask<kHT>(a, r, sh.jm, sh.red[1]);
    pm.mark(0);
    d_body_hbm<kEv>(a, sh, scratch, cap, lr, r, k, src, slot, jpay ? sh.jm : nullptr, pcol, pok, pm);
}

template <bool kEv>
__global__ void __launch_bounds__(kHT, 1) pview_drain_hbm_kernel(PviewTickArgs a) {
    __shared__ DrainShared<kHT, kHBlock> sh;
    const int32_t cnt = a.long_list[kDrainHub];
    const int32_t *list = a.long_list + kDrainHead + kDrainHub * int64_t(a.rows);
    uint64_t *scratch = reinterpret_cast<uint64_t *>(a.scratch) + int64_t(blockIdx.x) * 2 * a.scratch_cap;
    for (int32_t i = int32_t(blockIdx.x); i < cnt; i += int32_t(gridDim.x)) {
        d_row_hbm<kEv>(a, sh, list[i], scratch, (i - int32_t(blockIdx.x)) / int32_t(gridDim.x));
        __syncthreads();                                         // LDS free for the next row
    }
}

// ---- LDS classes: one row's tuples in one LDS buffer, merged and folded in place ----------

constexpr int d_pow2_ceil(int x) { return x <= 1 ? 1 : 2 * d_pow2_ceil((x + 1) / 2); }

// An LDS row's inputs, fetched while the row before it runs (the persistent loop below): the
// chain list -> CSR offsets -> senders -> payload rows is three dependent HBM round trips,
// so the first two links and the own view are read one row ahead.
struct DIn {
    int32_t lr, o0, k;                          // lr < 0: no row
    bool dead;                                  // crashed, not started, or the job stopped
    int32_t s, sl;                              // lane t < k: CSR entry t (sender, its row)
    uint64_t own[2];                            // own-view slots (d_own's lane mapping)
};

__device__ __forceinline__ void d_fetch_row(const PviewTickArgs &a, DIn &in) {
    in.k = 0;
    in.o0 = 0;
    in.dead = true;
    if (in.lr < 0) return;
    const int32_t r = a.row0 + in.lr;
    in.o0 = a.csr_off[in.lr];
    in.k = a.csr_off[in.lr + 1] - in.o0;                          // <= kDrainStage (the class)
    in.dead = a.tick > a.fail_tick[r] || (a.start_tick && a.tick < a.start_tick[r]) || *a.err;
}

template <int NT>
__device__ __forceinline__ void d_fetch_senders(const PviewTickArgs &a, DIn &in) {
    const int32_t tid = threadIdx.x, V = a.view;
    const int32_t per = V > NT ? 2 : 1;                          // V <= 256 <= 2 NT: contiguous slots
    in.s = in.sl = 0;
    in.own[0] = in.own[1] = kPvEmpty;
    if (in.lr < 0 || in.dead) return;
    if (tid < in.k) {
        in.s = a.csr_src[in.o0 + tid];
        in.sl = a.csr_slot ? a.csr_slot[in.o0 + tid] : in.s - a.row0;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int32_t i = tid * per + q;
        if (q < per && i < V) in.own[q] = a.prev[int64_t(in.lr) * V + i];
    }
}

// Step 1 of an LDS row: lane t < k ranks its sender against all k (distinct keys, broadcast LDS
// reads; a JOINREP, sender kJoinRepSrc = -1, first: its sender is node 0) and writes the
// sender's staging word at its rank.
template <int NT>
__device__ __forceinline__ void d_rank_stage(const PviewTickArgs &a, const DIn &in, uint32_t *keys, uint64_t *stage) {
    const int32_t t = threadIdx.x;
    const uint32_t key = uint32_t(in.s + 1);
    if (t < in.k) keys[t] = key;
    d_sync_lds();
    if (t < in.k) {
        int32_t rank = 0;
        for (int32_t j = 0; j < in.k; ++j) rank += keys[j] < key ? 1 : 0;
        stage[rank] = in.s == kJoinRepSrc ? kStageJoinRep
                      : (uint64_t(uint32_t(in.s)) << 40) |
                            (in.sl >= 0 ? uint64_t(in.sl) : (kStageRemote | uint64_t(-int64_t(in.sl) - 1)));
    }
    d_sync_lds();
}

// The list's first form from the fetched own view (d_own).
template <int NT, class Sh, class P>
__device__ __forceinline__ int32_t d_own_fetched(Sh &sh, P X, const DIn &in, uint32_t r) {
    uint64_t e[2];
    uint32_t cnt = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        e[q] = in.own[q];
        const uint32_t x = uint32_t(e[q] >> 32), v = uint32_t(e[q]) & 0xFFFFu;
        if (!(e[q] != kPvEmpty && x != r && v != 0u)) e[q] = kPvEmpty;
        cnt += e[q] != kPvEmpty ? 1u : 0u;
    }
    uint32_t tot = 0;
    uint32_t pos = d_scan<NT>(cnt, &tot, sh.red[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q)
        if (e[q] != kPvEmpty) X[pos++] = d_tuple(uint32_t(e[q] >> 32), 0u, 1u, uint32_t(e[q]) & 0xFFFFu);
    return int32_t(tot);
}

// Step 2 of an LDS row (d_build for one chunk of every message): the lane's E >= its tuples
// payload loads all issued before the first is used -- one HBM round trip per row.
template <int NT, int E, class P>
__device__ __forceinline__ uint32_t d_build_lds(const PviewTickArgs &a, P X, const uint64_t *Y, int32_t L,
                                                int32_t k, int32_t Vp, int32_t lgV, uint32_t r, const uint32_t *jm) {
    const int32_t tid = threadIdx.x, V = a.view;
    const uint32_t tf = uint32_t(a.tfail), t5m1 = (uint32_t(a.tick) - 1u) & 31u;
    for (int32_t i = L + tid; i < Vp; i += NT) X[i] = kNone;
    const int32_t np = k << lgV;                                 // payload tuples
    const int32_t nt = np + ((k + Vp - 1) >> lgV << lgV);        // + the senders' run(s)
    uint64_t e[E];
    uint32_t cut = 0;                                            // bit u: slot not carried
#pragma unroll
    for (int u = 0; u < E; ++u) {
        const int32_t q = u * NT + tid;
        e[u] = kPvEmpty;
        if (q < np) {
            const int32_t m = q >> lgV, pos = q & (Vp - 1);
            const uint64_t w = Y[m];
            if (pos < V && !(w & kStageJoinRep)) {
                const int64_t row = int64_t(w & kStageRow);
                const uint64_t *p = (w & kStageRemote) ? a.remote : a.prev;
                e[u] = p[row * V + pos];
            } else if (pos < V && jm) {
                e[u] = a.intro[pos];                             // the introducer list
                cut |= ((jm[pos >> 5] >> (pos & 31)) & 1u) ? 0u : 1u << u;
            }
        } else if (q < nt && q - np < k) {
            e[u] = Y[q - np];                                    // the staging word
        }
    }
    uint32_t merged = 0;
#pragma unroll
    for (int u = 0; u < E; ++u) {
        const int32_t q = u * NT + tid;
        if (q >= nt) continue;
        uint64_t key = kNone;
        if (q < np) {
            if (e[u] != kPvEmpty) {                              // a slot not carried: a no-op tuple
                const bool carried = !((cut >> u) & 1u) && pv_gossiped(e[u], tf, t5m1);
                merged += carried ? 1u : 0u;
                const uint32_t x = uint32_t(e[u] >> 32), v = uint32_t(e[u]) & 0xFFFFu;
                key = d_tuple(x, uint32_t(q >> lgV) + 1u, 0u, (x == r || !carried) ? 0u : v);
            }
        } else if (q - np < k) {
            const uint32_t s = (e[u] & kStageJoinRep) ? 0u : uint32_t(e[u] >> 40);
            key = d_tuple(s, uint32_t(q - np) + 1u, 1u, 0u);
        }
        X[Vp + q] = key;
    }
    __syncthreads();
    return merged;
}

// One row of an LDS class, every message in one pass; nxt's inputs fetched on the way.
template <bool kEv, int NT, int CAP>
__device__ __forceinline__ void d_row_lds(const PviewTickArgs &a, DrainShared<NT, CAP> &sh, const DIn &cur,
                                          DIn &nxt, int32_t it) {
    constexpr int E = d_pow2_ceil((CAP + NT - 1) / NT);          // tuples per lane (a power of two)
    const int32_t tid = threadIdx.x, lr = cur.lr, k = cur.k;
    const uint32_t r = uint32_t(a.row0 + lr);
    if (a.rows_run && tid == 0) atomicAdd(a.rows_run, 1);       // tests: each row exactly once
    if (cur.dead) {                                              // crashed, not started, or stopped
        if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
        d_fetch_row(a, nxt);
        d_fetch_senders<NT>(a, nxt);
        return;
    }
    const int32_t V = a.view;
    const uint32_t t5 = uint32_t(a.tick) & 31u, tr = uint32_t(a.tremove);
    DMark pm;
    pm.init(a.prof, it, k);
    for (int32_t i = tid; i < 256; i += NT) sh.hist[i] = 0;     // d_finish's first histogram
    d_rank_stage<NT>(a, cur, reinterpret_cast<uint32_t *>(sh.buf), sh.stage);   // 1. ascending senders
    d_fetch_row(a, nxt);
    uint32_t pcol;
    bool pok;
    pv_swim_probe(a, lr, r, pcol, pok);
    const bool jpay = k > 0 && a.intro_list > 0 && (sh.stage[0] & kStageJoinRep);   // block-uniform
    if (jpay) d_intro_mask<NT>(a, r, sh.jm, sh.red[1]);
    pm.mark(0);
    int32_t lgV = 0;
    while ((1 << lgV) < V) ++lgV;
    const int32_t Vp = 1 << lgV;
    const SkewBuf X{sh.buf};
    const int32_t L0 = d_own_fetched<NT>(sh, X, cur, r);         // <= V: padded to Vp
    pm.mark(1);
    const uint32_t merged = d_build_lds<NT, E>(a, X, sh.stage, L0, k, Vp, lgV, r, jpay ? sh.jm : nullptr);
    d_fetch_senders<NT>(a, nxt);                                 // in flight through steps 3-6
    pm.mark(2);
    const int32_t N = Vp + (k << lgV) + ((k + Vp - 1) >> lgV << lgV);
    d_merge_ip<NT, E>(X, N, Vp);
    pm.mark(3);
    const int32_t L = d_fold_ip<NT, E>(sh, X, N, t5, tr);
    pm.mark(4);
    // k <= 64 and L <= CAP: the counts fit the per-row record (no contended global atomics)
    d_finish<kEv, NT, true>(a, sh, X, L, lr, r, k, merged, pcol, pok, pm);
}

// The rows of LDS class kCls: workgroup b takes rows b, b + grid, ... (a persistent grid of
// rows-per-CU x CUs, or, with the host's copy of the class sizes, one row per workgroup)
template <bool kEv, int NT, int CAP, int kCls, int kWaves = 4>
__global__ void __launch_bounds__(NT, kWaves) pview_drain_lds_kernel(PviewTickArgs a) {
    __shared__ DrainShared<NT, CAP> sh;
    const int32_t cnt = a.long_list[kCls];
    const int32_t *list = a.long_list + kDrainHead + int64_t(kCls) * a.rows;
    const int32_t step = int32_t(gridDim.x);
    int32_t i = int32_t(blockIdx.x);
    if (i >= cnt) return;
    DIn cur, nxt;
    cur.lr = list[i];
    d_fetch_row(a, cur);
    d_fetch_senders<NT>(a, cur);
    for (; i < cnt; i += step) {
        nxt.lr = i + step < cnt ? list[i + step] : -1;
        d_row_lds<kEv, NT, CAP>(a, sh, cur, nxt, (i - int32_t(blockIdx.x)) / step);
        d_sync_lds();                                            // LDS free for the next row
        cur = nxt;
    }
}

template <bool kEv>
void launch_drain_classes(const PviewTickArgs &a, hipStream_t st, int parts) {
    const unsigned cus = unsigned(a.cus);
    // grid: the class's rows when the host knows them (zero: no launch), else persistent
    auto grid = [&](int c, unsigned per_cu) -> unsigned {
        if (!a.drain_rows) return per_cu * cus;
        const int32_t rows = a.drain_rows[c];
        return unsigned(rows < int32_t(per_cu * cus) ? rows : int32_t(per_cu * cus));
    };
    auto mark = [&](int i) { if (a.drain_ev) (void)hipEventRecord(a.drain_ev[i], st); };
    if (parts & 1) {
        mark(0);
#define GSP_DRAIN_LDS(C, NT, CAP, PER_CU, W)                                                        \
    if (const unsigned g = grid(C, PER_CU))                                                           \
        hipLaunchKernelGGL((pview_drain_lds_kernel<kEv, NT, CAP, C, W>), dim3(g), dim3(NT), 0, st, a); \
    mark(C + 1);
    // class c: rows of at most CAP update tuples (pv_drain_class), PER_CU rows per CU by LDS
    GSP_DRAIN_LDS(0, 192, kDrainCap0, kDrainPerCU0, kDrainWaves0)
    GSP_DRAIN_LDS(1, 256, 4096, 4, 4)
    GSP_DRAIN_LDS(2, 512, 8192, 2, 4)
    GSP_DRAIN_LDS(3, 1024, kDrainLdsMax, 1, 4)
#undef GSP_DRAIN_LDS
    }
    if (parts & 2) {
        // on a stream of its own (parts == 2) the hub kernel's interval starts at its own event
        if (parts == 2 && a.drain_ev) (void)hipEventRecord(a.drain_ev[kDrainClasses + 1], st);
        if (grid(kDrainHub, 1)) hipLaunchKernelGGL((pview_drain_hbm_kernel<kEv>), dim3(grid(kDrainHub, 1)), dim3(kHT), 0, st, a);
        mark(kDrainHub + 1);
    }
}

}  // namespace

hipError_t launch_pview_drain(const PviewTickArgs &a, hipStream_t st, int parts) {
    if (!a.drain || a.rows == 0) return hipSuccess;
    if (!a.long_list || !a.scratch || a.cus < 1 || a.scratch_cap < 8192 || a.drain_lds < 1 ||
        a.drain_lds > kDrainLdsMax)
        return hipErrorInvalidValue;
    if (a.ev.buf) launch_drain_classes<true>(a, st, parts);
    else launch_drain_classes<false>(a, st, parts);
    return hipGetLastError();
}

}  // namespace gsp
