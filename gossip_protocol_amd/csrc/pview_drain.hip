// gossip_protocol_amd/csrc/pview_drain.hip -- the DRAIN-ALL partial view (inbox = 0).
//
// The reference drains every queued message (checkMessages, MP1Node.cpp:200-212).  With
// gsp_pview_params.inbox = 0 the partial view does too: a receiver sent k <= kPvMaxInbox
// messages runs in the tick kernels as before (they merge all k), and a receiver sent more
// (a "long" row: the receipt kernel lists it) runs here, one workgroup per row, merging its
// messages one after the other in ascending sender order into a list that may grow past the
// view:
//   1. the segment's senders are sorted ascending (in LDS up to kDrainCap, else in the
//      workgroup's HBM scratch) and written back in place;
//   2. the list starts as the own view (ids ascending, values hb << 5 | ts5, kOwnBit set);
//   3. message j (sender s, payload = s's view of t - 1): each payload entry binary-searches
//      its id in the list -- found: the max-merge (MP1Node.cpp:247-251); absent: a copy when
//      fresh and not this node (:282-301) -- and thread 0 does the same for s (hb + 1, ts = t,
//      or (1, t), :237-243).  The ids of one payload are distinct and s is in no payload of its
//      own, so every update has its own slot.  The new ids go in by one shift of the list
//      (their ranks from one block scan);
//   4. TREMOVE (:339-348), then eviction to V by (age, -hb, id or rotated id): the V-th
//      smallest 37-bit key age << 32 | (2047 - hb) << 21 | tie key, by a binary search over key
//      values (37 counting passes), keeps exactly V (the keys are distinct);
//   5. the new view in id order, the row's counts straight into the tick digest (a long row's
//      counts overflow the per-row record's 8- and 16-bit fields), its events.
// The list lives in LDS (kDrainCap entries, 64 KB: two rows per CU) and moves to the
// workgroup's HBM scratch when a message could overflow it (the hubs: thousands of senders).
// A list or segment past the scratch (scratch_cap entries) stops the job (GSP_ERR_CAPACITY).
// Oracle: oracle/pview_oracle.c with inbox = 0 (the same fold over every message).
#include <cstdint>

#include "join_kernels.hpp"
#include "philox.hpp"
#include "pview_kernels.hpp"
#include "pview_rules.hpp"
#include "scale_kernels.hpp"
#include "wave_ops.hpp"

namespace gsp {
namespace {

constexpr int kDT = 256;                        // threads per drain workgroup (4 waves)
constexpr int kDrainCap = 8192;                 // LDS list capacity (entries)
constexpr int kPer = kDrainCap / kDT;           // list entries per lane in the LDS shift
constexpr uint32_t kOwnBit = 1u << 16;          // the id was in the own view at the start
constexpr uint64_t kKeyHi = (1ull << 37) - 1;   // eviction keys are 37 bits

struct alignas(16) DrainShared {
    uint32_t ids[kDrainCap];                    // the row's list, ascending ids
    uint32_t vals[kDrainCap];                   // packed value | kOwnBit
    uint32_t ins[kPvMaxView + 8];               // insertion points of one message's new ids
    uint32_t red[2][8];                         // block scan words (two buffers, alternated)
};

// exclusive block scan over the 256 lanes; *total = the sum
__device__ inline uint32_t d_scan(uint32_t v, uint32_t *total, uint32_t *buf) {
    const int32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if (lane == 63) buf[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int q = 0; q < kDT / 64; ++q) {
        const uint32_t x = buf[q];
        before += q < wave ? x : 0u;
        all += x;
    }
    *total = all;
    return incl - v + before;
}

__device__ inline uint32_t d_sum(uint32_t v, uint32_t *buf) {
    uint32_t total = 0;
    (void)d_scan(v, &total, buf);
    return total;
}

// lower bound of x in ids[0, L)
__device__ inline int32_t d_lower(const uint32_t *ids, int32_t L, uint32_t x) {
    int32_t lo = 0, hi = L;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (ids[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Bitonic sort, ascending, of the P (a power of two) u64 keys at k (LDS or the workgroup's
// HBM scratch), every thread of the workgroup taking part.
__device__ inline void d_bitonic(uint64_t *k, int32_t P) {
    for (int32_t size = 2; size <= P; size <<= 1)
        for (int32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (int32_t i = threadIdx.x; i < P / 2; i += kDT) {
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
__device__ void d_sort_segment(int32_t *src, int32_t *slot, int32_t k, int32_t P, int32_t row0,
                               uint64_t *keys) {
    for (int32_t i = threadIdx.x; i < P; i += kDT) {
        uint64_t key = ~0ull;
        if (i < k) {
            const int32_t s = src[i];
            const int32_t sl = slot ? slot[i] : s - row0;
            key = (uint64_t(uint32_t(s + 1)) << 32) | uint64_t(uint32_t(sl));
        }
        keys[i] = key;
    }
    __syncthreads();
    d_bitonic(keys, P);
    for (int32_t i = threadIdx.x; i < k; i += kDT) {
        const uint64_t key = keys[i];
        src[i] = int32_t(uint32_t(key >> 32)) - 1;
        if (slot) slot[i] = int32_t(uint32_t(key));
    }
    __syncthreads();
}

// The row's list: in LDS, or in the HBM scratch (a = current, b = the next message's)
struct DrainList {
    int32_t L;                                  // length (block-uniform)
    bool hbm;
    uint32_t *aid, *aval, *bid, *bval;
};

// Merge one message into the list: sender s, this lane's payload entry e (kPvEmpty: none).
template <bool kHbm>
__device__ inline void d_message(DrainShared &sh, DrainList &d, uint32_t r, uint32_t s, uint64_t e,
                                 uint32_t t5, uint32_t tr) {
    const int32_t tid = threadIdx.x;
    uint32_t *ids = kHbm ? d.aid : sh.ids;
    uint32_t *vals = kHbm ? d.aval : sh.vals;
    const int32_t L = d.L;
    const bool ok = e != kPvEmpty;
    const uint32_t x = uint32_t(e >> 32), v = uint32_t(e) & 0xFFFFu;
    int32_t pos = 0;
    bool ins = false;
    if (ok) {
        pos = d_lower(ids, L, x);
        if (pos < L && ids[pos] == x) {                          // MP1Node.cpp:247-251
            const uint32_t cur = vals[pos];
            vals[pos] = (cur & kOwnBit) | pv_merge(cur & 0xFFFFu, v, t5, tr);
        } else {                                                 // MP1Node.cpp:282-301
            ins = x != r && ((t5 - v) & 31u) < tr;
        }
    }
    // the sender's entry (MP1Node.cpp:237-243), thread 0
    int32_t spos = 0;
    bool sins = false;
    if (tid == 0) {
        spos = d_lower(ids, L, s);
        if (spos < L && ids[spos] == s) {
            const uint32_t cur = vals[spos];
            vals[spos] = (cur & kOwnBit) | pv_event(cur & 0xFFFFu, t5);
        } else {
            sins = true;
        }
    }
    // ranks of the new ids: the payload's in lane (= id) order, the sender's among them -- one
    // scan of three 11-bit counts (payload inserts, those below s, the sender's insert)
    uint32_t tot = 0;
    const uint32_t ex = d_scan((ins ? 1u : 0u) | ((ins && x < s) ? 1u << 11 : 0u) | (sins ? 1u << 22 : 0u),
                               &tot, sh.red[0]);
    const bool s_ins = (tot >> 22) != 0;
    const int32_t s_rank = int32_t((tot >> 11) & 0x7FFu);
    const int32_t m = int32_t(tot & 0x7FFu) + (s_ins ? 1 : 0);
    if (m == 0) {
        __syncthreads();                                         // red[0] is read to its end
        return;
    }
    const int32_t rank = int32_t(ex & 0x7FFu) + ((s_ins && s < x) ? 1 : 0);
    if (ins) sh.ins[rank] = uint32_t(pos);
    if (tid == 0 && s_ins) sh.ins[s_rank] = uint32_t(spos);
    __syncthreads();                                             // insertion points, updates
    // the shift: old entry i moves up by the number of new ids inserted at or below it
    if constexpr (!kHbm) {
        const int32_t per = (L + kDT - 1) / kDT, c0 = tid * per;
        uint32_t rid[kPer], rv[kPer];
        int32_t q = d_lower(sh.ins, m, uint32_t(c0) + 1u);       // inserts with position <= c0
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            rid[i] = rv[i] = 0;
            if (i < per && c0 + i < L) { rid[i] = ids[c0 + i]; rv[i] = vals[c0 + i]; }
        }
        __syncthreads();                                         // every read before any write
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int32_t at = c0 + i;
            if (i < per && at < L) {
                while (q < m && int32_t(sh.ins[q]) <= at) ++q;
                ids[at + q] = rid[i];
                vals[at + q] = rv[i];
            }
        }
        if (ins) { ids[pos + rank] = x; vals[pos + rank] = v; }
        if (tid == 0 && s_ins) { ids[spos + s_rank] = s; vals[spos + s_rank] = pv_event(0u, t5); }
    } else {
        for (int32_t i = tid; i < L; i += kDT) {
            const int32_t q = d_lower(sh.ins, m, uint32_t(i) + 1u);
            d.bid[i + q] = ids[i];
            d.bval[i + q] = vals[i];
        }
        if (ins) { d.bid[pos + rank] = x; d.bval[pos + rank] = v; }
        if (tid == 0 && s_ins) { d.bid[spos + s_rank] = s; d.bval[spos + s_rank] = pv_event(0u, t5); }
        uint32_t *ti = d.aid, *tv = d.aval;
        d.aid = d.bid; d.aval = d.bval; d.bid = ti; d.bval = tv;
    }
    d.L = L + m;
    __syncthreads();
}

// eviction key of a surviving entry: (age, -hb, tie key) ascending = the order entries are kept
__device__ inline uint64_t d_key(uint32_t x, uint32_t v, uint32_t t5, uint32_t mrot, uint32_t n, bool rot) {
    const uint32_t age = (t5 - v) & 31u, hb = v >> 5;
    const uint32_t tk = rot ? (x >= mrot ? x - mrot : x + n - mrot) : x;
    return (uint64_t(age) << 32) | (uint64_t(2047u - hb) << 21) | uint64_t(tk);
}

// TREMOVE, eviction, the new view, the row's digest counts and events (steps 4-5).
template <bool kEv>
__device__ void d_finish(const PviewTickArgs &a, DrainShared &sh, const DrainList &d, int32_t lr,
                         uint32_t r, int32_t k, uint32_t merged) {
    const int32_t tid = threadIdx.x;
    const uint32_t *ids = d.hbm ? d.aid : sh.ids;
    const uint32_t *vals = d.hbm ? d.aval : sh.vals;
    const int32_t L = d.L, V = a.view;
    const uint32_t t = uint32_t(a.tick), t5 = t & 31u, tr = uint32_t(a.tremove);
    const uint64_t Sj = pv_seed(1, t, r), Sr = pv_seed(2, t, r), Se = pv_seed(3, t, r);
    const bool rot = a.evict_rot != 0;
    const uint32_t mrot = rot ? draw_u31(kDomainEvict, a.seed, t, r, 0u, 0u) % uint32_t(a.n) : 0u;
    const bool ev = kEv && a.ev.buf != nullptr;
    uint32_t joins = 0, removes = 0, surv = 0;
    uint64_t hsum = 0;
    // joins (not in the own view at the start) and TREMOVE (MP1Node.cpp:339-348)
    for (int32_t i = tid; i < L; i += kDT) {
        const uint32_t val = vals[i], x = ids[i], v = val & 0xFFFFu;
        const bool jn = !(val & kOwnBit), rm = ((t5 - v) & 31u) >= tr;
        joins += jn ? 1u : 0u;
        removes += rm ? 1u : 0u;
        surv += rm ? 0u : 1u;
        if (jn) hsum += pv_hash(uint32_t(Sj), x);
        if (rm) hsum += pv_hash(uint32_t(Sr), x);
    }
    if (ev) {
        for (int32_t base = 0; base < L; base += kDT) {          // wave-uniform trips
            const int32_t i = base + tid;
            uint32_t val = 0, x = 0;
            if (i < L) { val = vals[i]; x = ids[i]; }
            const bool jn = i < L && !(val & kOwnBit) && (a.ev.kinds & GSP_EVENTS_JOIN);
            const bool rm = i < L && ((t5 - (val & 0xFFFFu)) & 31u) >= tr && (a.ev.kinds & GSP_EVENTS_REMOVE);
            uint64_t p = wave_reserve_events(ev_stripe_count(a.ev), (jn ? 1u : 0u) + (rm ? 1u : 0u));
            unsigned long long *eb = ev_stripe_buf(a.ev);
            if (jn) { if (int64_t(p) < a.ev.cap) eb[p] = event_record(1u, t, r, x); ++p; }
            if (rm) { if (int64_t(p) < a.ev.cap) eb[p] = event_record(2u, t, r, x); }
        }
    }
    const uint32_t C = d_sum(surv, sh.red[0]);
    // the V-th smallest key: smallest T with #{key <= T} >= V (keys are distinct)
    uint64_t T = kKeyHi;
    if (int32_t(C) > V) {
        uint64_t lo = 0, hi = kKeyHi;
        int b = 1;
        while (lo < hi) {                                        // block-uniform
            const uint64_t mid = lo + ((hi - lo) >> 1);
            uint32_t c = 0;
            for (int32_t i = tid; i < L; i += kDT) {
                const uint32_t v = vals[i] & 0xFFFFu;
                c += (((t5 - v) & 31u) < tr && d_key(ids[i], v, t5, mrot, uint32_t(a.n), rot) <= mid) ? 1u : 0u;
            }
            if (d_sum(c, sh.red[b]) >= uint32_t(V)) hi = mid; else lo = mid + 1;
            b ^= 1;
        }
        T = lo;
    }
    // the kept entries in id order, evictions counted
    uint64_t *out = a.cur + int64_t(lr) * V;
    uint32_t evicts = 0;
    int32_t w = 0, b = 0;
    for (int32_t base = 0; base < L; base += kDT) {
        const int32_t i = base + tid;
        uint32_t x = 0, v = 0;
        bool keep = false, evict = false;
        if (i < L) {
            x = ids[i];
            v = vals[i] & 0xFFFFu;
            if (((t5 - v) & 31u) < tr) {
                keep = d_key(x, v, t5, mrot, uint32_t(a.n), rot) <= T;
                evict = !keep;
            }
        }
        uint32_t tot = 0;
        const uint32_t pos = d_scan(keep ? 1u : 0u, &tot, sh.red[b]);
        b ^= 1;
        if (keep) __builtin_nontemporal_store((uint64_t(x) << 32) | uint64_t(v), out + w + int32_t(pos));
        if (evict) { evicts++; hsum += pv_hash(uint32_t(Se), x); }
        if (ev && (a.ev.kinds & GSP_EVENTS_EVICT)) {
            uint64_t p = wave_reserve_events(ev_stripe_count(a.ev), evict ? 1u : 0u);
            if (evict && int64_t(p) < a.ev.cap) ev_stripe_buf(a.ev)[p] = event_record(3u, t, r, x);
        }
        w += int32_t(tot);
    }
    for (int32_t i = w + tid; i < V; i += kDT) __builtin_nontemporal_store(kPvEmpty, out + i);
    // the row's counts: straight into the tick digest (its per-row record stays zero)
    const uint32_t jr = d_sum(joins, sh.red[b]);
    b ^= 1;
    const uint32_t rm = d_sum(removes, sh.red[b]);
    b ^= 1;
    const uint32_t evs = d_sum(evicts, sh.red[b]);
    b ^= 1;
    const uint32_t mg = d_sum(merged, sh.red[b]);
    b ^= 1;
    const uint64_t h_lo = d_sum(uint32_t(hsum) & 0xFFFFu, sh.red[b]);
    b ^= 1;
    const uint64_t h_mid = d_sum((uint32_t(hsum) >> 16) & 0xFFFFu, sh.red[b]);
    b ^= 1;
    const uint64_t h_hi = d_sum(uint32_t(hsum >> 32), sh.red[b]);
    if (tid == 0) {
        unsigned long long *dig = a.dig + (blockIdx.x % kPvDigSlots) * kPvFields;
        atomicAdd(dig + kPvRounds, 1ull);
        atomicAdd(dig + kPvMerges, (unsigned long long)(mg + uint32_t(k)));
        atomicAdd(dig + kPvDelivered, (unsigned long long)k);
        if (jr) atomicAdd(dig + kPvJoins, (unsigned long long)jr);
        if (rm) atomicAdd(dig + kPvRemoves, (unsigned long long)rm);
        if (evs) atomicAdd(dig + kPvEvicts, (unsigned long long)evs);
        const uint64_t h = h_lo + (h_mid << 16) + (h_hi << 32) + uint64_t(jr) * Sj + uint64_t(rm) * Sr +
                           uint64_t(evs) * Se;
        atomicAdd(dig + kPvHash, (unsigned long long)h);
        a.len_cur[lr] = w;
        // alive at every tick since it started (pre-joined: ticks 1..t)
        const int32_t st = a.start_tick ? a.start_tick[r] : 0;
        a.own_hb[lr] = int32_t(t) - (st > 0 ? st - 1 : 0);
    }
    if (tid < 16 && tid != 3) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;   // w3: the send kernel's
}

template <bool kEv>
__device__ void d_row(const PviewTickArgs &a, DrainShared &sh, int32_t lr, uint32_t *scratch) {
    const int32_t tid = threadIdx.x;
    const uint32_t r = uint32_t(a.row0 + lr);
    if (a.rows_run && tid == 0) atomicAdd(a.rows_run, 1);       // tests: each row exactly once
    // crashed, not started yet, or the job stopped
    if (a.tick > a.fail_tick[r] || (a.start_tick && a.tick < a.start_tick[r]) || *a.err) {
        if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
        return;
    }
    const int32_t V = a.view;
    const uint32_t t5 = uint32_t(a.tick) & 31u, tr = uint32_t(a.tremove);
    const int64_t cap = a.scratch_cap;
    DrainList d{0, false, scratch, scratch + cap, scratch + 2 * cap, scratch + 3 * cap};
    const int32_t o0 = a.csr_off[lr];
    const int32_t k = a.csr_off[lr + 1] - o0;
    int32_t *src = a.csr_src + o0;
    int32_t *slot = a.csr_slot ? a.csr_slot + o0 : nullptr;
    // 1. ascending sender order
    int32_t P = 1;
    while (P < k) P <<= 1;
    if (P <= a.drain_lds) {
        d_sort_segment(src, slot, k, P, a.row0, reinterpret_cast<uint64_t *>(sh.ids));
    } else if (P <= cap) {
        d_sort_segment(src, slot, k, P, a.row0, reinterpret_cast<uint64_t *>(d.aid));
    } else {
        if (tid == 0) atomicCAS(a.err, 0, a.tick);
        if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
        return;
    }
    // 2. the own view, this node itself left out (never listed)
    {
        const uint64_t e = tid < V ? __builtin_nontemporal_load(a.prev + int64_t(lr) * V + tid) : kPvEmpty;
        const uint32_t x = uint32_t(e >> 32), v = uint32_t(e) & 0xFFFFu;
        const bool keep = e != kPvEmpty && x != r && v != 0u;
        uint32_t tot = 0;
        const uint32_t pos = d_scan(keep ? 1u : 0u, &tot, sh.red[1]);
        if (keep) { sh.ids[pos] = x; sh.vals[pos] = v | kOwnBit; }
        d.L = int32_t(tot);
        __syncthreads();
    }
    // 3. every message, ascending sender; the next payload is loaded while one merges
    // a JOINREP (join schedule without an introducer list: validated on the host) is node 0's
    // sender entry with an empty payload
    auto payload = [&](int32_t j) -> uint64_t {
        if (src[j] == kJoinRepSrc) return kPvEmpty;
        const int32_t sl = slot ? slot[j] : src[j] - a.row0;
        const uint64_t *row = sl >= 0 ? a.prev + int64_t(sl) * V : a.remote + int64_t(-sl - 1) * V;
        return tid < V ? __builtin_nontemporal_load(row + tid) : kPvEmpty;
    };
    uint32_t merged = 0;
    uint64_t nxt = k > 0 ? payload(0) : kPvEmpty;
    for (int32_t j = 0; j < k; ++j) {
        const uint64_t e = nxt;
        const int32_t sj = __builtin_amdgcn_readfirstlane(src[j]);
        const uint32_t s = sj == kJoinRepSrc ? 0u : uint32_t(sj);
        if (j + 1 < k) nxt = payload(j + 1);
        merged += e != kPvEmpty ? 1u : 0u;
        if (!d.hbm && d.L + V + 1 > a.drain_lds) {              // spill the list to HBM
            for (int32_t i = tid; i < d.L; i += kDT) { d.aid[i] = sh.ids[i]; d.aval[i] = sh.vals[i]; }
            d.hbm = true;
            __syncthreads();
        }
        if (d.hbm) {
            if (d.L + V + 1 > cap) {                             // past the scratch: stop the job
                if (tid == 0) atomicCAS(a.err, 0, a.tick);
                if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
                return;
            }
            d_message<true>(sh, d, r, s, e, t5, tr);
        } else {
            d_message<false>(sh, d, r, s, e, t5, tr);
        }
    }
    // 4-5.
    d_finish<kEv>(a, sh, d, lr, r, k, merged);
}

// Persistent: each workgroup takes the listed rows blockIdx.x, blockIdx.x + grid, ...
template <bool kEv>
__global__ void __launch_bounds__(kDT, 2) pview_drain_kernel(PviewTickArgs a) {
    __shared__ DrainShared sh;
    const int32_t cnt = a.long_list[0];
    uint32_t *scratch = a.scratch + int64_t(blockIdx.x) * 4 * a.scratch_cap;
    for (int32_t i = int32_t(blockIdx.x); i < cnt; i += int32_t(gridDim.x)) {
        d_row<kEv>(a, sh, a.long_list[1 + i], scratch);
        __syncthreads();                                         // LDS free for the next row
    }
}

}  // namespace

hipError_t launch_pview_drain(const PviewTickArgs &a, hipStream_t st) {
    if (!a.drain || a.rows == 0) return hipSuccess;
    if (!a.long_list || !a.scratch || a.drain_grid < 1 || a.scratch_cap < kDrainCap ||
        a.drain_lds < 1 || a.drain_lds > kDrainCap)
        return hipErrorInvalidValue;
    const dim3 g(unsigned(a.drain_grid)), blk(kDT);
    if (a.ev.buf) hipLaunchKernelGGL(pview_drain_kernel<true>, g, blk, 0, st, a);
    else hipLaunchKernelGGL(pview_drain_kernel<false>, g, blk, 0, st, a);
    return hipGetLastError();
}

}  // namespace gsp
