// gossip_protocol_amd/csrc/scale_kernels.hip -- SCALE-mode HIP kernels for gfx950.
//
// scale_tick_kernel is the per-tick hot path of one receiver row, fused:
//   merge   (MP1Node::recvCallBack GOSSIP branch, MP1Node.cpp:234-256) of every message the
//           row received, in ascending sender order, 8 packed entries per lane per 16-B load;
//   ops     (MP1Node::nodeLoopOps, MP1Node.cpp:335-348): own heartbeat bump, TREMOVE scan;
//   events  join/remove detection, counted and hashed (order-independent digest);
//   send    (one GPU) peer choice by Philox rank-select over the row's presence bitmap in
//           LDS, the drop draw and the destination count for next tick's CSR; (column
//           shards) the slice's presence bitmap and count, resolved after an all-gather by
//           scale_resolve_kernel / scale_finalize_kernel.
// One 256-lane workgroup per row streams the row in 2048-column chunks: it reads its own
// row and each sender's row once (16 B per lane, fully coalesced) and writes its row once,
// so the kernel is HBM-bound at (2 + k) * stride * 2 bytes per row with k messages.
#include "join_kernels.hpp"
#include "philox.hpp"
#include "scale_kernels.hpp"
#include "wave_ops.hpp"

namespace gsp {

namespace {

__device__ inline uint64_t event_mix(uint32_t kind, uint32_t t, uint32_t r, uint32_t x) {
    uint64_t z = (uint64_t(kind) << 62) | (uint64_t(t & 0xFFFFF) << 42) |
                 (uint64_t(r & 0x1FFFFF) << 21) | uint64_t(x & 0x1FFFFF);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ---- scalar form: one entry at a time ---------------------------------------------------
// Merge one payload entry v (the sender's) into the receiver's entry e (both packed
// hb << 5 | ts5, 0 = absent):
//   present: max-merge, ts = now only on a strict heartbeat increase (MP1Node.cpp:247-251)
//   absent:  copy v when v is present and fresh, t - ts_v < TREMOVE (MP1Node.cpp:294)
__device__ inline uint32_t merge_entry(uint32_t e, uint32_t v, uint32_t t5, uint32_t tr) {
    const uint32_t he = e >> 5, hv = v >> 5;
    const uint32_t upd = (hv > he) ? ((v & 0xFFE0u) | t5) : e;
    const uint32_t fresh = ((t5 - v) & 31u) < tr;
    const uint32_t add = (v != 0u && fresh) ? v : 0u;
    return e ? upd : add;
}

__device__ inline uint32_t merge_word_scalar(uint32_t e, uint32_t v, uint32_t t5, uint32_t tr) {
    const uint32_t lo = merge_entry(e & 0xFFFFu, v & 0xFFFFu, t5, tr);
    const uint32_t hi = merge_entry(e >> 16, v >> 16, t5, tr);
    return lo | (hi << 16);
}

// ---- packed form: two entries per 32-bit word on the v_pk_*_u16 ALUs --------------------
// hipcc folds min(sub_sat(a, b), 1) back into compares + selects, so the packed ops are
// spelled out; every operand is a VGPR and nothing reads EXEC or the memory counters.
__device__ inline uint32_t pk_max(uint32_t a, uint32_t b) {
    uint32_t r; asm("v_pk_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ inline uint32_t pk_min(uint32_t a, uint32_t b) {
    uint32_t r; asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ inline uint32_t pk_sub(uint32_t a, uint32_t b) {
    uint32_t r; asm("v_pk_sub_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ inline uint32_t pk_subc(uint32_t a, uint32_t b) {   // saturating at 0
    uint32_t r; asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ inline uint32_t pk_mad(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r; asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); return r;
}
__device__ inline uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {   // (m & a) | (~m & b)
    uint32_t r; asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b)); return r;
}

struct PackedConsts {
    uint32_t one, t5x2, t32, tr, trm1, low5, hbmask, zero;
};

__device__ inline PackedConsts packed_consts(uint32_t t5, uint32_t tr) {
    PackedConsts c;
    c.one = 0x00010001u;
    c.t5x2 = t5 | (t5 << 16);
    c.t32 = c.t5x2 + 0x00200020u;
    c.tr = tr | (tr << 16);
    c.trm1 = (tr - 1) | ((tr - 1) << 16);
    c.low5 = 0x001F001Fu;
    c.hbmask = 0xFFE0FFE0u;
    c.zero = 0u;
    return c;
}

// Same function as merge_word_scalar (checked exhaustively over hb in {0..3, 31, 100, 1000,
// 2046, 2047} x every ts5 x every t5 x tr in {1, 5, 20, 31}):
//   present e:  m = max(v & hbmask, e); e' = m + (m != e) * t5
//   absent e:   e' = v if v present and (t5 + 32 - ts5(v)) mod 32 < tr, else 0
__device__ inline uint32_t merge_word_packed(uint32_t e, uint32_t v, const PackedConsts &c) {
    const uint32_t m = pk_max(v & c.hbmask, e);
    const uint32_t rp = pk_mad(pk_min(pk_sub(m, e), c.one), c.t5x2, m);
    const uint32_t age = (c.t32 - (v & c.low5)) & c.low5;
    const uint32_t ok = pk_min(pk_subc(c.tr, age), pk_min(v, c.one));
    const uint32_t ra = v & pk_sub(c.zero, ok);
    return bfi(pk_sub(c.zero, pk_min(e, c.one)), rp, ra);
}

// Replace entry i (runtime, 0..7) of a 16-B lane vector.  Only ever reached on the one
// lane whose chunk holds the sender's or the receiver's own column, so the compare-select
// chain (which keeps every index compile-time: no scratch) costs nothing in the stream.
template <typename F>
__device__ inline void patch16(uint4 &w, int i, F f) {
    uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < kEntriesPerLane; ++q) {
        const int sh = (q & 1) * 16;
        const uint32_t old = (ws[q >> 1] >> sh) & 0xFFFFu;
        const uint32_t nv = f(old) & 0xFFFFu;
        if (q == i) ws[q >> 1] = (ws[q >> 1] & ~(0xFFFFu << sh)) | (nv << sh);
    }
    w = make_uint4(ws[0], ws[1], ws[2], ws[3]);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte row accesses; kNT selects the non-temporal (streaming) cache policy.  It must be
// a compile-time choice: a runtime select between the two forms is CSE'd into one plain load.
template <bool kNT>
__device__ inline uint4 ld16(const uint16_t *p) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
    u32x4 v;
    if constexpr (kNT) v = __builtin_nontemporal_load(q);
    else v = *q;
    return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool kNT>
__device__ inline void st16(uint16_t *p, const uint32_t (&w)[4]) {
    u32x4 v;
    v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3];
    u32x4 *q = reinterpret_cast<u32x4 *>(p);
    if constexpr (kNT) __builtin_nontemporal_store(v, q);
    else *q = v;
}

__device__ inline uint64_t wave_sum_u64(uint64_t v) { return wave_sum64(v); }

// rank-th set bit (0-based) of a bitmap of `words` 32-bit words, by one wave; -1 if none.
// lane_cnt / pre: this lane's popcount over its words and the exclusive prefix.
template <typename W>
__device__ inline int32_t wave_select(W word, int32_t per, uint32_t lane_cnt, uint32_t pre,
                                      uint32_t rank, int32_t lane) {
    const bool mine = rank >= pre && rank < pre + lane_cnt;
    int32_t col = -1;
    if (mine) {
        uint32_t m = rank - pre;
        for (int32_t w = 0; w < per; ++w) {
            uint32_t bw = word(lane * per + w);
            const uint32_t pc = __builtin_popcount(bw);
            if (m < pc) {
                for (uint32_t q = 0; q < m; ++q) bw &= bw - 1;
                col = (lane * per + w) * 32 + (__builtin_ffs(bw) - 1);
                break;
            }
            m -= pc;
        }
    }
    const unsigned long long owner = __ballot(mine);
    if (!owner) return -1;
    return int32_t(lane_of(uint32_t(col), __builtin_ffsll(owner) - 1));
}

__device__ inline uint32_t wave_excl_prefix(uint32_t v, int32_t, uint32_t *total) {
    const uint32_t incl = wave_incl_scan(v);
    *total = lane_of(incl, 63);
    return incl - v;
}

// JOINREP payload (the bounded introducer list, join_kernels.hpp): the B = min(intro_list,
// cnt0) ranks Philox(JOIN; t - 1, 0, r, i) chooses among node 0's cnt0 gossipable members of
// tick t - 1, resolved to this slice's columns by one forward pass of wave 0 over the
// introducer's row (512 columns per step: a ballot-free wave prefix of the step's member
// counts).  Writes the chosen (global column, entry) pairs this slice holds to jc / jv and
// returns their number (wave 0 only; every lane gets the same result).
__device__ inline int32_t join_choose(const ScaleTickArgs &a, int32_t r, int32_t t, int32_t *jc,
                                      uint32_t *jv) {
    const int32_t lane = threadIdx.x & 63;
    const int32_t cnt0 = a.cnt_prev[0];
    const int32_t B = a.intro_list < cnt0 ? a.intro_list : cnt0;
    int32_t ranks[kMaxIntro];
    int32_t nch = 0;
    for (int32_t i = 0; i < B; ++i)
        next_distinct_rank(draw_u31(kDomainJoin, a.seed, uint32_t(t - 1), 0u, uint32_t(r), uint32_t(i)),
                           cnt0, i, ranks, nch);
    int32_t pre = 0, own = cnt0;          // ranks [pre, pre + own) live in this slice
    if (a.intro_cnt) {
        own = a.intro_cnt[int64_t(a.shard) * a.n];
        for (int32_t g = 0; g < a.shard; ++g) pre += a.intro_cnt[int64_t(g) * a.n];
    }
    const uint32_t tf = uint32_t(a.tfail), t5m1 = uint32_t(t - 1) & 31u;
    int32_t q = 0, found = 0;
    while (q < B && ranks[q] < pre) ++q;
    int32_t seen = pre;                   // gossipable members before the current step
    for (int64_t c0 = 0; c0 < a.stride && q < B && ranks[q] < pre + own; c0 += 512) {
        const int64_t c = c0 + int64_t(lane) * 8;
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        if (c < a.stride) {
            const uint4 v = *reinterpret_cast<const uint4 *>(a.intro + c);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        }
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const uint32_t ent = (w[e >> 1] >> ((e & 1) * 16)) & 0xFFFFu;
            const bool g = ent && (tf == 0 || ((t5m1 - ent) & 31u) < tf);
            bits |= (g ? 1u : 0u) << e;
        }
        const uint32_t cnt = __builtin_popcount(bits);
        const uint32_t incl = wave_incl_scan(cnt);
        const int32_t total = int32_t(lane_of(incl, 63));
        while (q < B && ranks[q] < seen + total) {
            const uint32_t want = uint32_t(ranks[q] - seen);          // rank within the step
            const bool mine = want >= incl - cnt && want < incl;
            const unsigned long long who = __ballot(mine);
            const int32_t l = __builtin_ffsll(who) - 1;
            uint32_t col = 0, val = 0;
            if (mine) {
                uint32_t m = want - (incl - cnt), bb = bits;
                for (uint32_t z = 0; z < m; ++z) bb &= bb - 1;
                const int e = __builtin_ffs(bb) - 1;
                col = uint32_t(c) + uint32_t(e);
                val = (w[e >> 1] >> ((e & 1) * 16)) & 0xFFFFu;
            }
            col = lane_of(col, l);
            val = lane_of(val, l);
            if (found < kMaxIntro) {
                jc[found] = int32_t(int64_t(a.col0) + col);
                jv[found] = val;
            }
            found++;
            q++;
        }
        seen += total;
    }
    return found;
}

// A receiver segment longer than the LDS sort holds (k > kMaxSegment, e.g. a join burst on the
// introducer): sorted in place in HBM by the row's workgroup into the canonical receipt order
// (ascending sender; MP1Node::checkMessages drains a queue of any length, MP1Node.cpp:200-212),
// slots moved along.  An all-ascending bitonic network over the next power of two: every
// compare-exchange keeps the smaller key at the lower index, so the virtual +inf keys past k
// never move and pairs reaching past k are skipped.  A segment belongs to one workgroup per
// launch, and the launches that share a CSR (column tiles) run in stream order, so a later
// launch re-sorts a sorted segment.
__device__ inline void sort_long_segment(int32_t *src, int32_t *slot, int32_t k) {
    int32_t P = 1;
    while (P < k) P <<= 1;
    for (int32_t size = 2; size <= P; size <<= 1) {
        for (int32_t half = size >> 1; half > 0; half >>= 1) {
            for (int32_t i = int32_t(threadIdx.x); i < (P >> 1); i += kScaleBlock) {
                const int32_t b = i / half, o = i - b * half;
                const bool flip = half == (size >> 1);   // pair i with its mirror in the block
                const int32_t lo = flip ? b * size + o : b * 2 * half + o;
                const int32_t hi = flip ? b * size + size - 1 - o : lo + half;
                if (hi >= k) continue;
                const int32_t x = src[lo], y = src[hi];
                if (y < x) {
                    src[lo] = y;
                    src[hi] = x;
                    if (slot) {
                        const int32_t u = slot[lo];
                        slot[lo] = slot[hi];
                        slot[hi] = u;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// kPolicy bit 0: non-temporal own-row loads/stores; bit 1: non-temporal sender-row loads.
// kPipe: software-pipelined chunk loads (the next chunk is requested before this one merges).
// kTfail: TFAIL suspicion (a.tfail > 0): a sender's payload holds only the members it could
// gossip at send time (t - 1 - ts < tfail), and only members with t - ts < tfail get a
// presence bit (peer choice) and count.
// kSwim: SWIM ping/ack probing (a.swim paths, oracle/scale_oracle.c): the probe this row sent at
// t - 1 is resolved after the merges (answered: ts of the target = t; unanswered: ts = t -
// TREMOVE, so the TREMOVE scan removes it), and wave 0 picks this tick's probe target.
// The row's LDS (namespace scope: one set per kernel, shared by both row forms below).
extern __shared__ __attribute__((aligned(16))) uint32_t s_bits[];   // fused: stride/32 words
__shared__ int32_t s_src[kMaxSegment];
__shared__ int32_t s_slot[kMaxSegment];
__shared__ unsigned long long s_red[4][4];
__shared__ int32_t s_jc[kMaxIntro];      // JOINREP payload: chosen columns / entries
__shared__ uint32_t s_jv[kMaxIntro];
__shared__ int32_t s_njc;
__shared__ uint32_t s_evf[4];            // event stream: staged records per wave
__shared__ unsigned long long s_evbase;

// One row lr of the tick.  kLong: a row whose segment is longer than the LDS sort (k >
// kMaxSegment, a join burst on the introducer), run by scale_long_kernel -- its own kernel,
// because any share of its state in the tick kernel's body (one body with a runtime branch, an
// inlined second copy, a called function) cost the plain rows registers: +1.1 % to +30 %
// VGPRs or SGPR spills at config 3.  The tick kernel only defers such a row (a list entry).
template <bool kInit, bool kSlice, int kMerge, int kPolicy, bool kPipe, bool kTfail, bool kSwim,
          bool kLong>
__device__ __forceinline__ void scale_tick_row(const ScaleTickArgs &a, const int32_t lr) {
    constexpr bool kNtOwn = (kPolicy & 1) != 0, kNtSrc = (kPolicy & 2) != 0;

    const int32_t tid = threadIdx.x;
    const int32_t lane = tid & 63, wave = tid >> 6;
    const int32_t r = a.row0 + lr;
    const int32_t t = a.tick;
    const int32_t F = a.fanout;

    if (!kInit && *a.err) return;      // a capacity error froze the job at an earlier tick
    // crashed (Application.cpp:186) or not started yet (Application.cpp:143): no recv, no
    // ops, no send
    if (t > a.fail_tick[r] || (a.start_tick && t < a.start_tick[r])) {
        if (!kSlice && tid < F) a.out_dst[int64_t(lr) * F + tid] = -1;
        return;
    }

    int32_t k = 0;
    // a long segment (k > kMaxSegment): sorted in HBM, its first k - kMaxSegment messages are
    // merged by the premerge below and the chunk loop merges the rest from LDS
    constexpr bool lng = kLong;
    if (!kInit) {
        const int32_t o0 = a.off[lr];
        k = a.off[lr + 1] - o0;
        if (k > a.max_segment) {      // tests only (GSP_TEST_MAX_SEGMENT): a capacity error
            if (tid == 0) atomicCAS(a.err, 0, t);
            if (!kSlice && tid < F) a.out_dst[int64_t(lr) * F + tid] = -1;
            return;
        }
        if (!lng && k > kMaxSegment) {   // deferred to scale_long_kernel (one list per CSR)
            if (tid == 0 && a.long_list)
                a.long_list[1 + atomicAdd(&a.long_list[0], 1)] = lr;
            return;
        }
    }
    if constexpr (lng) {
        const int32_t o0 = a.off[lr];
        sort_long_segment(a.csr_src + o0, a.csr_slot ? a.csr_slot + o0 : nullptr, k);
        if (tid == 0) s_src[0] = a.csr_src[o0];           // the JOINREP test below
        __syncthreads();
    } else if (!kInit) {
        const int32_t o0 = a.off[lr];
        for (int32_t i = tid; i < k; i += kScaleBlock) s_src[i] = a.csr_src[o0 + i];
        __syncthreads();
        // canonical receipt order: ascending sender (senders are distinct per receiver)
        int32_t rank[kMaxSegment / kScaleBlock], val[kMaxSegment / kScaleBlock],
            slot[kMaxSegment / kScaleBlock];
#pragma unroll
        for (int q = 0; q < kMaxSegment / kScaleBlock; ++q) {
            const int32_t i = tid + q * kScaleBlock;
            rank[q] = -1;
            if (i < k) {
                val[q] = s_src[i];
                slot[q] = a.csr_slot ? a.csr_slot[o0 + i] : val[q] - a.row0;
                int32_t rk = 0;
                for (int32_t j = 0; j < k; ++j) rk += s_src[j] < val[q];
                rank[q] = rk;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kMaxSegment / kScaleBlock; ++q)
            if (rank[q] >= 0) { s_src[rank[q]] = val[q]; s_slot[rank[q]] = slot[q]; }
        __syncthreads();
    }
    // a JOINREP (sender kJoinRepSrc, sorted first) is merged apart from the GOSSIP loop: wave 0
    // resolves its payload columns, and the GOSSIPs are s_src[jr .. k)
    int32_t jr = (!kInit && k > 0 && s_src[0] == kJoinRepSrc) ? 1 : 0;
    if (jr) {
        if (wave == 0) {
            const int32_t nj = join_choose(a, r, t, s_jc, s_jv);
            if (lane == 0) s_njc = nj < kMaxIntro ? nj : kMaxIntro;
        }
        __syncthreads();
    }
    const int32_t njc = jr ? s_njc : 0;

    const uint32_t t5 = uint32_t(t) & 31u;
    const uint32_t tr = uint32_t(a.tremove);
    const PackedConsts pc = packed_consts(t5, tr);
    const uint32_t tf = uint32_t(a.tfail);
    const uint32_t tfx2 = tf | (tf << 16);
    const uint32_t t5m1 = uint32_t(t - 1) & 31u;                  // the senders' tick, mod 32
    const uint32_t t32m1 = (t5m1 | (t5m1 << 16)) + 0x00200020u;
    // kTfail: drop the payload entries the sender had suspected when it sent (packed pair)
    auto gossiped = [&](uint32_t w) -> uint32_t {
        const uint32_t age = (t32m1 - (w & pc.low5)) & pc.low5;
        return w & pk_sub(pc.zero, pk_min(pk_subc(tfx2, age), pc.one));
    };
    // kSwim: the probe of t - 1 (target pcol, read before wave 0 rewrites a.ping[lr] below the
    // block reduction's barrier); one direct + a.swim - 1 indirect paths, each with a drop draw
    int32_t pcol = -1;
    uint32_t pts = 0;                  // the target's new ts mod 32
    if (kSwim && !kInit) {
        pcol = a.ping[lr];
        if (pcol >= 0) {
            bool ok = false;
            for (int32_t i = 0; i < a.swim; ++i) {
                const uint32_t dr = draw_u31(kDomainPing, a.seed, uint32_t(t - 1), uint32_t(r),
                                             uint32_t(pcol), uint32_t(i));
                ok = ok || int32_t(dr % 100u) >= a.drop_prev;     // paths sent at t - 1
            }
            ok = ok && t <= a.fail_tick[pcol] && (!a.start_tick || t >= a.start_tick[pcol]);
            pts = ok ? t5 : ((t5 - tr) & 31u);
        }
    }
    const int64_t stride = a.stride;
    const uint16_t *own_prev = a.prev + int64_t(lr) * stride;
    uint16_t *own_cur = a.cur + int64_t(lr) * stride;
    uint32_t live = 0, joins = 0, removes = 0;
    uint64_t hsum = 0;
    if constexpr (lng) {
        // Premerge of a long segment: the JOINREP and the GOSSIPs at sorted positions [jr, pend)
        // merged in order into the own row, written to this tick's row (read back by the chunk
        // loop as its own row, so the chunk loop merges senders [pend, k) after them: the same
        // order).  The joins made here are counted here: absent before the tick, present after
        // the premerge -- such an entry is fresh, and later merges only raise it, so the TREMOVE
        // scan never removes it -- except the own column (cleared after the merges) and an
        // unanswered probe target (made stale, then removed by the TREMOVE scan).
        const int32_t o0 = a.off[lr], pend = k - kMaxSegment;
        unsigned long long *const evb = (a.ev.buf && (a.ev.kinds & GSP_EVENTS_JOIN)) ? ev_stripe_buf(a.ev) : nullptr;
        for (int64_t c0 = 0; c0 < stride; c0 += kChunk) {
            const int64_t lc0 = c0 + int64_t(tid) * kEntriesPerLane, gc0 = a.col0 + lc0;
            uint4 e = ld16<false>(own_prev + lc0);
            const uint4 b = e;
            if (jr) {
                const int64_t d0 = -gc0;
                if (d0 >= 0 && d0 < kEntriesPerLane)
                    patch16(e, int(d0), [t5](uint32_t old) { return old ? ((((old >> 5) + 1u) << 5) | t5)
                                                                        : ((1u << 5) | t5); });
                for (int32_t q = 0; q < njc; ++q) {
                    const int64_t dq = int64_t(s_jc[q]) - gc0;
                    const uint32_t v = s_jv[q];
                    if (dq >= 0 && dq < kEntriesPerLane)
                        patch16(e, int(dq), [v, t5, tr](uint32_t old) { return merge_entry(old, v, t5, tr); });
                }
            }
            for (int32_t j = jr; j < pend; ++j) {
                const int32_t sj = a.csr_src[o0 + j];
                const int32_t sl = a.csr_slot ? a.csr_slot[o0 + j] : sj - a.row0;
                const uint16_t *row = sl >= 0 ? a.prev + int64_t(sl) * stride : a.remote + int64_t(-sl - 1) * stride;
                uint4 v = ld16<false>(row + lc0);
                if (kTfail) {
                    v.x = gossiped(v.x);
                    v.y = gossiped(v.y);
                    v.z = gossiped(v.z);
                    v.w = gossiped(v.w);
                }
                e.x = merge_word_scalar(e.x, v.x, t5, tr);
                e.y = merge_word_scalar(e.y, v.y, t5, tr);
                e.z = merge_word_scalar(e.z, v.z, t5, tr);
                e.w = merge_word_scalar(e.w, v.w, t5, tr);
                const int64_t ds = int64_t(sj) - gc0;
                if (ds >= 0 && ds < kEntriesPerLane)
                    patch16(e, int(ds), [t5](uint32_t old) { return (((old >> 5) + 1u) << 5) | t5; });
            }
            const uint32_t bw[4] = {b.x, b.y, b.z, b.w};
            const uint32_t ew[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
            for (int i = 0; i < kEntriesPerLane; ++i) {
                const int sh = (i & 1) * 16;
                const int64_t col = gc0 + i;
                const bool before = (bw[i >> 1] >> sh) & 0xFFFFu, after = (ew[i >> 1] >> sh) & 0xFFFFu;
                if (!before && after && col != r && !(kSwim && col == pcol && pts != t5)) {
                    joins++;
                    hsum += event_mix(1, uint32_t(t), uint32_t(r), uint32_t(col));
                    if (evb) {
                        const unsigned long long p = atomicAdd(ev_stripe_count(a.ev), 1ull);
                        if (int64_t(p) < a.ev.cap) evb[p] = event_record(1u, uint32_t(t), uint32_t(r), uint32_t(col));
                    }
                }
            }
            st16<false>(own_cur + lc0, ew);
        }
        // the chunk loop: the own row is the premerged one, the senders the last kMaxSegment
        for (int32_t i = tid; i < kMaxSegment; i += kScaleBlock) {
            const int32_t sj = a.csr_src[o0 + pend + i];
            s_src[i] = sj;
            s_slot[i] = a.csr_slot ? a.csr_slot[o0 + pend + i] : sj - a.row0;
        }
        __syncthreads();
        own_prev = own_cur;
        jr = 0;
        k = kMaxSegment;
    }
    // event stream: each wave stages its records as kind << 30 | column in LDS (after the
    // bitmap, kEvStage words per wave) and the row takes one ring reservation at its end; a
    // wave whose stage would overflow flushes it with a reservation of its own
    uint32_t *const s_ev = s_bits + (kSlice ? 4 : (stride >> 5)) + wave * kEvStage;
    uint32_t ev_fill = 0;                                           // wave-uniform
    unsigned long long *const ev_buf = a.ev.buf ? ev_stripe_buf(a.ev) : nullptr;
    unsigned long long *const ev_count = ev_stripe_count(a.ev);
    auto ev_flush = [&](uint32_t fill, unsigned long long base) {   // fill records -> ring
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = uint32_t(lane); i < fill; i += 64) {
            const uint32_t s = s_ev[i];
            if (int64_t(base + i) < a.ev.cap)
                ev_buf[base + i] = event_record(s >> 30, uint32_t(t), uint32_t(r), s & 0x3FFFFFFFu);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };

    // kPipe: the first 4 sender rows as wave-uniform (scalar) pointers, and the request of one
    // chunk's own + sender vectors (16 B per lane each) issued one chunk ahead
    const uint16_t *srow[4];
    uint4 pe = make_uint4(0u, 0u, 0u, 0u), pv[4];
    auto issue = [&](int64_t col) {
        pe = ld16<kNtOwn>(own_prev + col);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (jr + u < k) pv[u] = ld16<kNtSrc>(srow[u] + col);
    };
    if (kPipe && !kInit) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pv[u] = make_uint4(0u, 0u, 0u, 0u);
            const int32_t sl = __builtin_amdgcn_readfirstlane(jr + u < k ? s_slot[jr + u] : 0);
            srow[u] = sl >= 0 ? a.prev + int64_t(sl) * stride : a.remote + int64_t(-sl - 1) * stride;
        }
        issue(int64_t(tid) * kEntriesPerLane);
    }

    for (int64_t c0 = 0; c0 < stride; c0 += kChunk) {
        const int64_t lc0 = c0 + int64_t(tid) * kEntriesPerLane;   // column in this table
        const int64_t gc0 = a.col0 + lc0;                            // global column
        uint32_t ws[4];
        uint32_t w0[4] = {0u, 0u, 0u, 0u};
        if (kInit) {
            // pre-joined: the nodes that start at tick 0 list each other (h0, ts 0)
            const bool late_row = a.start_tick && a.start_tick[r] > 0;
            const uint32_t h = uint32_t(a.h0) << 5;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t x0 = gc0 + 2 * i, x1 = x0 + 1;
                bool on0 = x0 < a.n && x0 != r && !late_row, on1 = x1 < a.n && x1 != r && !late_row;
                if (a.start_tick) {
                    on0 = on0 && a.start_tick[x0] == 0;
                    on1 = on1 && a.start_tick[x1] == 0;
                }
                ws[i] = (on0 ? h : 0u) | ((on1 ? h : 0u) << 16);
            }
        } else {
            uint4 e;
            uint4 cv[4];
            if (kPipe) {
                // chunk c's own and first 4 sender vectors arrived with the previous request;
                // chunk c + 1's are requested before chunk c is merged
                e = pe;
#pragma unroll
                for (int u = 0; u < 4; ++u) cv[u] = pv[u];
                if (c0 + kChunk < stride) issue(lc0 + kChunk);
            } else {
                e = ld16<kNtOwn>(own_prev + lc0);
            }
            w0[0] = e.x; w0[1] = e.y; w0[2] = e.z; w0[3] = e.w;
            if (jr) {                         // the JOINREP: the introducer's sender entry
                const int64_t d0 = -gc0;      // (MP1Node.cpp:237-243), then its chosen members
                if (d0 >= 0 && d0 < kEntriesPerLane)
                    patch16(e, int(d0), [t5](uint32_t old) { return old ? ((((old >> 5) + 1u) << 5) | t5)
                                                                        : ((1u << 5) | t5); });
                for (int32_t q = 0; q < njc; ++q) {
                    const int64_t dq = int64_t(s_jc[q]) - gc0;
                    const uint32_t v = s_jv[q];
                    if (dq >= 0 && dq < kEntriesPerLane)
                        patch16(e, int(dq), [v, t5, tr](uint32_t old) { return merge_entry(old, v, t5, tr); });
                }
            }
            for (int32_t j0 = jr; j0 < k; j0 += 4) {
                uint4 v[4];
                if (kPipe && j0 == jr) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) v[u] = cv[u];
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (j0 + u < k) {
                            const int32_t sl = s_slot[j0 + u];
                            const uint16_t *row = sl >= 0 ? a.prev + int64_t(sl) * stride
                                                          : a.remote + int64_t(-sl - 1) * stride;
                            v[u] = ld16<kNtSrc>(row + lc0);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (j0 + u >= k) break;
                    if (kTfail) {
                        v[u].x = gossiped(v[u].x);
                        v[u].y = gossiped(v[u].y);
                        v[u].z = gossiped(v[u].z);
                        v[u].w = gossiped(v[u].w);
                    }
                    if (kMerge == 1) {
                        e.x = merge_word_packed(e.x, v[u].x, pc);
                        e.y = merge_word_packed(e.y, v[u].y, pc);
                        e.z = merge_word_packed(e.z, v[u].z, pc);
                        e.w = merge_word_packed(e.w, v[u].w, pc);
                    } else {
                        e.x = merge_word_scalar(e.x, v[u].x, t5, tr);
                        e.y = merge_word_scalar(e.y, v[u].y, t5, tr);
                        e.z = merge_word_scalar(e.z, v[u].z, t5, tr);
                        e.w = merge_word_scalar(e.w, v[u].w, t5, tr);
                    }
                    // the sender's own entry: hb + 1 and ts = now, or add (1, now)
                    // (MP1Node.cpp:237-243); the sender's row never holds itself
                    const int64_t ds = int64_t(s_src[j0 + u]) - gc0;
                    if (ds >= 0 && ds < kEntriesPerLane)
                        patch16(e, int(ds), [t5](uint32_t old) { return (((old >> 5) + 1u) << 5) | t5; });
                }
            }
            const int64_t dr = int64_t(r) - gc0;      // never list yourself (MP1Node.cpp:290)
            if (dr >= 0 && dr < kEntriesPerLane) patch16(e, int(dr), [](uint32_t) { return 0u; });
            if (kSwim && pcol >= 0) {                 // the probe's answer (or its absence)
                const int64_t dp = int64_t(pcol) - gc0;
                if (dp >= 0 && dp < kEntriesPerLane)
                    patch16(e, int(dp), [pts](uint32_t old) { return old ? ((old & 0xFFE0u) | pts) : 0u; });
            }
            ws[0] = e.x; ws[1] = e.y; ws[2] = e.z; ws[3] = e.w;
        }

        // TREMOVE scan, events and presence bits of the 8 entries
        bool slow = !kInit;
        uint32_t bits = 0;
        if (kMerge == 1 && !kInit) {
            uint32_t ev = 0, q = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t pe = pk_min(ws[i], pc.one);
                const uint32_t age = (pc.t32 - (ws[i] & pc.low5)) & pc.low5;
                ev |= pk_min(pk_subc(age, pc.trm1), pe);          // present and stale
                ev |= pk_subc(pe, pk_min(w0[i], pc.one));          // absent before, present now
                const uint32_t pg = kTfail ? pk_min(pe, pk_min(pk_subc(tfx2, age), pc.one)) : pe;
                q |= ((pg | (pg >> 15)) & 3u) << (2 * i);
            }
            slow = ev != 0;
            bits = q;
        }
        uint32_t evj = 0, evr = 0;            // this chunk's join / remove entries (event stream)
        if (kInit || slow) {
            bits = 0;
#pragma unroll
            for (int i = 0; i < kEntriesPerLane; ++i) {
                const int sh = (i & 1) * 16;
                uint32_t ent = (ws[i >> 1] >> sh) & 0xFFFFu;
                if (!kInit && ent) {
                    const uint32_t before = (w0[i >> 1] >> sh) & 0xFFFFu;
                    if (((t5 - ent) & 31u) >= tr) {     // TREMOVE scan (MP1Node.cpp:340)
                        removes++;
                        hsum += event_mix(2, uint32_t(t), uint32_t(r), uint32_t(gc0 + i));
                        ws[i >> 1] &= ~(0xFFFFu << sh);
                        ent = 0;
                        evr |= 1u << i;
                    } else if (!before) {
                        joins++;
                        hsum += event_mix(1, uint32_t(t), uint32_t(r), uint32_t(gc0 + i));
                        evj |= 1u << i;
                    }
                }
                const bool counted = ent && (!kTfail || ((t5 - ent) & 31u) < tf);
                bits |= (counted ? 1u : 0u) << i;
            }
        }
        if (!kInit && ev_buf) {               // the event stream: stage this chunk's records
            uint32_t both = ((a.ev.kinds & GSP_EVENTS_JOIN) ? evj : 0u) |
                            ((a.ev.kinds & GSP_EVENTS_REMOVE) ? (evr << 8) : 0u);
            const uint32_t cnt = uint32_t(__builtin_popcount(both));
            if (__ballot(cnt > 0)) {          // wave-uniform
                const uint32_t incl = wave_incl_scan(cnt);
                const uint32_t total = lane_of(incl, 63);
                if (ev_fill + total > uint32_t(kEvStage)) {
                    unsigned long long base = 0;
                    if (lane == 0) base = atomicAdd(ev_count, (unsigned long long)ev_fill);
                    base = (uint64_t(lane_of(uint32_t(base >> 32), 0)) << 32) | lane_of(uint32_t(base), 0);
                    ev_flush(ev_fill, base);
                    ev_fill = 0;
                }
                uint32_t p = ev_fill + incl - cnt;
                while (both) {
                    const uint32_t b = uint32_t(__builtin_ffs(both) - 1);
                    both &= both - 1;
                    s_ev[p++] = ((b < 8 ? 1u : 2u) << 30) | uint32_t(gc0 + (b & 7u));
                }
                ev_fill += total;
            }
        }
        live += __builtin_popcount(bits);
        st16<kNtOwn>(own_cur + lc0, ws);
        // presence bitmap: 8 bits per lane -> byte (lc0 / 8)
        if (kSlice)
            a.bitmap[int64_t(lr) * (stride >> 3) + (lc0 >> 3)] = uint8_t(bits);
        else
            reinterpret_cast<uint8_t *>(s_bits)[lc0 >> 3] = uint8_t(bits);
    }

    // block reduction: live, joins, removes, hash
    const uint64_t v0 = wave_sum_u64(live), v1 = wave_sum_u64(joins), v2 = wave_sum_u64(removes);
    const uint64_t v3 = wave_sum_u64(hsum);
    if (lane == 0) { s_red[wave][0] = v0; s_red[wave][1] = v1; s_red[wave][2] = v2; s_red[wave][3] = v3; }
    if (!kInit && ev_buf && lane == 0) s_evf[wave] = ev_fill;
    __syncthreads();
    const uint64_t tot_live = s_red[0][0] + s_red[1][0] + s_red[2][0] + s_red[3][0];
    if (!kInit && ev_buf) {                   // the row's one ring reservation
        const uint32_t f0 = s_evf[0], f1 = s_evf[1], f2 = s_evf[2], f3 = s_evf[3];
        if (tid == 0 && f0 + f1 + f2 + f3) s_evbase = atomicAdd(ev_count, (unsigned long long)(f0 + f1 + f2 + f3));
        __syncthreads();
        if (f0 + f1 + f2 + f3) {
            const uint32_t before = (wave > 0 ? f0 : 0u) + (wave > 1 ? f1 : 0u) + (wave > 2 ? f2 : 0u);
            ev_flush(ev_fill, s_evbase + before);
        }
    }

    unsigned long long *dig = a.dig + (blockIdx.x % kDigSlots) * kDigFields;
    if (tid == 0) {
        a.cnt_cur[r] = int32_t(tot_live);
        if (!kInit) {
            a.own_hb[lr] += 1;
            if (a.count_rounds) {
                unsigned long long merges = 0;
                if (jr) {                     // a JOINREP carries min(B, cnt0) members
                    const int32_t c0 = a.cnt_prev[0];
                    merges += 1ull + uint64_t(a.intro_list < c0 ? a.intro_list : c0);
                }
                // the whole segment (a long one's premerged part too, from the sorted CSR)
                int32_t ka = k;
                if constexpr (lng) {
                    const int32_t o0 = a.off[lr];
                    ka = a.off[lr + 1] - o0;
                    if (a.csr_src[o0] == kJoinRepSrc) {   // the JOINREP went to the premerge
                        const int32_t c0 = a.cnt_prev[0];
                        merges += 1ull + uint64_t(a.intro_list < c0 ? a.intro_list : c0);
                    }
                    for (int32_t j = a.csr_src[o0] == kJoinRepSrc ? 1 : 0; j < ka; ++j)
                        merges += 1ull + uint64_t(a.cnt_prev[a.csr_src[o0 + j]]);
                } else {
                    for (int32_t j = jr; j < k; ++j) merges += 1ull + uint64_t(a.cnt_prev[s_src[j]]);
                }
                atomicAdd(&dig[kDigRounds], 1ull);
                atomicAdd(&dig[kDigMerges], merges);
                atomicAdd(&dig[kDigDelivered], (unsigned long long)ka);
            }
            atomicAdd(&dig[kDigJoins], s_red[0][1] + s_red[1][1] + s_red[2][1] + s_red[3][1]);
            atomicAdd(&dig[kDigRemoves], s_red[0][2] + s_red[1][2] + s_red[2][2] + s_red[3][2]);
            atomicAdd(&dig[kDigHash], s_red[0][3] + s_red[1][3] + s_red[2][3] + s_red[3][3]);
        }
    }
    if (kSlice) return;

    // send: wave 0 picks min(F, live) distinct members by Philox rank-select
    if (wave == 0) {
        const int32_t per = int32_t(stride >> 5) >> 6;   // bitmap words per lane
        uint32_t lane_cnt = 0;
        for (int32_t w = 0; w < per; ++w) lane_cnt += __builtin_popcount(s_bits[lane * per + w]);
        uint32_t total = 0;
        const uint32_t pre = wave_excl_prefix(lane_cnt, lane, &total);
        const int32_t cnt = int32_t(tot_live);
        const int32_t keff = F < cnt ? F : cnt;
        int32_t chosen[16];
        int32_t nch = 0;
        unsigned long long sent = 0, dropped = 0;
        for (int32_t kk = 0; kk < F; ++kk) {
            int32_t dst = -1;
            if (kk < keff) {
                const uint32_t u = draw_u31(kDomainPeer, a.seed, uint32_t(t), uint32_t(r),
                                            uint32_t(kk), 0u);
                const int32_t rk = next_distinct_rank(u, cnt, kk, chosen, nch);
                dst = wave_select([&](int32_t w) { return s_bits[w]; }, per, lane_cnt, pre,
                                  uint32_t(rk), lane);
                sent++;
                const uint32_t dr = draw_u31(kDomainSend, a.seed, uint32_t(t), uint32_t(r),
                                             uint32_t(dst), 3u);
                if (int32_t(dr % 100u) < a.drop_pct) { dropped++; dst = -1; }
            }
            if (lane == 0) {
                a.out_dst[int64_t(lr) * F + kk] = dst;
                if (dst >= 0) atomicAdd(&a.deg[dst], 1);
            }
        }
        if (lane == 0 && sent) {
            atomicAdd(&dig[kDigSent], sent);
            atomicAdd(&dig[kDigDropped], dropped);
        }
        if (kSwim) {                                  // this tick's probe target
            int32_t p = -1;
            if (cnt > 0) {
                const uint32_t u = draw_u31(kDomainPing, a.seed, uint32_t(t), uint32_t(r), 0u, 0x100u);
                p = wave_select([&](int32_t w) { return s_bits[w]; }, per, lane_cnt, pre,
                                u % uint32_t(cnt), lane);
            }
            if (lane == 0) a.ping[lr] = p;
        }
    }
}

template <bool kInit, bool kSlice, int kMerge, int kPolicy, bool kPipe = false, bool kTfail = false,
          bool kSwim = false>
__global__ void __launch_bounds__(kScaleBlock) scale_tick_kernel(ScaleTickArgs a) {
    scale_tick_row<kInit, kSlice, kMerge, kPolicy, kPipe, kTfail, kSwim, false>(a, int32_t(blockIdx.x));
}

// The rows the tick kernels deferred (k > kMaxSegment), after every tick-kernel launch of the
// tick: tile g's args are its template of this tick's parity (made by the host, upload_long_tpl
// in scale_engine.cpp) with the tick's own fields patched below -- tick, drop_pct, drop_prev,
// the digest offset; a per-tick args field not in that list must be added there; each tile's list is its CSR's (the tiles of an in-process group share
// one).  Launched once per tick; without a deferred row every workgroup reads the counts and
// exits.  It also clears the lists of the next tick's parity.
template <bool kSlice, bool kTfail, bool kSwim>
__global__ void __launch_bounds__(kScaleBlock) scale_long_kernel(ScaleTickArgs a, const ScaleTickArgs *tpl,
                                                                 int32_t ntiles) {
    const int32_t t = a.tick;
    for (int32_t g = 0; g < ntiles; ++g) {
        ScaleTickArgs ag = tpl[2 * g + (t & 1)];
        ag.tick = t;
        ag.drop_pct = a.drop_pct;
        ag.drop_prev = a.drop_prev;
        ag.dig += size_t(t) * kDigSlots * kDigFields;
        const int32_t cnt = ag.long_list[0];
        for (int32_t i = int32_t(blockIdx.x); i < cnt; i += int32_t(gridDim.x)) {
            scale_tick_row<false, kSlice, 1, 0, false, kTfail, kSwim, true>(ag, ag.long_list[1 + i]);
            __syncthreads();                    // the row's LDS is read to its end
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int32_t g = 0; g < ntiles; ++g) tpl[2 * g + ((t + 1) & 1)].long_list[0] = 0;
}

// Column mode: one wave per sender.  The global member order of row s is the shards'
// slices in ascending column order, so rank rk lives on the first shard whose inclusive
// prefix of slice counts exceeds rk; that shard resolves the column from its bitmap.
__global__ void __launch_bounds__(256) scale_resolve_kernel(ScaleResolveArgs a) {
    const int32_t lane = threadIdx.x & 63;
    const int32_t s = int32_t(blockIdx.x) * 4 + int32_t(threadIdx.x >> 6);
    if (s >= a.n) return;
    const int32_t F = a.fanout;
    const int32_t W = F + (a.swim > 0 ? 1 : 0);        // pick slots per sender
    if (a.tick > a.fail_tick[s] || (a.start_tick && a.tick < a.start_tick[s])) {
        if (lane < W) a.picks[int64_t(s) * W + lane] = -1;
        return;
    }
    const uint32_t c = lane < a.shards ? uint32_t(a.cnt_all[int64_t(lane) * a.n + s]) : 0u;
    uint32_t total = 0;
    const uint32_t cpre = wave_excl_prefix(c, lane, &total);
    if (lane == 0) a.cnt_total[s] = int32_t(total);
    const int32_t cnt = int32_t(total);
    const int32_t keff = F < cnt ? F : cnt;
    const int32_t per = int32_t(a.stride >> 5) >> 6;
    // the bitmap of shard g's slice of row s, and its per-lane popcounts / prefix (cached for
    // the last shard used: a sender's picks fall into few shards' slices)
    const uint32_t *bm = nullptr;
    int32_t bm_g = -1;
    uint32_t lane_cnt = 0, pre = 0;
    auto resolve = [&](uint32_t rk) -> int32_t {        // wave-uniform rank -> column or -1
        const unsigned long long own = __ballot(lane < a.shards && rk >= cpre && rk < cpre + c);
        const int32_t g = __builtin_ffsll(own) - 1;
        if (a.tiled ? (g < a.tile_lo || g >= a.tile_lo + a.tile_cnt) : g != a.shard)
            return -1;                                   // another shard / rank resolves it
        if (g != bm_g) {
            bm = reinterpret_cast<const uint32_t *>(a.bitmap + (a.tiled ? int64_t(g - a.tile_lo) * a.tile_bytes : 0) +
                                                    int64_t(s) * (a.stride >> 3));
            lane_cnt = 0;
            for (int32_t w = 0; w < per; ++w) lane_cnt += __builtin_popcount(bm[lane * per + w]);
            uint32_t tot = 0;
            pre = wave_excl_prefix(lane_cnt, lane, &tot);
            bm_g = g;
        }
        const uint32_t local = rk - __shfl(cpre, g, 64);
        const int32_t col = wave_select([&](int32_t w) { return bm[w]; }, per, lane_cnt, pre, local, lane);
        return int32_t(int64_t(g) * a.stride + col);
    };
    int32_t chosen[16];
    int32_t nch = 0;
    for (int32_t kk = 0; kk < F; ++kk) {
        int32_t pick = -1;
        if (kk < keff) {
            const uint32_t u = draw_u31(kDomainPeer, a.seed, uint32_t(a.tick), uint32_t(s),
                                        uint32_t(kk), 0u);
            pick = resolve(uint32_t(next_distinct_rank(u, cnt, kk, chosen, nch)));
        }
        if (lane == 0) a.picks[int64_t(s) * W + kk] = pick;
    }
    if (a.swim > 0) {      // the probe target: one more rank-select over the same global order
        int32_t pick = -1;
        if (cnt > 0) {
            const uint32_t u = draw_u31(kDomainPing, a.seed, uint32_t(a.tick), uint32_t(s), 0u, 0x100u);
            pick = resolve(u % uint32_t(cnt));
        }
        if (lane == 0) a.picks[int64_t(s) * W + F] = pick;
    }
    if (lane == 0 && a.count_rounds && keff > 0)
        atomicAdd(&a.dig[(s % kDigSlots) * kDigFields + kDigSent], (unsigned long long)keff);
}

__global__ void scale_finalize_kernel(ScaleResolveArgs a) {
    const int64_t slots = int64_t(a.n) * a.fanout;
    const int32_t W = a.fanout + (a.swim > 0 ? 1 : 0);
    unsigned long long dropped = 0;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < slots;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int32_t s = int32_t(i / a.fanout);
        if (a.swim > 0 && i % a.fanout == 0) a.ping[s] = a.picks[int64_t(s) * W + a.fanout];
        int32_t d = a.picks[int64_t(s) * W + (i - int64_t(s) * a.fanout)];
        if (d >= 0) {
            const uint32_t dr = draw_u31(kDomainSend, a.seed, uint32_t(a.tick), uint32_t(s),
                                         uint32_t(d), 3u);
            if (int32_t(dr % 100u) < a.drop_pct) { dropped++; d = -1; }
            else atomicAdd(&a.deg[d], 1);
        }
        a.out_dst[i] = d;
    }
    dropped = wave_sum_u64(dropped);
    if ((threadIdx.x & 63) == 0 && dropped && a.count_rounds)
        atomicAdd(&a.dig[(blockIdx.x % kDigSlots) * kDigFields + kDigDropped], dropped);
}

__global__ void max_into_kernel(int32_t *dst, const int32_t *src, int64_t count) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < count;
         i += int64_t(gridDim.x) * blockDim.x)
        dst[i] = max(dst[i], src[i]);
}

// Exclusive scan of the destination counts, two launches: (1) every 1024-thread block sums
// its kScanTile elements; (2) every block adds the sums of the blocks before it (at most
// a few hundred values, read from L2) to an in-block scan of its tile.
constexpr int kScanThreads = 1024, kScanPer = 4, kScanTile = kScanThreads * kScanPer;

__device__ inline int32_t block_scan_incl(int32_t v, int32_t *s_wave) {
    const int32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int32_t u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    if (lane == 63) s_wave[wave] = v;
    __syncthreads();
    if (wave == 0) {
        int32_t w = lane < 16 ? s_wave[lane] : 0;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const int32_t u = __shfl_up(w, d, 64);
            if (lane >= d) w += u;
        }
        if (lane < 16) s_wave[lane] = w;
    }
    __syncthreads();
    return v + (wave ? s_wave[wave - 1] : 0);
}

__global__ void __launch_bounds__(kScanThreads) tile_sum_kernel(const int32_t *deg, int32_t n,
                                                                int32_t *tile_sum) {
    __shared__ int32_t s_wave[16];
    const int64_t base = int64_t(blockIdx.x) * kScanTile + int64_t(threadIdx.x) * kScanPer;
    int32_t v = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i)
        if (base + i < n) v += deg[base + i];
    const int32_t incl = block_scan_incl(v, s_wave);
    if (threadIdx.x == kScanThreads - 1) tile_sum[blockIdx.x] = incl;
}

__global__ void __launch_bounds__(kScanThreads) tile_scan_kernel(const int32_t *deg, int32_t n,
                                                                 const int32_t *tile_sum,
                                                                 int32_t *off) {
    __shared__ int32_t s_wave[16];
    __shared__ int32_t s_base;
    if (threadIdx.x < 64) {
        int32_t acc = 0;
        for (int32_t b = threadIdx.x; b < int32_t(blockIdx.x); b += 64) acc += tile_sum[b];
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) acc += __shfl_xor(acc, d, 64);
        if (threadIdx.x == 0) s_base = acc;
    }
    __syncthreads();
    const int64_t base = int64_t(blockIdx.x) * kScanTile + int64_t(threadIdx.x) * kScanPer;
    int32_t v[kScanPer];
    int32_t sum = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        v[i] = base + i < n ? deg[base + i] : 0;
        sum += v[i];
    }
    int32_t run = block_scan_incl(sum, s_wave) - sum + s_base;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        if (base + i < n) off[base + i] = run;
        run += v[i];
    }
    if (base < n && base + kScanPer >= n) off[n] = run;   // the thread holding element n-1
}

__global__ void scatter_kernel(const int32_t *out_dst, int64_t slots, int32_t fanout,
                               int32_t row0, const int32_t *off, int32_t *fill,
                               int32_t *csr_src) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < slots;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int32_t d = out_dst[i];
        if (d < 0) continue;
        const int32_t p = atomicAdd(&fill[d], 1);
        csr_src[off[d] + p] = row0 + int32_t(i / fanout);
    }
}

// the capacity test of the tick kernel, ahead of it (row shards of a communicator: the flag is
// then all-reduced, so every rank's tick kernels of t see it)
__global__ void segment_check_kernel(const int32_t *off, int32_t rows, int32_t max_segment, int32_t *err,
                                     int32_t t) {
    for (int32_t i = int32_t(blockIdx.x * blockDim.x + threadIdx.x); i < rows; i += int32_t(gridDim.x * blockDim.x))
        if (off[i + 1] - off[i] > max_segment) atomicCAS(err, 0, t);
}

unsigned grid_for(int64_t items, int64_t per_block, int64_t cap) {
    int64_t b = (items + per_block - 1) / per_block;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return unsigned(b);
}

}  // namespace

size_t scale_lds_bytes(int64_t stride, bool slice, bool events) {
    return (slice ? 16 : size_t(stride / 8)) + (events ? size_t(4 * kEvStage * 4) : 0);
}

hipError_t launch_scale_init(const ScaleTickArgs &a, bool slice, hipStream_t st) {
    if (a.stride % kChunk || a.fanout < 1 || a.fanout > 16) return hipErrorInvalidValue;
    const size_t lds = scale_lds_bytes(a.stride, slice, false);
    if (slice)
        hipLaunchKernelGGL((scale_tick_kernel<true, true, 1, 0>), dim3(a.rows), dim3(kScaleBlock), lds, st, a);
    else if (a.swim > 0)
        hipLaunchKernelGGL((scale_tick_kernel<true, false, 1, 0, false, false, true>), dim3(a.rows),
                           dim3(kScaleBlock), lds, st, a);
    else
        hipLaunchKernelGGL((scale_tick_kernel<true, false, 1, 0>), dim3(a.rows), dim3(kScaleBlock), lds, st, a);
    return hipGetLastError();
}

template <bool kSlice, int kMerge>
void launch_tick_policy(const ScaleTickArgs &a, int policy, size_t lds, hipStream_t st) {
    const dim3 grid(a.rows), block(kScaleBlock);
    if (a.swim > 0) {
        if (a.tfail > 0)
            hipLaunchKernelGGL((scale_tick_kernel<false, kSlice, kMerge, 1, false, true, true>), grid, block, lds, st, a);
        else
            hipLaunchKernelGGL((scale_tick_kernel<false, kSlice, kMerge, 1, false, false, true>), grid, block, lds, st, a);
        return;
    }
    if (a.tfail > 0) {
        hipLaunchKernelGGL((scale_tick_kernel<false, kSlice, kMerge, 1, false, true>), grid, block, lds, st, a);
        return;
    }
    if (a.pipe && kMerge == 1 && (policy & 3) == 1) {
        hipLaunchKernelGGL((scale_tick_kernel<false, kSlice, kMerge, 1, true>), grid, block, lds, st, a);
        return;
    }
    switch (policy & 3) {
        case 0: hipLaunchKernelGGL((scale_tick_kernel<false, kSlice, kMerge, 0>), grid, block, lds, st, a); break;
        case 1: hipLaunchKernelGGL((scale_tick_kernel<false, kSlice, kMerge, 1>), grid, block, lds, st, a); break;
        case 2: hipLaunchKernelGGL((scale_tick_kernel<false, kSlice, kMerge, 2>), grid, block, lds, st, a); break;
        default: hipLaunchKernelGGL((scale_tick_kernel<false, kSlice, kMerge, 3>), grid, block, lds, st, a); break;
    }
}

hipError_t launch_scale_tick(const ScaleTickArgs &a, bool slice, int merge, hipStream_t st) {
    if (a.stride % kChunk || a.fanout < 1 || a.fanout > 16) return hipErrorInvalidValue;
    const size_t lds = scale_lds_bytes(a.stride, slice, a.ev.buf != nullptr) + size_t(a.lds_pad);
    const int policy = (a.nt_own ? 1 : 0) | (a.nt_src ? 2 : 0);
    if (slice) {
        if (merge == 1) launch_tick_policy<true, 1>(a, policy, lds, st);
        else launch_tick_policy<true, 0>(a, policy, lds, st);
    } else {
        if (merge == 1) launch_tick_policy<false, 1>(a, policy, lds, st);
        else launch_tick_policy<false, 0>(a, policy, lds, st);
    }
    return hipGetLastError();
}

hipError_t launch_scale_long(const ScaleTickArgs &a, const ScaleTickArgs *tpl, int32_t ntiles, bool slice,
                             hipStream_t st) {
    if (ntiles < 1) return hipErrorInvalidValue;
    const size_t lds = scale_lds_bytes(a.stride, slice, a.ev.buf != nullptr) + size_t(a.lds_pad);
    const dim3 grid(64), block(kScaleBlock);
    const int v = (slice ? 4 : 0) | (a.tfail > 0 ? 2 : 0) | (a.swim > 0 ? 1 : 0);
    switch (v) {
        case 0: hipLaunchKernelGGL((scale_long_kernel<false, false, false>), grid, block, lds, st, a, tpl, ntiles); break;
        case 1: hipLaunchKernelGGL((scale_long_kernel<false, false, true>), grid, block, lds, st, a, tpl, ntiles); break;
        case 2: hipLaunchKernelGGL((scale_long_kernel<false, true, false>), grid, block, lds, st, a, tpl, ntiles); break;
        case 3: hipLaunchKernelGGL((scale_long_kernel<false, true, true>), grid, block, lds, st, a, tpl, ntiles); break;
        case 4: hipLaunchKernelGGL((scale_long_kernel<true, false, false>), grid, block, lds, st, a, tpl, ntiles); break;
        case 5: hipLaunchKernelGGL((scale_long_kernel<true, false, true>), grid, block, lds, st, a, tpl, ntiles); break;
        case 6: hipLaunchKernelGGL((scale_long_kernel<true, true, false>), grid, block, lds, st, a, tpl, ntiles); break;
        default: hipLaunchKernelGGL((scale_long_kernel<true, true, true>), grid, block, lds, st, a, tpl, ntiles); break;
    }
    return hipGetLastError();
}

hipError_t launch_scale_resolve(const ScaleResolveArgs &a, hipStream_t st) {
    if (a.stride % kChunk || a.shards < 1 || a.shards > 64 || a.fanout > 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(scale_resolve_kernel, dim3(unsigned((a.n + 3) / 4)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_scale_finalize(const ScaleResolveArgs &a, hipStream_t st) {
    const int64_t slots = int64_t(a.n) * a.fanout;
    hipLaunchKernelGGL(scale_finalize_kernel, dim3(grid_for(slots, 256, 4096)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_max_into(int32_t *dst, const int32_t *src, int64_t count, hipStream_t st) {
    hipLaunchKernelGGL(max_into_kernel, dim3(grid_for(count, 256, 4096)), dim3(256), 0, st, dst, src,
                       count);
    return hipGetLastError();
}

hipError_t launch_exclusive_scan(const int32_t *deg, int32_t *off, int32_t n, int32_t *tile_sum,
                                 hipStream_t st) {
    const int32_t tiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(tile_sum_kernel, dim3(tiles), dim3(kScanThreads), 0, st, deg, n, tile_sum);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(tiles), dim3(kScanThreads), 0, st, deg, n, tile_sum,
                       off);
    return hipGetLastError();
}

hipError_t launch_segment_check(const int32_t *off, int32_t rows, int32_t max_segment, int32_t *err,
                                int32_t t, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(segment_check_kernel, dim3(grid_for(rows, 256, 1024)), dim3(256), 0, st, off, rows,
                       max_segment, err, t);
    return hipGetLastError();
}

hipError_t launch_scatter(const int32_t *out_dst, int64_t slots, int32_t fanout, int32_t row0,
                          const int32_t *off, int32_t *fill, int32_t *csr_src, hipStream_t st) {
    hipLaunchKernelGGL(scatter_kernel, dim3(grid_for(slots, 256, 4096)), dim3(256), 0, st, out_dst,
                       slots, fanout, row0, off, fill, csr_src);
    return hipGetLastError();
}

}  // namespace gsp
