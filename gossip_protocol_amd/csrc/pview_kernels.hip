// gossip_protocol_amd/csrc/pview_kernels.hip -- PARTIAL-VIEW tick kernel for gfx950.
//
// One 256-lane workgroup per receiver row; the row's work lives in ~25 KB of LDS (6 rows per
// CU in flight):
//   1. receipt order: its <= K smallest senders (canonical order; the rest = inbox overflow);
//   2. keys: its own view and the k sender views, each a sorted block of 256 slots, as 32-bit
//      keys id << 11 | source << 8 | slot (source 0 = own view, j = the payload of message j;
//      the 16-bit value hb << 5 | ts5 stays behind in vals[source][slot]), so equal ids sort
//      in message order;
//   3. union: a tree of merge-path merges (one co-rank binary search per lane per level, then
//      a register merge of the lane's kBlocks outputs): 256 -> 512 -> 1024 -> 2048 keys, with
//      the lanes past the (k + 1) * 256 real keys idle;
//   4. fold: the lane holding the first key of an id folds MP1Node::recvCallBack's rules over
//      that id's run (own entry, sender event j, payload entry j, ...; MP1Node.cpp:234-301)
//      and runs the TREMOVE test (MP1Node.cpp:339-348).  A sender found in no list becomes a
//      new (1, t) entry ("orphan"), adopted by the lane whose key range brackets its id;
//   5. survivors compacted in id order (one block scan); eviction to V by (age, -hb, id) with
//      an age histogram, an hb histogram of the boundary age and an id-order tie prefix, all
//      resolved by a single packed block scan;
//   6. the new sorted view is written back (2 KB, coalesced); Philox rank-select picks the
//      peers (draws precomputed by lanes 0..F-1, drop draws in parallel).
// HBM bytes per node-round: 2 * V * 8 (own view read + write) + k * V * 8 (sender views).
#include "philox.hpp"
#include "pview_kernels.hpp"

namespace gsp {
namespace {

constexpr int kSlots = kPvMaxView;                    // slots per source block
constexpr int kMaxBlocks = kPvMaxInbox + 1;           // own view + K sender views
constexpr int kMaxKeys = kSlots * kMaxBlocks;         // 2048
constexpr int kUCap = kMaxKeys + 8;                   // survivors + orphans
constexpr uint32_t kKeyMax = 0xFFFFFFFFu;             // id field 2^21 - 1: above every node id
static_assert(kMaxBlocks == 8, "the merge tree assumes 8 blocks of 256 keys");

__device__ inline uint64_t pv_event_mix(uint32_t kind, uint32_t t, uint32_t r, uint32_t x) {
    uint64_t z = (uint64_t(kind) << 62) | (uint64_t(t & 0xFFFFF) << 42) |
                 (uint64_t(r & 0x1FFFFF) << 21) | uint64_t(x & 0x1FFFFF);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// the reference's merge of one payload entry (packed hb << 5 | ts5, 0 = absent)
__device__ inline uint32_t pv_merge(uint32_t e, uint32_t v, uint32_t t5, uint32_t tr) {
    const uint32_t upd = ((v >> 5) > (e >> 5)) ? ((v & 0xFFE0u) | t5) : e;
    const uint32_t add = (v != 0u && ((t5 - v) & 31u) < tr) ? v : 0u;
    return e ? upd : add;
}

__device__ inline uint32_t key_id(uint32_t k) { return k >> 11; }
__device__ inline uint32_t key_src(uint32_t k) { return (k >> 8) & 7u; }
__device__ inline uint32_t key_slot(uint32_t k) { return k & 255u; }

__device__ inline uint32_t wave_sum32(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
__device__ inline uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// exclusive block scan over the 256 lanes (fenced by barriers); *total = sum of all lanes
__device__ inline uint32_t block_scan(uint32_t v, uint32_t *total, uint32_t *s_wave) {
    const int32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(incl, d, 64);
        if (lane >= d) incl += u;
    }
    __syncthreads();
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = s_wave[q];
        before += q < wave ? x : 0u;
        all += x;
    }
    *total = all;
    return incl - v + before;
}

template <int N>
__device__ inline void lds_store(uint32_t *p, const uint32_t (&v)[N]) {
    if constexpr (N == 1) {
        p[0] = v[0];
    } else if constexpr (N == 2) {
        *reinterpret_cast<uint2 *>(p) = make_uint2(v[0], v[1]);
    } else {
#pragma unroll
        for (int i = 0; i < N; i += 4)
            *reinterpret_cast<uint4 *>(p + i) = make_uint4(v[i], v[i + 1], v[i + 2], v[i + 3]);
    }
}

template <int N>
__device__ inline void lds_load(const uint32_t *p, uint32_t (&v)[N]) {
    if constexpr (N == 1) {
        v[0] = p[0];
    } else if constexpr (N == 2) {
        const uint2 x = *reinterpret_cast<const uint2 *>(p);
        v[0] = x.x; v[1] = x.y;
    } else {
#pragma unroll
        for (int i = 0; i < N; i += 4) {
            const uint4 x = *reinterpret_cast<const uint4 *>(p + i);
            v[i] = x.x; v[i + 1] = x.y; v[i + 2] = x.z; v[i + 3] = x.w;
        }
    }
}

struct alignas(16) PvShared {
    uint32_t keys[2][kUCap];             // merge ping-pong; then survivor ids (U), kept ids (W)
    uint16_t vals[kMaxKeys];             // values by (source, slot); then hb histogram; then W vals
    uint16_t uval[kUCap];                // survivor values
    uint32_t age_hist[32];
    uint32_t peer_u[16];                 // Philox peer draws of lanes 0..F-1
    int32_t pick[16], chosen[16];
    int32_t src[kPvMaxInbox], slot[kPvMaxInbox], found[kPvMaxInbox];
    int32_t misc[8];
    uint32_t wave_scan[4];
    unsigned long long red[4][4];
};

struct RowOut {
    const uint32_t *ids;
    const uint16_t *vals;
    int32_t len;
    uint32_t joins, removes, evicts;
    uint64_t hsum;
};

// Steps 2-5 for a row with k <= kBlocks - 1 merged messages (kBlocks = 1, 2, 4 or 8).
template <int kBlocks>
__device__ __forceinline__ void pv_merge_row(const PviewTickArgs &a, PvShared &sh, int32_t lr,
                                             int32_t r, int32_t k, RowOut &ro) {
    constexpr int Q = kBlocks;                           // keys per lane
    constexpr int P = kBlocks * kSlots;
    const int32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t V = a.view;
    const uint32_t t = uint32_t(a.tick), t5 = t & 31u, tr = uint32_t(a.tremove);
    const int32_t Pe = (k + 1) * kSlots;                // keys that can be real

    // ---- 2. keys: one sorted block of 256 slots per source -----------------------------------
    // every row load is issued before any is consumed (one HBM round trip, not k + 1)
    uint64_t ent[kBlocks];
#pragma unroll
    for (int m = 0; m < kBlocks; ++m) {
        ent[m] = kPvEmpty;
        if (m <= k && tid < V) {
            const uint64_t *row;
            if (m == 0) row = a.prev + int64_t(lr) * V;
            else {
                const int32_t sl = sh.slot[m - 1];
                row = sl >= 0 ? a.prev + int64_t(sl) * V : a.remote + int64_t(-sl - 1) * V;
            }
            ent[m] = __builtin_nontemporal_load(row + tid);
        }
    }
#pragma unroll
    for (int m = 0; m < kBlocks; ++m) {
        const bool ok = ent[m] != kPvEmpty;
        sh.keys[0][m * kSlots + tid] =
            ok ? (uint32_t(ent[m] >> 32) << 11) | (uint32_t(m) << 8) | uint32_t(tid) : kKeyMax;
        sh.vals[m * kSlots + tid] = uint16_t(ent[m]);
        if (m > k) sh.keys[1][m * kSlots + tid] = kKeyMax;     // padding for the ping-pong
    }
    {   // payload entries merged (MP1Node.cpp:245 loop trips): the senders' view sizes
        uint32_t ne = 0;
#pragma unroll
        for (int m = 1; m < kBlocks; ++m) ne += (m <= k && ent[m] != kPvEmpty) ? 1u : 0u;
        ne = wave_sum32(ne);
        if (lane == 0 && ne) atomicAdd(reinterpret_cast<uint32_t *>(&sh.misc[5]), ne);
    }
    __syncthreads();

    // ---- 3. merge-path tree: sorted union of every source, ties in message order ------------
    const int32_t beg = tid * Q;
    int cur = 0;
#pragma unroll
    for (int s = kSlots; s < P; s <<= 1) {
        if (beg < Pe) {
            const uint32_t *X = sh.keys[cur];
            uint32_t *Y = sh.keys[cur ^ 1];
            const int32_t b = beg / (2 * s), o = beg - b * 2 * s;
            const uint32_t *A = X + b * 2 * s, *B = A + s;
            int32_t lo = o > s ? o - s : 0, hi = o < s ? o : s;
            while (lo < hi) {                                  // co-rank of output o
                const int32_t mid = (lo + hi) >> 1;
                if (A[mid] < B[o - mid - 1]) lo = mid + 1; else hi = mid;
            }
            int32_t i = lo, j = o - lo;
            uint32_t va = i < s ? A[i] : kKeyMax, vb = j < s ? B[j] : kKeyMax;
            uint32_t outk[Q];
#pragma unroll
            for (int e = 0; e < Q; ++e) {
                const bool ta = va <= vb;                      // equal only for padding
                outk[e] = ta ? va : vb;
                i += ta ? 1 : 0;
                j += ta ? 0 : 1;
                const int32_t ii = ta ? i : j;
                const uint32_t nv = ii < s ? (ta ? A : B)[ii] : kKeyMax;
                va = ta ? nv : va;
                vb = ta ? vb : nv;
            }
            lds_store<Q>(Y + beg, outk);
        }
        __syncthreads();
        cur ^= 1;
    }
    const uint32_t *C = sh.keys[cur];

    // ---- 4. fold each id's run ------------------------------------------------------------
    uint32_t ck[Q];
    lds_load<Q>(C + beg, ck);
    const uint32_t lo_id = tid > 0 ? key_id(C[beg - 1]) + 1u : 0u;  // this lane brackets ids
    const uint32_t hi_id = tid < kPvBlock - 1 ? key_id(ck[Q - 1]) : kKeyMax;  // [lo_id, hi_id]
    uint32_t ssrc[kPvMaxInbox];
#pragma unroll
    for (int jj = 0; jj < kPvMaxInbox; ++jj) ssrc[jj] = jj < k ? uint32_t(sh.src[jj]) : kKeyMax;

    uint32_t res[Q], rid[Q];
    uint32_t nloc = 0, joins = 0, removes = 0, evicts = 0, found_mask = 0;
    uint64_t hsum = 0;
#pragma unroll
    for (int e = 0; e < Q; ++e) {
        res[e] = 0;
        rid[e] = 0;
        const uint32_t kk0 = ck[e];
        const uint32_t x = key_id(kk0);
        const bool first = e == 0 ? x >= lo_id : x != key_id(ck[e - 1]);
        if (kk0 == kKeyMax || !first) continue;
        int32_t jsend = 0;
#pragma unroll
        for (int jj = 0; jj < kPvMaxInbox; ++jj) jsend = ssrc[jj] == x ? jj + 1 : jsend;
        if (jsend) found_mask |= 1u << (jsend - 1);
        if (x == uint32_t(r)) continue;                       // never list yourself
        int32_t pos = beg + e;
        uint32_t nk = kk0, v = 0, e0 = 0;
        if (key_src(nk) == 0) {
            e0 = v = sh.vals[key_slot(nk)];
            ++pos;
            nk = pos < Pe ? C[pos] : kKeyMax;
        }
        for (int32_t jj = 1; jj <= k; ++jj) {
            if (jj == jsend) v = (((v >> 5) + 1u) << 5) | t5;              // MP1Node.cpp:237-243
            if (key_id(nk) == x && key_src(nk) == uint32_t(jj)) {
                v = pv_merge(v, sh.vals[jj * kSlots + key_slot(nk)], t5, tr);  // MP1Node.cpp:247-301
                ++pos;
                nk = pos < Pe ? C[pos] : kKeyMax;
            }
        }
        if (!v) continue;
        if (!e0) { joins++; hsum += pv_event_mix(1, t, uint32_t(r), x); }
        if (((t5 - v) & 31u) >= tr) {                          // TREMOVE scan
            removes++;
            hsum += pv_event_mix(2, t, uint32_t(r), x);
            continue;
        }
        res[e] = v;
        rid[e] = x;
        nloc++;
    }
    // candidate orphans: senders whose id falls in this lane's bracket
    uint32_t adopt = 0;
    int32_t ains[kPvMaxInbox];
#pragma unroll
    for (int jj = 0; jj < kPvMaxInbox; ++jj) {
        ains[jj] = 0;
        const uint32_t x = ssrc[jj];
        if (jj < k && x >= lo_id && x <= hi_id && beg <= Pe) {
            int32_t c = 0;
#pragma unroll
            for (int e = 0; e < Q; ++e) c += key_id(ck[e]) < x ? 1 : 0;
            ains[jj] = c;
            adopt |= 1u << jj;
        }
    }
    if (found_mask) {
#pragma unroll
        for (int jj = 0; jj < kPvMaxInbox; ++jj)
            if ((found_mask >> jj) & 1u) sh.found[jj] = 1;
    }
    __syncthreads();
    if (adopt) {
#pragma unroll
        for (int jj = 0; jj < kPvMaxInbox; ++jj) {
            if (!((adopt >> jj) & 1u)) continue;
            if (sh.found[jj]) { adopt &= ~(1u << jj); continue; }
            nloc++;
            joins++;
            hsum += pv_event_mix(1, t, uint32_t(r), ssrc[jj]);
        }
    }

    // ---- 5a. survivors (and adopted orphans), compacted in id order -------------------------
    uint32_t total = 0;
    const uint32_t base = block_scan(nloc, &total, sh.wave_scan);
    uint32_t *Uid = sh.keys[cur ^ 1];
    uint16_t *Uval = sh.uval;
    const bool evict = int32_t(total) > V;
    {
        uint32_t w = base;
        if (!adopt) {
#pragma unroll
            for (int e = 0; e < Q; ++e)
                if (res[e]) {
                    Uid[w] = rid[e];
                    Uval[w] = uint16_t(res[e]);
                    if (evict) atomicAdd(&sh.age_hist[(t5 - res[e]) & 31u], 1u);
                    w++;
                }
        } else {
            const uint32_t fresh = (1u << 5) | t5;             // an orphan: (hb 1, ts t)
#pragma unroll
            for (int e = 0; e <= Q; ++e) {
#pragma unroll
                for (int jj = 0; jj < kPvMaxInbox; ++jj)
                    if (((adopt >> jj) & 1u) && ains[jj] == e) {
                        Uid[w] = ssrc[jj];
                        Uval[w] = uint16_t(fresh);
                        if (evict) atomicAdd(&sh.age_hist[0], 1u);
                        w++;
                    }
                if (e < Q && res[e]) {
                    Uid[w] = rid[e];
                    Uval[w] = uint16_t(res[e]);
                    if (evict) atomicAdd(&sh.age_hist[(t5 - res[e]) & 31u], 1u);
                    w++;
                }
            }
        }
    }
    ro.ids = Uid;
    ro.vals = Uval;
    ro.len = int32_t(total);

    // ---- 5b. eviction to V by (age, -hb, id) ------------------------------------------------
    if (evict) {
        uint32_t *hist = reinterpret_cast<uint32_t *>(sh.vals);   // 2048 hb bins, u16 pairs
        for (int32_t i = tid; i < kMaxKeys / 2; i += kPvBlock) hist[i] = 0;
        __syncthreads();
        if (wave == 0) {                                   // boundary age: first cum >= V
            const uint32_t hv = lane < 32 ? sh.age_hist[lane] : 0u;
            uint32_t incl = hv;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t u = __shfl_up(incl, d, 64);
                if (lane >= d) incl += u;
            }
            const unsigned long long hit = __ballot(lane < 32 && incl >= uint32_t(V));
            const int32_t ab = __builtin_ffsll(hit) - 1;
            const uint32_t before = __shfl(incl - hv, ab, 64);
            const uint32_t at = __shfl(hv, ab, 64);
            if (lane == 0) {
                sh.misc[0] = ab;
                sh.misc[1] = V - int32_t(before);          // kept at the boundary age
                sh.misc[2] = int32_t(at);
            }
        }
        __syncthreads();
        const uint32_t astar = uint32_t(sh.misc[0]);
        const int32_t need = sh.misc[1];
        const bool tie = sh.misc[2] > need;
        uint32_t hstar = 0;
        int32_t need2 = 0;
        if (tie) {                                         // boundary hb among age == astar
            for (uint32_t i = base; i < base + nloc; ++i) {
                const uint32_t v = Uval[i];
                if (((t5 - v) & 31u) == astar)
                    atomicAdd(&hist[(v >> 5) >> 1], 1u << (((v >> 5) & 1u) * 16u));
            }
            __syncthreads();
            // lane t owns hb bins 2047 - 8t - 7 .. 2047 - 8t (descending order of lanes)
            const uint16_t *h16 = sh.vals;
            uint32_t loc = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) loc += h16[2047 - 8 * tid - b];
            uint32_t tot = 0;
            const uint32_t ex = block_scan(loc, &tot, sh.wave_scan);
            if (ex < uint32_t(need) && uint32_t(need) <= ex + loc) {
                uint32_t cum = ex;
                for (int b = 0; b < 8; ++b) {
                    const int32_t h = 2047 - 8 * tid - b;
                    const uint32_t c = h16[h];
                    if (cum + c >= uint32_t(need)) {
                        sh.misc[3] = h;
                        sh.misc[4] = need - int32_t(cum);  // kept among (astar, h) ties
                        break;
                    }
                    cum += c;
                }
            }
            __syncthreads();
            hstar = uint32_t(sh.misc[3]);
            need2 = sh.misc[4];
        }
        // one packed scan: ties before this lane (low 16) and plain keeps before it (high 16)
        uint32_t nt = 0, nk = 0;
        for (uint32_t i = base; i < base + nloc; ++i) {
            const uint32_t v = Uval[i], age = (t5 - v) & 31u, hb = v >> 5;
            const bool is_tie = tie && age == astar && hb == hstar;
            nt += is_tie ? 1u : 0u;
            nk += (!is_tie && (age < astar || (age == astar && (!tie || hb > hstar)))) ? 1u : 0u;
        }
        uint32_t sums = 0;
        const uint32_t ex = block_scan(nt | (nk << 16), &sums, sh.wave_scan);
        uint32_t tie_before = ex & 0xFFFFu;
        const uint32_t ties_kept_before = tie_before < uint32_t(need2) ? tie_before : uint32_t(need2);
        uint32_t w = (ex >> 16) + (tie ? ties_kept_before : 0u);
        uint32_t *Wid = sh.keys[cur];                       // C is dead
        uint16_t *Wval = sh.vals;                           // the histogram is dead
        for (uint32_t i = base; i < base + nloc; ++i) {
            const uint32_t v = Uval[i], age = (t5 - v) & 31u, hb = v >> 5;
            bool keep = age < astar || (age == astar && (!tie || hb > hstar));
            if (tie && age == astar && hb == hstar) keep = int32_t(tie_before++) < need2;
            if (keep) {
                Wid[w] = Uid[i];
                Wval[w] = uint16_t(v);
                w++;
            } else {
                evicts++;
                hsum += pv_event_mix(3, t, uint32_t(r), Uid[i]);
            }
        }
        ro.ids = Wid;
        ro.vals = Wval;
        ro.len = V;
    }
    ro.joins = joins;
    ro.removes = removes;
    ro.evicts = evicts;
    ro.hsum = hsum;
    __syncthreads();
}

// ---- 6. write the view, heartbeat, digest, sends ------------------------------------------
__device__ __forceinline__ void pv_finish(const PviewTickArgs &a, PvShared &sh, int32_t lr,
                                          int32_t r, int32_t k, int32_t k_all, bool init,
                                          const RowOut &ro) {
    const int32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t V = a.view, F = a.fanout, len = ro.len;
    const uint32_t t = uint32_t(a.tick);
    uint64_t *out = a.cur + int64_t(lr) * V;
    for (int32_t i = tid; i < V; i += kPvBlock)
        __builtin_nontemporal_store(
            i < len ? (uint64_t(ro.ids[i]) << 32) | uint64_t(ro.vals[i]) : kPvEmpty, out + i);

    unsigned long long *dig = a.dig + (blockIdx.x % kPvDigSlots) * kPvFields;
    if (!init) {
        const uint32_t j = wave_sum32(ro.joins), rm = wave_sum32(ro.removes), ev = wave_sum32(ro.evicts);
        const uint64_t h = wave_sum64(ro.hsum);
        if (lane == 0) { sh.red[wave][0] = j; sh.red[wave][1] = rm; sh.red[wave][2] = ev; sh.red[wave][3] = h; }
        __syncthreads();
    }
    if (wave != 0) return;
    // peers: min(F, len) distinct members by Philox rank-select over the id order
    const int32_t keff = F < len ? F : len;
    if (lane == 0) {
        int32_t nch = 0;
        for (int32_t kk = 0; kk < keff; ++kk) {
            int32_t rk = int32_t(sh.peer_u[kk] % uint32_t(len - kk));
            int32_t pos = 0;
            while (pos < nch && rk >= sh.chosen[pos]) { rk++; pos++; }
            for (int32_t q2 = nch; q2 > pos; --q2) sh.chosen[q2] = sh.chosen[q2 - 1];
            sh.chosen[pos] = rk;
            nch++;
            sh.pick[kk] = int32_t(ro.ids[rk]);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    bool drop = false;
    if (lane < F) {
        int32_t dst = -1;
        if (lane < keff) {
            dst = sh.pick[lane];
            const uint32_t dr = draw_u31(kDomainSend, a.seed, t, uint32_t(r), uint32_t(dst), 3u);
            if (int32_t(dr % 100u) < a.drop_pct) { drop = true; dst = -1; }
        }
        a.out_dst[int64_t(lr) * F + lane] = dst;
        if (dst >= 0) atomicAdd(&a.deg[dst], 1);
    }
    const uint32_t dropped = uint32_t(__popcll(__ballot(drop)));
    if (lane == 0) {
        a.len_cur[lr] = len;
        if (keff) {
            atomicAdd(&dig[kPvSent], (unsigned long long)keff);
            if (dropped) atomicAdd(&dig[kPvDropped], (unsigned long long)dropped);
        }
        if (!init) {
            a.own_hb[lr] += 1;
            const unsigned long long merges = uint64_t(k) + uint64_t(uint32_t(sh.misc[5]));
            atomicAdd(&dig[kPvRounds], 1ull);
            atomicAdd(&dig[kPvMerges], merges);
            atomicAdd(&dig[kPvDelivered], (unsigned long long)k);
            if (k_all > k) atomicAdd(&dig[kPvOverflow], (unsigned long long)(k_all - k));
            const unsigned long long j = sh.red[0][0] + sh.red[1][0] + sh.red[2][0] + sh.red[3][0];
            const unsigned long long rm = sh.red[0][1] + sh.red[1][1] + sh.red[2][1] + sh.red[3][1];
            const unsigned long long ev = sh.red[0][2] + sh.red[1][2] + sh.red[2][2] + sh.red[3][2];
            if (j) atomicAdd(&dig[kPvJoins], j);
            if (rm) atomicAdd(&dig[kPvRemoves], rm);
            if (ev) atomicAdd(&dig[kPvEvicts], ev);
            atomicAdd(&dig[kPvHash], sh.red[0][3] + sh.red[1][3] + sh.red[2][3] + sh.red[3][3]);
        }
    }
}

template <bool kInit>
__global__ void __launch_bounds__(kPvBlock) pview_tick_kernel(PviewTickArgs a) {
    __shared__ PvShared sh;
    const int32_t tid = threadIdx.x;
    const int32_t lr = blockIdx.x;
    const int32_t r = a.row0 + lr;
    const int32_t F = a.fanout, V = a.view;

    if (a.tick > a.fail_tick[r]) {          // crashed: no recv, no ops, no send
        if (tid < F) a.out_dst[int64_t(lr) * F + tid] = -1;
        return;
    }
    if (tid < F)
        sh.peer_u[tid] = draw_u31(kDomainPeer, a.seed, uint32_t(a.tick), uint32_t(r), uint32_t(tid), 0u);
    if (tid < 32) sh.age_hist[tid] = 0;
    if (tid < kPvMaxInbox) sh.found[tid] = 0;
    if (tid == 0) sh.misc[5] = 0;

    RowOut ro{};
    int32_t k = 0, k_all = 0;
    if (kInit) {
        // pre-joined bounded view: {(r + 1 + j * (n / V)) mod n}, or everyone if n - 1 <= V
        const int32_t n = a.n;
        uint32_t *ids = sh.keys[0];
        if (n - 1 <= V) {
            for (int32_t x = tid; x < n; x += kPvBlock)
                if (x != r) ids[x < r ? x : x - 1] = uint32_t(x);
            ro.len = n - 1;
        } else {
            const int64_t stride = n / V;
            const int64_t first_wrap = (int64_t(n) - r - 1 + stride - 1) / stride;
            const int32_t J = int32_t(first_wrap < V ? first_wrap : V);
            for (int32_t j = tid; j < V; j += kPvBlock) {
                int64_t x = int64_t(r) + 1 + int64_t(j) * stride;
                int32_t p;
                if (x >= n) { x -= n; p = j - J; } else { p = j + (V - J); }
                ids[p] = uint32_t(x);
            }
            ro.len = V;
        }
        for (int32_t i = tid; i < ro.len; i += kPvBlock) sh.uval[i] = uint16_t(a.h0 << 5);
        ro.ids = ids;
        ro.vals = sh.uval;
        __syncthreads();
    } else {
        // ---- 1. receipt order --------------------------------------------------------------
        const int32_t o0 = a.off[lr];
        k_all = a.off[lr + 1] - o0;
        if (k_all > 1024) {
            if (tid == 0) atomicOr(a.err, 1);
            if (tid < F) a.out_dst[int64_t(lr) * F + tid] = -1;
            return;
        }
        int32_t *raw = reinterpret_cast<int32_t *>(sh.keys[1]);          // scratch
        int32_t *raw_slot = raw + 1024;
        for (int32_t i = tid; i < k_all; i += kPvBlock) {
            raw[i] = a.csr_src[o0 + i];
            raw_slot[i] = a.csr_slot ? a.csr_slot[o0 + i] : raw[i] - a.row0;
        }
        __syncthreads();
        k = k_all < a.inbox ? k_all : a.inbox;
        for (int32_t i = tid; i < k_all; i += kPvBlock) {
            int32_t rank = 0;
            for (int32_t j = 0; j < k_all; ++j) rank += raw[j] < raw[i];
            if (rank < k) {
                sh.src[rank] = raw[i];
                sh.slot[rank] = raw_slot[i];
            }
        }
        __syncthreads();
        if (k == 0) pv_merge_row<1>(a, sh, lr, r, k, ro);
        else if (k == 1) pv_merge_row<2>(a, sh, lr, r, k, ro);
        else if (k <= 3) pv_merge_row<4>(a, sh, lr, r, k, ro);
        else pv_merge_row<8>(a, sh, lr, r, k, ro);
    }
    (void)V;
    pv_finish(a, sh, lr, r, k, k_all, kInit, ro);
}

}  // namespace

hipError_t launch_pview_init(const PviewTickArgs &a, hipStream_t st) {
    if (a.view < 1 || a.view > kPvMaxView || a.inbox < 1 || a.inbox > kPvMaxInbox ||
        a.fanout < 1 || a.fanout > 16 || a.n >= (1 << 21))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(pview_tick_kernel<true>, dim3(a.rows), dim3(kPvBlock), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_pview_tick(const PviewTickArgs &a, hipStream_t st) {
    if (a.view < 1 || a.view > kPvMaxView || a.inbox < 1 || a.inbox > kPvMaxInbox ||
        a.fanout < 1 || a.fanout > 16 || a.n >= (1 << 21))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(pview_tick_kernel<false>, dim3(a.rows), dim3(kPvBlock), 0, st, a);
    return hipGetLastError();
}

}  // namespace gsp
