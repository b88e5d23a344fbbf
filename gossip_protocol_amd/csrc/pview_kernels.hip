// gossip_protocol_amd/csrc/pview_kernels.hip -- PARTIAL-VIEW tick kernel for gfx950.
//
// One 256-lane workgroup per receiver row, everything in LDS (35 KB):
//   1. its <= K smallest senders (canonical receipt order, rest = inbox overflow);
//   2. its own view and the K sender views (each <= V entries, sorted by id), one entry per
//      lane per list;
//   3. per-id fold of MP1Node::recvCallBack's rules over the message sequence
//      (MP1Node.cpp:234-301): every id is handled by the lane holding its FIRST occurrence
//      (own view, then sender 1, payload 1, sender 2, ...), found with binary searches in the
//      earlier lists; then the TREMOVE scan (MP1Node.cpp:339-348);
//   4. union in id order: rank = sum over sources of owned survivors with a smaller id
//      (per-source prefix counts from one packed block scan);
//   5. eviction to V by (age, -hb, id): an age histogram, an hb histogram for the boundary
//      age, an id-order prefix for the last tie -- no sort;
//   6. the new sorted view is written back; Philox rank-select picks the peers.
// Bytes per node-round: 2 * V * 8 (own view read + write) + k * V * 8 (sender views).
#include "philox.hpp"
#include "pview_kernels.hpp"

namespace gsp {
namespace {

constexpr int kLists = 1 + kPvMaxInbox;                   // own view + K payloads
constexpr int kSrc = kLists + 1;                          // + the sender pseudo-list
constexpr int kCand = kPvMaxView * kLists + kPvMaxInbox;  // survivors bound (2312)
constexpr int32_t kNoId = 0x7FFFFFFF;

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

__device__ inline int32_t lbound(const int32_t *ids, int32_t len, int32_t x) {
    int32_t lo = 0, hi = len;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (ids[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ inline uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// exclusive block scan (256 lanes) of W packed words; *total = inclusive sum of all lanes
template <int W>
__device__ inline void block_scan_words(uint32_t (&v)[W], uint32_t (&total)[W], uint32_t *s_wave) {
    const int32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
        incl[w] = v[w];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t u = __shfl_up(incl[w], d, 64);
            if (lane >= d) incl[w] += u;
        }
    }
    __syncthreads();
    if (lane == 63)
#pragma unroll
        for (int w = 0; w < W; ++w) s_wave[wave * W + w] = incl[w];
    __syncthreads();
#pragma unroll
    for (int w = 0; w < W; ++w) {
        uint32_t before = 0, all = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t x = s_wave[q * W + w];
            before += q < wave ? x : 0u;
            all += x;
        }
        total[w] = all;
        v[w] = incl[w] - v[w] + before;
    }
}

struct PvShared {
    int32_t ids[kLists][kPvMaxView];     // list ids (kNoId past the end); later: histograms
    uint16_t val[kLists][kPvMaxView];    // packed hb/ts of the list entries
    uint8_t flag[kLists][kPvMaxView];    // owned survivor flags
    uint16_t pre[kSrc][kPvMaxView + 1];  // exclusive prefix of flags per source
    int32_t oid[kCand];                  // survivors in id order (scratch: raw senders)
    uint16_t oval[kCand];
    int32_t src[kPvMaxInbox], slot[kPvMaxInbox], len[kLists];
    uint8_t sflag[kPvMaxInbox];
    uint32_t wave_scan[4 * 4];
    int32_t misc[8];
    unsigned long long red[4][6];
};

// Packed flag words for the prefix scan: 10-bit fields, 3 per word, sources 0..kSrc-1.
constexpr int kScanWords = (kSrc + 2) / 3;

template <bool kInit>
__global__ void __launch_bounds__(kPvBlock) pview_tick_kernel(PviewTickArgs a) {
    __shared__ PvShared sh;
    const int32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t lr = blockIdx.x;
    const int32_t r = a.row0 + lr;
    const int32_t t = a.tick, F = a.fanout, V = a.view;
    const uint32_t t5 = uint32_t(t) & 31u, tr = uint32_t(a.tremove);

    if (t > a.fail_tick[r]) {          // crashed: no recv, no ops, no send
        if (tid < F) a.out_dst[int64_t(lr) * F + tid] = -1;
        return;
    }

    int32_t new_len = 0;
    uint64_t joins = 0, removes = 0, evicts = 0, hsum = 0;
    int32_t k = 0, k_all = 0;

    if (kInit) {
        // pre-joined bounded view: {(r + 1 + j * (n / V)) mod n}, or everyone if n - 1 <= V
        const int32_t n = a.n;
        if (n - 1 <= V) {
            for (int32_t x = tid; x < n; x += kPvBlock)
                if (x != r) { const int32_t p = x < r ? x : x - 1; sh.oid[p] = x; sh.oval[p] = uint16_t(a.h0 << 5); }
            new_len = n - 1;
        } else {
            const int64_t stride = n / V;
            const int64_t first_wrap = (int64_t(n) - r - 1 + stride - 1) / stride;   // j that wraps
            const int32_t J = int32_t(first_wrap < V ? first_wrap : V);
            if (tid < V) {
                const int32_t j = tid;
                int64_t x = int64_t(r) + 1 + int64_t(j) * stride;
                int32_t p;
                if (x >= n) { x -= n; p = j - J; } else { p = j + (V - J); }
                sh.oid[p] = int32_t(x);
                sh.oval[p] = uint16_t(a.h0 << 5);
            }
            new_len = V;
        }
        __syncthreads();
    } else {
        // ---- 1. receipt order: the K smallest senders of the segment --------------------
        const int32_t o0 = a.off[lr];
        k_all = a.off[lr + 1] - o0;
        if (k_all > 1024) {
            if (tid == 0) atomicOr(a.err, 1);
            if (tid < F) a.out_dst[int64_t(lr) * F + tid] = -1;
            return;
        }
        int32_t *raw = sh.oid;                       // scratch before the union is built
        int32_t *raw_slot = &sh.ids[0][0];
        for (int32_t i = tid; i < k_all; i += kPvBlock) {
            raw[i] = a.csr_src[o0 + i];
            raw_slot[i] = a.csr_slot ? a.csr_slot[o0 + i] : raw[i] - a.row0;
        }
        __syncthreads();
        k = k_all < a.inbox ? k_all : a.inbox;
        for (int32_t i = tid; i < k_all; i += kPvBlock) {
            int32_t rank = 0;
            for (int32_t j = 0; j < k_all; ++j) rank += raw[j] < raw[i];
            if (rank < k) { sh.src[rank] = raw[i]; sh.slot[rank] = raw_slot[i]; }
        }
        __syncthreads();

        // ---- 2. own view and the k sender views into LDS -------------------------------
        for (int32_t m = 0; m <= k; ++m) {
            const uint64_t *row;
            if (m == 0) row = a.prev + int64_t(lr) * V;
            else {
                const int32_t sl = sh.slot[m - 1];
                row = sl >= 0 ? a.prev + int64_t(sl) * V : a.remote + int64_t(-sl - 1) * V;
            }
            if (tid < kPvMaxView) {
                const uint64_t ent = tid < V ? row[tid] : kPvEmpty;
                sh.ids[m][tid] = ent == kPvEmpty ? kNoId : int32_t(ent >> 32);
                sh.val[m][tid] = ent == kPvEmpty ? 0 : uint16_t(ent & 0xFFFFu);
            }
            if (tid == 0) sh.len[m] = m == 0 ? a.len_prev[r] : a.len_prev[sh.src[m - 1]];
        }
        for (int32_t m = 0; m < kLists; ++m)
            if (tid < kPvMaxView) sh.flag[m][tid] = 0;
        if (tid < kPvMaxInbox) sh.sflag[tid] = 0;
        __syncthreads();

        // ---- 3. per-id fold over the message sequence, by the first occurrence ---------
        // lane `tid` handles entry tid of every list, and sender tid+1 when tid < k
        uint32_t fin[kSrc];
        for (int q = 0; q < kSrc; ++q) fin[q] = 0;
#pragma unroll
        for (int q = 0; q < kSrc; ++q) {
            // q in [0, kLists): list q entry tid;  q == kLists: sender pseudo-entry tid + 1
            const bool is_sender = q == kLists;
            const int32_t j = is_sender ? tid + 1 : q;          // message index (0 = own view)
            if (j > k) continue;
            if (!is_sender && tid >= sh.len[q]) continue;
            const int32_t x = is_sender ? sh.src[tid] : sh.ids[q][tid];
            if (x == r) continue;                                // never list yourself
            bool owned = true;
            int32_t p0 = -1;
            if (j > 0 || is_sender) {
                p0 = lbound(sh.ids[0], sh.len[0], x);
                owned = !(p0 < sh.len[0] && sh.ids[0][p0] == x);
                for (int32_t jj = 1; owned && jj < j; ++jj) {
                    if (sh.src[jj - 1] == x) { owned = false; break; }
                    const int32_t p = lbound(sh.ids[jj], sh.len[jj], x);
                    if (p < sh.len[jj] && sh.ids[jj][p] == x) owned = false;
                }
            }
            if (!owned) continue;
            const uint32_t e0 = (j == 0 && !is_sender) ? sh.val[0][tid] : 0u;
            uint32_t cur = e0;
            for (int32_t jj = 1; jj <= k; ++jj) {
                if (sh.src[jj - 1] == x) {                       // sender entry, MP1Node.cpp:237-243
                    cur = (((cur >> 5) + 1u) << 5) | t5;
                    continue;
                }
                if (jj < j) continue;                            // x is absent from earlier payloads
                const int32_t p = lbound(sh.ids[jj], sh.len[jj], x);
                if (p < sh.len[jj] && sh.ids[jj][p] == x) cur = pv_merge(cur, sh.val[jj][p], t5, tr);
            }
            if (!cur) continue;
            if (!e0) { joins++; hsum += pv_event_mix(1, uint32_t(t), uint32_t(r), uint32_t(x)); }
            if (((t5 - cur) & 31u) >= tr) {                      // TREMOVE scan
                removes++;
                hsum += pv_event_mix(2, uint32_t(t), uint32_t(r), uint32_t(x));
                continue;
            }
            fin[q] = cur;
            if (is_sender) sh.sflag[tid] = 1; else sh.flag[q][tid] = 1;
        }
        __syncthreads();

        // ---- 4. union in id order -------------------------------------------------------
        uint32_t words[kScanWords], totw[kScanWords];
#pragma unroll
        for (int w = 0; w < kScanWords; ++w) words[w] = 0;
#pragma unroll
        for (int q = 0; q < kSrc; ++q) {
            uint32_t f = 0;
            if (q < kLists) f = (tid < kPvMaxView) ? sh.flag[q][tid] : 0u;
            else f = tid < kPvMaxInbox ? sh.sflag[tid] : 0u;
            words[q / 3] |= f << (10 * (q % 3));
        }
        block_scan_words<kScanWords>(words, totw, sh.wave_scan);
        if (tid < kPvMaxView) {
#pragma unroll
            for (int q = 0; q < kSrc; ++q) sh.pre[q][tid] = uint16_t((words[q / 3] >> (10 * (q % 3))) & 1023u);
        }
        if (tid == 0) {
#pragma unroll
            for (int q = 0; q < kSrc; ++q) sh.pre[q][kPvMaxView] = uint16_t((totw[q / 3] >> (10 * (q % 3))) & 1023u);
        }
        int32_t total = 0;
#pragma unroll
        for (int q = 0; q < kSrc; ++q) total += int32_t((totw[q / 3] >> (10 * (q % 3))) & 1023u);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kSrc; ++q) {
            if (!fin[q]) continue;
            const bool is_sender = q == kLists;
            const int32_t x = is_sender ? sh.src[tid] : sh.ids[q][tid];
            int32_t rank = 0;
            for (int32_t m = 0; m <= k; ++m) {
                const int32_t p = lbound(sh.ids[m], sh.len[m], x);
                rank += sh.pre[m][p];
            }
            int32_t ps = 0;
            while (ps < k && sh.src[ps] < x) ps++;
            rank += sh.pre[kLists][ps];
            sh.oid[rank] = x;
            sh.oval[rank] = uint16_t(fin[q]);
        }
        __syncthreads();

        // ---- 5. eviction to V by (age, -hb, id) -----------------------------------------
        new_len = total;
        if (total > V) {
            int32_t *hist = &sh.ids[0][0];                       // lists are no longer needed
            for (int32_t i = tid; i < 2048; i += kPvBlock) hist[i] = 0;
            __syncthreads();
            for (int32_t i = tid; i < total; i += kPvBlock)
                atomicAdd(&hist[(t5 - sh.oval[i]) & 31u], 1);
            __syncthreads();
            if (tid == 0) {
                int32_t cum = 0, ab = 0;
                for (ab = 0; ab < 32; ++ab) {
                    if (cum + hist[ab] >= V) break;
                    cum += hist[ab];
                }
                sh.misc[0] = ab;
                sh.misc[1] = V - cum;                            // kept at the boundary age
                sh.misc[2] = hist[ab];
            }
            __syncthreads();
            const uint32_t astar = uint32_t(sh.misc[0]);
            const int32_t need = sh.misc[1];
            const bool tie = sh.misc[2] > need;
            uint32_t hstar = 0;
            int32_t need2 = 0;
            if (tie) {
                for (int32_t i = tid; i < 2048; i += kPvBlock) hist[i] = 0;
                __syncthreads();
                for (int32_t i = tid; i < total; i += kPvBlock)
                    if (((t5 - sh.oval[i]) & 31u) == astar) atomicAdd(&hist[sh.oval[i] >> 5], 1);
                __syncthreads();
                if (tid == 0) {
                    int32_t cum = 0, h;
                    for (h = 2047; h > 0; --h) {
                        if (cum + hist[h] >= need) break;
                        cum += hist[h];
                    }
                    sh.misc[3] = h;
                    sh.misc[4] = need - cum;                     // kept among (astar, h) ties
                }
                __syncthreads();
                hstar = uint32_t(sh.misc[3]);
                need2 = sh.misc[4];
            }
            // keep flags and compaction in id order, chunk by chunk
            int32_t kept = 0, ties = 0;
            for (int32_t c0 = 0; c0 < total; c0 += kPvBlock) {
                const int32_t i = c0 + tid;
                int32_t x = 0;
                uint32_t v = 0, keep = 0, istie = 0;
                if (i < total) {
                    x = sh.oid[i];
                    v = sh.oval[i];
                    const uint32_t age = (t5 - v) & 31u, hb = v >> 5;
                    istie = tie && age == astar && hb == hstar;
                    keep = age < astar || (age == astar && (!tie || hb > hstar));
                }
                uint32_t w2[2] = {istie, 0u}, tot2[2];
                block_scan_words<2>(w2, tot2, sh.wave_scan);
                if (istie && int32_t(w2[0]) + ties < need2) keep = 1;
                ties += int32_t(tot2[0]);
                if (i < total && !keep) {
                    evicts++;
                    hsum += pv_event_mix(3, uint32_t(t), uint32_t(r), uint32_t(x));
                }
                uint32_t w3[2] = {keep, 0u}, tot3[2];
                block_scan_words<2>(w3, tot3, sh.wave_scan);   // its barriers fence the reads
                if (keep) { sh.oid[kept + int32_t(w3[0])] = x; sh.oval[kept + int32_t(w3[0])] = uint16_t(v); }
                kept += int32_t(tot3[0]);
                __syncthreads();
            }
            new_len = kept;
        }
    }

    // ---- 6. write the new view; heartbeat; send ------------------------------------------
    uint64_t *out = a.cur + int64_t(lr) * V;
    for (int32_t i = tid; i < V; i += kPvBlock)
        out[i] = i < new_len ? ((uint64_t(uint32_t(sh.oid[i])) << 32) | sh.oval[i]) : kPvEmpty;

    const uint64_t r0 = wave_sum(joins), r1 = wave_sum(removes), r2 = wave_sum(evicts), r3 = wave_sum(hsum);
    if (lane == 0) { sh.red[wave][0] = r0; sh.red[wave][1] = r1; sh.red[wave][2] = r2; sh.red[wave][3] = r3; }
    __syncthreads();
    unsigned long long *dig = a.dig + (blockIdx.x % kPvDigSlots) * kPvFields;
    if (tid == 0) {
        a.len_cur[r] = new_len;
        if (!kInit) {
            a.own_hb[lr] += 1;
            unsigned long long merges = 0;
            for (int32_t j = 0; j < k; ++j) merges += 1ull + uint64_t(a.len_prev[sh.src[j]]);
            atomicAdd(&dig[kPvRounds], 1ull);
            atomicAdd(&dig[kPvMerges], merges);
            atomicAdd(&dig[kPvDelivered], (unsigned long long)k);
            if (k_all > k) atomicAdd(&dig[kPvOverflow], (unsigned long long)(k_all - k));
            atomicAdd(&dig[kPvJoins], sh.red[0][0] + sh.red[1][0] + sh.red[2][0] + sh.red[3][0]);
            atomicAdd(&dig[kPvRemoves], sh.red[0][1] + sh.red[1][1] + sh.red[2][1] + sh.red[3][1]);
            atomicAdd(&dig[kPvEvicts], sh.red[0][2] + sh.red[1][2] + sh.red[2][2] + sh.red[3][2]);
            atomicAdd(&dig[kPvHash], sh.red[0][3] + sh.red[1][3] + sh.red[2][3] + sh.red[3][3]);
        }
        // peers: min(F, len) distinct members by Philox rank-select over the id order
        const int32_t keff = F < new_len ? F : new_len;
        int32_t chosen[16];
        int32_t nch = 0;
        unsigned long long sent = 0, dropped = 0;
        for (int32_t kk = 0; kk < F; ++kk) {
            int32_t dst = -1;
            if (kk < keff) {
                const uint32_t u = draw_u31(kDomainPeer, a.seed, uint32_t(t), uint32_t(r),
                                            uint32_t(kk), 0u);
                int32_t rk = int32_t(u % uint32_t(new_len - kk));
                int32_t pos = 0;
                while (pos < nch && rk >= chosen[pos]) { rk++; pos++; }
                for (int32_t q = nch; q > pos; --q) chosen[q] = chosen[q - 1];
                chosen[pos] = rk;
                nch++;
                dst = sh.oid[rk];
                sent++;
                const uint32_t dr = draw_u31(kDomainSend, a.seed, uint32_t(t), uint32_t(r),
                                             uint32_t(dst), 3u);
                if (int32_t(dr % 100u) < a.drop_pct) { dropped++; dst = -1; }
            }
            a.out_dst[int64_t(lr) * F + kk] = dst;
            if (dst >= 0) atomicAdd(&a.deg[dst], 1);
        }
        if (sent) {
            atomicAdd(&dig[kPvSent], sent);
            atomicAdd(&dig[kPvDropped], dropped);
        }
    }
}

}  // namespace

hipError_t launch_pview_init(const PviewTickArgs &a, hipStream_t st) {
    if (a.view < 1 || a.view > kPvMaxView || a.inbox < 1 || a.inbox > kPvMaxInbox ||
        a.fanout < 1 || a.fanout > 16)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(pview_tick_kernel<true>, dim3(a.rows), dim3(kPvBlock), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_pview_tick(const PviewTickArgs &a, hipStream_t st) {
    if (a.view < 1 || a.view > kPvMaxView || a.inbox < 1 || a.inbox > kPvMaxInbox ||
        a.fanout < 1 || a.fanout > 16)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(pview_tick_kernel<false>, dim3(a.rows), dim3(kPvBlock), 0, st, a);
    return hipGetLastError();
}

}  // namespace gsp
