// gossip_protocol_amd/csrc/scale_kernels.hip -- SCALE-mode HIP kernels for gfx950.
//
// scale_tick_kernel<false> is the whole per-tick hot path of one receiver row, fused:
//   merge   (MP1Node::recvCallBack GOSSIP branch, MP1Node.cpp:234-256) of every message the
//           row received, in ascending sender order, 8 packed entries per lane per 16-B load;
//   ops     (MP1Node::nodeLoopOps, MP1Node.cpp:335-348): own heartbeat bump, TREMOVE scan;
//   events  join/remove detection, counted and hashed (order-independent digest);
//   send    peer choice by Philox rank-select over the row's presence bitmap in LDS, the
//           drop draw, and the destination count for next tick's CSR.
// One 256-lane workgroup per row streams the row in 2048-column chunks: it reads its own
// row and each sender's row once (16 B per lane, fully coalesced) and writes its row once,
// so the kernel is HBM-bound at (2 + k) * stride * 2 bytes per row with k messages.
#include "philox.hpp"
#include "scale_kernels.hpp"

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

__device__ inline uint32_t merge_word(uint32_t e, uint32_t v, uint32_t t5, uint32_t tr) {
    const uint32_t lo = merge_entry(e & 0xFFFFu, v & 0xFFFFu, t5, tr);
    const uint32_t hi = merge_entry(e >> 16, v >> 16, t5, tr);
    return lo | (hi << 16);
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

// 16-byte row accesses; kNT selects the non-temporal (streaming) cache policy
template <bool kNT>
__device__ inline uint4 ld16(const uint16_t *p) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
    const u32x4 v = kNT ? __builtin_nontemporal_load(q) : *q;
    return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool kNT>
__device__ inline void st16(uint16_t *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    u32x4 v;
    v.x = a; v.y = b; v.z = c; v.w = d;
    u32x4 *q = reinterpret_cast<u32x4 *>(p);
    if (kNT) __builtin_nontemporal_store(v, q);
    else *q = v;
}

__device__ inline uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// kPolicy bit 0: non-temporal own-row loads/stores; bit 1: non-temporal sender-row loads
template <bool kInit, int kPolicy>
__global__ void __launch_bounds__(kScaleBlock) scale_tick_kernel(ScaleTickArgs a) {
    constexpr bool kNtOwn = (kPolicy & 1) != 0, kNtSrc = (kPolicy & 2) != 0;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_bits[];   // stride / 32 words
    __shared__ int32_t s_src[kMaxSegment];
    __shared__ int32_t s_raw[kMaxSegment];
    __shared__ unsigned long long s_red[4][4];

    const int32_t tid = threadIdx.x;
    const int32_t lane = tid & 63, wave = tid >> 6;
    const int32_t lr = blockIdx.x;
    const int32_t r = a.row0 + lr;
    const int32_t t = a.tick;
    const int32_t F = a.fanout;

    if (t > a.fail_tick[r]) {          // crashed (Application.cpp:186): no recv, no ops, no send
        if (tid < F) a.out_dst[int64_t(lr) * F + tid] = -1;
        return;
    }

    int32_t k = 0;
    if (!kInit) {
        const int32_t o0 = a.off[lr];
        k = a.off[lr + 1] - o0;
        if (k > kMaxSegment) {
            if (tid == 0) atomicOr(a.err, 1);
            if (tid < F) a.out_dst[int64_t(lr) * F + tid] = -1;
            return;
        }
        for (int32_t i = tid; i < k; i += kScaleBlock) s_raw[i] = a.csr_src[o0 + i];
        __syncthreads();
        // canonical receipt order: ascending sender (senders are distinct per receiver)
        for (int32_t i = tid; i < k; i += kScaleBlock) {
            const int32_t v = s_raw[i];
            int32_t rank = 0;
            for (int32_t j = 0; j < k; ++j) rank += s_raw[j] < v;
            s_src[rank] = v;
        }
        __syncthreads();
    }

    const uint32_t t5 = uint32_t(t) & 31u;
    const uint32_t tr = uint32_t(a.tremove);
    const int64_t stride = a.stride;
    const uint16_t *own_prev = a.prev + int64_t(lr) * stride;
    uint16_t *own_cur = a.cur + int64_t(lr) * stride;
    uint32_t live = 0, joins = 0, removes = 0;
    uint64_t hsum = 0;

    for (int64_t c0 = 0; c0 < stride; c0 += kChunk) {
        const int64_t col0 = c0 + int64_t(tid) * kEntriesPerLane;
        uint4 e;
        uint4 e0 = make_uint4(0, 0, 0, 0);
        if (kInit) {
            const uint32_t h = uint32_t(a.h0) << 5;
            uint32_t ws[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t x0 = col0 + 2 * i, x1 = x0 + 1;
                const uint32_t lo = (x0 < a.n && x0 != r) ? h : 0u;
                const uint32_t hi = (x1 < a.n && x1 != r) ? h : 0u;
                ws[i] = lo | (hi << 16);
            }
            e = make_uint4(ws[0], ws[1], ws[2], ws[3]);
        } else {
            e = ld16<kNtOwn>(own_prev + col0);
            e0 = e;
            for (int32_t j0 = 0; j0 < k; j0 += 4) {
                uint4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (j0 + u < k)
                        v[u] = ld16<kNtSrc>(a.prev + int64_t(s_src[j0 + u] - a.row0) * stride + col0);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (j0 + u >= k) break;
                    e.x = merge_word(e.x, v[u].x, t5, tr);
                    e.y = merge_word(e.y, v[u].y, t5, tr);
                    e.z = merge_word(e.z, v[u].z, t5, tr);
                    e.w = merge_word(e.w, v[u].w, t5, tr);
                    // the sender's own entry: hb + 1 and ts = now, or add (1, now)
                    // (MP1Node.cpp:237-243); the sender's row never holds itself
                    const int64_t ds = int64_t(s_src[j0 + u]) - col0;
                    if (ds >= 0 && ds < kEntriesPerLane)
                        patch16(e, int(ds), [t5](uint32_t old) { return (((old >> 5) + 1u) << 5) | t5; });
                }
            }
            const int64_t dr = int64_t(r) - col0;      // never list yourself (MP1Node.cpp:290)
            if (dr >= 0 && dr < kEntriesPerLane) patch16(e, int(dr), [](uint32_t) { return 0u; });
        }

        uint32_t bits = 0;
        uint32_t ws[4] = {e.x, e.y, e.z, e.w};
        const uint32_t w0[4] = {e0.x, e0.y, e0.z, e0.w};
#pragma unroll
        for (int i = 0; i < kEntriesPerLane; ++i) {
            const int sh = (i & 1) * 16;
            uint32_t ent = (ws[i >> 1] >> sh) & 0xFFFFu;
            if (!kInit && ent) {
                const uint32_t before = (w0[i >> 1] >> sh) & 0xFFFFu;
                if (((t5 - ent) & 31u) >= tr) {     // TREMOVE scan (MP1Node.cpp:340)
                    removes++;
                    hsum += event_mix(2, uint32_t(t), uint32_t(r), uint32_t(col0 + i));
                    ws[i >> 1] &= ~(0xFFFFu << sh);
                    ent = 0;
                } else if (!before) {
                    joins++;
                    hsum += event_mix(1, uint32_t(t), uint32_t(r), uint32_t(col0 + i));
                }
            }
            bits |= (ent ? 1u : 0u) << i;
        }
        live += __builtin_popcount(bits);
        st16<kNtOwn>(own_cur + col0, ws[0], ws[1], ws[2], ws[3]);
        // presence bitmap: 8 bits per lane -> byte (col0 / 8)
        reinterpret_cast<uint8_t *>(s_bits)[col0 >> 3] = uint8_t(bits);
    }

    // block reduction: live, joins, removes, hash
    uint64_t v0 = wave_sum_u64(live), v1 = wave_sum_u64(joins), v2 = wave_sum_u64(removes);
    uint64_t v3 = wave_sum_u64(hsum);
    if (lane == 0) { s_red[wave][0] = v0; s_red[wave][1] = v1; s_red[wave][2] = v2; s_red[wave][3] = v3; }
    __syncthreads();
    const uint64_t tot_live = s_red[0][0] + s_red[1][0] + s_red[2][0] + s_red[3][0];

    unsigned long long *dig = a.dig + (blockIdx.x % kDigSlots) * kDigFields;
    if (tid == 0) {
        a.cnt_cur[r] = int32_t(tot_live);
        if (!kInit) {
            a.own_hb[lr] += 1;
            unsigned long long merges = 0;
            for (int32_t j = 0; j < k; ++j) merges += 1ull + uint64_t(a.cnt_prev[s_src[j]]);
            atomicAdd(&dig[kDigRounds], 1ull);
            atomicAdd(&dig[kDigMerges], merges);
            atomicAdd(&dig[kDigDelivered], (unsigned long long)k);
            atomicAdd(&dig[kDigJoins], s_red[0][1] + s_red[1][1] + s_red[2][1] + s_red[3][1]);
            atomicAdd(&dig[kDigRemoves], s_red[0][2] + s_red[1][2] + s_red[2][2] + s_red[3][2]);
            atomicAdd(&dig[kDigHash], s_red[0][3] + s_red[1][3] + s_red[2][3] + s_red[3][3]);
        }
    }

    // send: wave 0 picks min(F, live) distinct members by Philox rank-select
    if (wave == 0) {
        const int32_t words = int32_t(stride >> 5);     // bitmap words
        const int32_t per = words >> 6;                 // words per lane (stride % 2048 == 0)
        uint32_t lane_cnt = 0;
        for (int32_t w = 0; w < per; ++w) lane_cnt += __builtin_popcount(s_bits[lane * per + w]);
        uint32_t incl = lane_cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t u = __shfl_up(incl, d, 64);
            if (lane >= d) incl += u;
        }
        const uint32_t pre = incl - lane_cnt;
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
                int32_t rk = int32_t(u % uint32_t(cnt - kk));
                int32_t pos = 0;
                while (pos < nch && rk >= chosen[pos]) { rk++; pos++; }
                for (int32_t q = nch; q > pos; --q) chosen[q] = chosen[q - 1];
                chosen[pos] = rk;
                nch++;
                const bool mine = uint32_t(rk) >= pre && uint32_t(rk) < pre + lane_cnt;
                int32_t col = -1;
                if (mine) {
                    uint32_t m = uint32_t(rk) - pre;
                    for (int32_t w = 0; w < per; ++w) {
                        uint32_t bw = s_bits[lane * per + w];
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
                const int32_t src_lane = __builtin_ffsll(owner) - 1;
                dst = __shfl(col, src_lane, 64);
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
    }
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

}  // namespace

size_t scale_lds_bytes(int64_t stride) { return size_t(stride / 8); }

hipError_t launch_scale_init(const ScaleTickArgs &a, hipStream_t st) {
    if (a.stride % kChunk || a.fanout < 1 || a.fanout > 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL((scale_tick_kernel<true, 0>), dim3(a.rows), dim3(kScaleBlock),
                       scale_lds_bytes(a.stride), st, a);
    return hipGetLastError();
}

hipError_t launch_scale_tick(const ScaleTickArgs &a, int policy, hipStream_t st) {
    if (a.stride % kChunk || a.fanout < 1 || a.fanout > 16) return hipErrorInvalidValue;
    const size_t lds = scale_lds_bytes(a.stride);
    switch (policy & 3) {
        case 0: hipLaunchKernelGGL((scale_tick_kernel<false, 0>), dim3(a.rows), dim3(kScaleBlock), lds, st, a); break;
        case 1: hipLaunchKernelGGL((scale_tick_kernel<false, 1>), dim3(a.rows), dim3(kScaleBlock), lds, st, a); break;
        case 2: hipLaunchKernelGGL((scale_tick_kernel<false, 2>), dim3(a.rows), dim3(kScaleBlock), lds, st, a); break;
        default: hipLaunchKernelGGL((scale_tick_kernel<false, 3>), dim3(a.rows), dim3(kScaleBlock), lds, st, a); break;
    }
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

hipError_t launch_scatter(const int32_t *out_dst, int64_t slots, int32_t fanout, int32_t row0,
                          const int32_t *off, int32_t *fill, int32_t *csr_src, hipStream_t st) {
    int64_t blocks = (slots + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(scatter_kernel, dim3(unsigned(blocks)), dim3(256), 0, st, out_dst, slots,
                       fanout, row0, off, fill, csr_src);
    return hipGetLastError();
}

}  // namespace gsp
