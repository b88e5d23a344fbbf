// gossip_protocol_amd/csrc/rowx_kernels.hip -- row-sharded gossip exchange kernels (gfx950).
// See rowx_kernels.hpp for the protocol and the HBM layout.  All of it is integer index
// work: the only bandwidth that matters is the row gather (2 KB per pair at V = 256), which
// is a plain coalesced copy.
#include "rowx_kernels.hpp"

#include <algorithm>

namespace gsp {
namespace {

constexpr int kMaxFanout = 16;

__device__ inline uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
    const int32_t lane = threadIdx.x & 63;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(incl, d, 64);
        if (lane >= d) incl += u;
    }
    *total = __shfl(incl, 63, 64);
    return incl - v;
}

// One lane per local sender; slots in pair / record regions are claimed with one atomic per
// (wave, destination shard), not one per message.
__global__ void __launch_bounds__(256) rowx_pack_kernel(RowxArgs a) {
    const int32_t lr = int32_t(blockIdx.x) * 256 + int32_t(threadIdx.x);
    const bool live = lr < a.rows;
    const int32_t F = a.fanout;
    int32_t h_of[kMaxFanout], d_of[kMaxFanout];
#pragma unroll
    for (int k = 0; k < kMaxFanout; ++k) {
        h_of[k] = -1;
        d_of[k] = -1;
        if (!live || k >= F) continue;
        const int32_t d = a.out_dst[int64_t(lr) * F + k];
        if (d < 0) continue;
        const int32_t h = rowx_owner(d, a.n, a.shards);
        if (h == a.shard) continue;                   // delivered by the local scatter
        h_of[k] = h;
        d_of[k] = d;
    }
    const int32_t lane = threadIdx.x & 63;
    for (int32_t h = 0; h < a.shards; ++h) {          // wave-uniform loop
        uint32_t nm = 0;
#pragma unroll
        for (int k = 0; k < kMaxFanout; ++k) nm += h_of[k] == h ? 1u : 0u;
        const unsigned long long pm = __ballot(nm > 0);
        if (!pm) continue;
        uint32_t mtot = 0;
        const uint32_t mpre = wave_excl_scan(nm, &mtot);
        int32_t pbase = 0, mbase = 0;
        if (lane == 0) {
            pbase = atomicAdd(&a.pair_cnt[h], int32_t(__popcll(pm)));
            mbase = atomicAdd(&a.msg_cnt[h], int32_t(mtot));
        }
        pbase = __shfl(pbase, 0, 64);
        mbase = __shfl(mbase, 0, 64);
        if (!nm) continue;
        // counts keep growing past the capacity (the host sees them and fails the tick);
        // nothing is written out of bounds
        const int32_t p = pbase + int32_t(__popcll(pm & ((1ull << lane) - 1ull)));
        const int64_t reg = rowx_region(h, a.shard);
        if (p < a.pair_cap) a.pair_row[reg * a.pair_cap + p] = lr;
        int32_t m = mbase + int32_t(mpre);
        const int32_t hrow0 = rowx_row0(h, a.n, a.shards);
#pragma unroll
        for (int k = 0; k < kMaxFanout; ++k)
            if (h_of[k] == h) {
                if (m < a.msg_cap && p < a.pair_cap)
                    a.send_rec[reg * a.msg_cap + m] = RowxRec{a.row0 + lr, d_of[k] - hrow0, p};
                m++;
            }
    }
}

// Pack one partial-view row (V u64 entries, ascending ids, empty slots last) into its wire
// slot (rowx_kernels.hpp): one wave; hs = 256 bytes of this wave's LDS.
__device__ inline void rowx_pack_row(const uint64_t *src, uint16_t *dst, int32_t V, uint8_t *hs) {
    const int32_t lane = threadIdx.x & 63;
    for (int32_t i = lane; i < V; i += 64) {
        const uint64_t e = __builtin_nontemporal_load(src + i);
        const bool empty = e == ~0ull;
        const uint32_t id = uint32_t(e >> 32);
        dst[i] = empty ? uint16_t(0) : uint16_t(id & 0xFFFFu);
        dst[V + i] = empty ? uint16_t(0) : uint16_t(e & 0xFFFFu);
        hs[i] = empty ? uint8_t(32) : uint8_t(id >> 16);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane <= 32) {                 // bound[h] = entries with id >> 16 below h (hs ascends)
        int32_t lo = 0, hi = V;
        while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if (int32_t(hs[mid]) < lane) lo = mid + 1; else hi = mid;
        }
        dst[2 * V + lane] = uint16_t(lo);
    }
    __builtin_amdgcn_wave_barrier();  // hs is reused by the wave's next row
}

// Decode one packed row into V u64 entries: one wave; bs = 33 u16 of this wave's LDS.
__device__ inline void rowx_unpack_row(const uint16_t *src, uint64_t *dst, int32_t V, uint16_t *bs) {
    const int32_t lane = threadIdx.x & 63;
    if (lane <= 32) bs[lane] = src[2 * V + lane];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int32_t ne = bs[32];
    for (int32_t i = lane; i < V; i += 64) {
        uint64_t e = ~0ull;
        if (i < ne) {
            int32_t lo = 1, hi = 33;  // first h >= 1 with bound[h] > i; the id's high bits are h - 1
            while (lo < hi) {
                const int32_t mid = (lo + hi) >> 1;
                if (int32_t(bs[mid]) <= i) lo = mid + 1; else hi = mid;
            }
            const uint32_t id = (uint32_t(lo - 1) << 16) | uint32_t(src[i]);
            e = (uint64_t(id) << 32) | uint64_t(src[V + i]);
        }
        dst[i] = e;
    }
    __builtin_amdgcn_wave_barrier();
}

// one wave per pair: copy the sender's row into the destination shard's send region
// (packed: encode it)
__global__ void __launch_bounds__(256) rowx_gather_packed_kernel(RowxArgs a) {
    __shared__ uint8_t hs[4][256];
    const int64_t w0 = (int64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const int64_t nw = (int64_t(gridDim.x) * 256) >> 6;
    const int32_t V = a.row_words, PW = rowx_packed_words(V);
    for (int32_t h = 0; h < a.shards; ++h) {
        if (h == a.shard) continue;
        const int64_t reg = rowx_region(h, a.shard);
        const int64_t cnt = a.pair_cnt[h] < a.pair_cap ? a.pair_cnt[h] : a.pair_cap;
        for (int64_t p = w0; p < cnt; p += nw) {
            const int32_t lr = a.pair_row[reg * a.pair_cap + p];
            rowx_pack_row(a.table + int64_t(lr) * V,
                          reinterpret_cast<uint16_t *>(a.send_rows + (reg * a.pair_cap + p) * PW), V,
                          hs[threadIdx.x >> 6]);
        }
    }
}

__global__ void __launch_bounds__(64) rowx_check_kernel(const int32_t *cnt_all, const int32_t *bounds,
                                                        int32_t G, int32_t self, int64_t pair_cap,
                                                        int64_t msg_cap, int32_t tick, int32_t *err,
                                                        int32_t *recv_pairs, int32_t *recv_msgs) {
    const int32_t S = 2 * G + 1;
    for (int32_t h = threadIdx.x; h < G; h += blockDim.x) {
        int32_t bad = cnt_all[int64_t(h) * S + 2 * G];        // shard h's receipt flag (a tick)
        for (int32_t g = 0; g < G && !bad; ++g) {             // every count sent to shard h
            if (g == h) continue;
            const int64_t pc = cnt_all[int64_t(g) * S + h], mc = cnt_all[int64_t(g) * S + G + h];
            const int64_t bp = bounds ? bounds[int64_t(g) * G + h] : pair_cap;
            const int64_t bm = bounds ? bounds[int64_t(G) * G + int64_t(g) * G + h] : msg_cap;
            if (pc > pair_cap || mc > msg_cap || pc > bp || mc > bm) bad = tick | kRowxErrBit;
        }
        if (bad) atomicCAS(err, 0, bad);
        // what this shard receives from h, clamped to what arrives
        int64_t rp = 0, rm = 0;
        if (h != self) {
            rp = cnt_all[int64_t(h) * S + self];
            rm = cnt_all[int64_t(h) * S + G + self];
            const int64_t bp = bounds ? bounds[int64_t(h) * G + self] : pair_cap;
            const int64_t bm = bounds ? bounds[int64_t(G) * G + int64_t(h) * G + self] : msg_cap;
            rp = rp < bp ? rp : bp;
            rp = rp < pair_cap ? rp : pair_cap;
            rm = rm < bm ? rm : bm;
            rm = rm < msg_cap ? rm : msg_cap;
        }
        recv_pairs[h] = int32_t(rp);
        recv_msgs[h] = int32_t(rm);
    }
}

// one wave per received pair: decode (packed) or copy (raw) into recv_rows
__global__ void __launch_bounds__(256) rowx_unpack_kernel(const uint64_t *wire, uint64_t *rows,
                                                          const int32_t *recv_pairs, int32_t G,
                                                          int32_t self, int64_t pair_cap, int32_t W,
                                                          int32_t packed) {
    __shared__ uint16_t bs[4][40];
    const int32_t lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const int64_t nw = (int64_t(gridDim.x) * 256) >> 6;
    const int32_t PW = packed ? rowx_packed_words(W) : W;
    for (int32_t h = 0; h < G; ++h) {
        if (h == self) continue;
        const int64_t reg = rowx_region(h, self);
        const int64_t cnt = recv_pairs[h];
        for (int64_t p = w0; p < cnt; p += nw) {
            const uint64_t *src = wire + (reg * pair_cap + p) * PW;
            uint64_t *dst = rows + (reg * pair_cap + p) * W;
            if (packed) rowx_unpack_row(reinterpret_cast<const uint16_t *>(src), dst, W, bs[threadIdx.x >> 6]);
            else for (int32_t i = lane; i < W; i += 64) dst[i] = src[i];
        }
    }
}

// in-process groups: shard g's send region for h -> shard h's receive region for g
__global__ void __launch_bounds__(256) rowx_local_copy_kernel(const uint64_t *send_rows, const RowxRec *send_rec,
                                                              uint64_t *recv_rows, RowxRec *recv_rec,
                                                              const int32_t *cnt_all, int32_t G, int32_t g,
                                                              int32_t h, int64_t pair_cap, int64_t msg_cap,
                                                              int32_t W, int32_t packed) {
    __shared__ uint16_t bs[4][40];
    const int32_t lane = threadIdx.x & 63, S = 2 * G + 1;
    const int64_t np = cnt_all[int64_t(g) * S + h] < pair_cap ? cnt_all[int64_t(g) * S + h] : pair_cap;
    const int64_t nm = cnt_all[int64_t(g) * S + G + h] < msg_cap ? cnt_all[int64_t(g) * S + G + h] : msg_cap;
    const int64_t so = rowx_region(h, g), ro = rowx_region(g, h);
    const int32_t PW = packed ? rowx_packed_words(W) : W;
    const int64_t w0 = (int64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const int64_t nw = (int64_t(gridDim.x) * 256) >> 6;
    for (int64_t p = w0; p < np; p += nw) {
        const uint64_t *src = send_rows + (so * pair_cap + p) * PW;
        uint64_t *dst = recv_rows + (ro * pair_cap + p) * W;
        if (packed) rowx_unpack_row(reinterpret_cast<const uint16_t *>(src), dst, W, bs[threadIdx.x >> 6]);
        else for (int32_t i = lane; i < W; i += 64) dst[i] = src[i];
    }
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < nm; i += int64_t(gridDim.x) * 256)
        recv_rec[ro * msg_cap + i] = send_rec[so * msg_cap + i];
}

// one wave per pair: copy the sender's row into the destination shard's send region
__global__ void __launch_bounds__(256) rowx_gather_kernel(RowxArgs a) {
    const int32_t lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const int64_t nw = (int64_t(gridDim.x) * 256) >> 6;
    const int32_t W = a.row_words;
    for (int32_t h = 0; h < a.shards; ++h) {
        if (h == a.shard) continue;
        const int64_t reg = rowx_region(h, a.shard);
        const int64_t cnt = a.pair_cnt[h] < a.pair_cap ? a.pair_cnt[h] : a.pair_cap;
        for (int64_t p = w0; p < cnt; p += nw) {
            const int32_t lr = a.pair_row[reg * a.pair_cap + p];
            const uint64_t *src = a.table + int64_t(lr) * W;
            uint64_t *dst = a.send_rows + (reg * a.pair_cap + p) * W;
            for (int32_t i = lane; i < W; i += 64) dst[i] = __builtin_nontemporal_load(src + i);
        }
    }
}

__global__ void __launch_bounds__(256) rowx_recv_deg_kernel(const RowxRec *rec, const int32_t *cnt,
                                                            int32_t shards, int32_t self,
                                                            int64_t msg_cap, int32_t row0,
                                                            int32_t *deg) {
    const int64_t i0 = int64_t(blockIdx.x) * 256 + threadIdx.x;
    const int64_t step = int64_t(gridDim.x) * 256;
    for (int32_t h = 0; h < shards; ++h) {
        if (h == self) continue;
        const int64_t m = cnt[h];
        const RowxRec *rh = rec + rowx_region(h, self) * msg_cap;
        for (int64_t i = i0; i < m; i += step) atomicAdd(&deg[row0 + rh[i].dst], 1);
    }
}

__global__ void __launch_bounds__(256) rowx_scatter_local_kernel(const int32_t *out_dst, int32_t rows,
                                                                 int32_t fanout, int32_t row0,
                                                                 const int32_t *off, int32_t *fill,
                                                                 int32_t *csr_src, int32_t *csr_slot) {
    const int64_t slots = int64_t(rows) * fanout;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < slots;
         i += int64_t(gridDim.x) * 256) {
        const int32_t d = out_dst[i] - row0;
        if (d < 0 || d >= rows) continue;             // none, or another shard's receiver
        const int32_t pos = off[d] + atomicAdd(&fill[d], 1);
        const int32_t lr = int32_t(i / fanout);
        csr_src[pos] = row0 + lr;
        csr_slot[pos] = lr;
    }
}

__global__ void __launch_bounds__(256) rowx_scatter_remote_kernel(const RowxRec *rec, const int32_t *cnt,
                                                                  int32_t shards, int32_t self,
                                                                  int64_t msg_cap, int64_t pair_cap,
                                                                  const int32_t *off, int32_t *fill,
                                                                  int32_t *csr_src, int32_t *csr_slot) {
    const int64_t i0 = int64_t(blockIdx.x) * 256 + threadIdx.x;
    const int64_t step = int64_t(gridDim.x) * 256;
    for (int32_t h = 0; h < shards; ++h) {
        if (h == self) continue;
        const int64_t m = cnt[h];
        const int64_t reg = rowx_region(h, self);
        for (int64_t i = i0; i < m; i += step) {
            const RowxRec r = rec[reg * msg_cap + i];
            const int32_t pos = off[r.dst] + atomicAdd(&fill[r.dst], 1);
            csr_src[pos] = r.src;
            csr_slot[pos] = -int32_t(reg * pair_cap + r.pair) - 1;
        }
    }
}

unsigned blocks_for(int64_t items, int64_t cap) {
    int64_t b = (items + 255) / 256;
    return unsigned(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

hipError_t launch_rowx_pack(const RowxArgs &a, hipStream_t st) {
    if (a.fanout < 1 || a.fanout > kMaxFanout || a.shards < 1 || a.rows < 0) return hipErrorInvalidValue;
    if (a.rows == 0) return hipSuccess;
    hipLaunchKernelGGL(rowx_pack_kernel, dim3(unsigned((a.rows + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_rowx_gather(const RowxArgs &a, hipStream_t st) {
    // up to 8 waves per CU-slot worth of pairs; every wave loops over its share
    const int64_t waves = int64_t(a.rows) * (a.shards - 1);
    if (a.packed) {
        if (a.row_words < 1 || a.row_words > 256) return hipErrorInvalidValue;
        hipLaunchKernelGGL(rowx_gather_packed_kernel, dim3(blocks_for(waves * 64, 8192)), dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL(rowx_gather_kernel, dim3(blocks_for(waves * 64, 8192)), dim3(256), 0, st, a);
    }
    return hipGetLastError();
}

hipError_t launch_rowx_check(const int32_t *cnt_all, const int32_t *bounds, int32_t shards, int32_t self,
                             int64_t pair_cap, int64_t msg_cap, int32_t tick, int32_t *err,
                             int32_t *recv_pairs, int32_t *recv_msgs, hipStream_t st) {
    hipLaunchKernelGGL(rowx_check_kernel, dim3(1), dim3(64), 0, st, cnt_all, bounds, shards, self, pair_cap,
                       msg_cap, tick, err, recv_pairs, recv_msgs);
    return hipGetLastError();
}

hipError_t launch_rowx_unpack(const uint64_t *recv_wire, uint64_t *recv_rows, const int32_t *recv_pairs,
                              int32_t shards, int32_t self, int64_t pair_cap, int32_t row_words,
                              int32_t packed, hipStream_t st) {
    if (packed && (row_words < 1 || row_words > 256)) return hipErrorInvalidValue;
    const int64_t waves = pair_cap * (shards - 1);
    hipLaunchKernelGGL(rowx_unpack_kernel, dim3(blocks_for(waves * 64, 8192)), dim3(256), 0, st, recv_wire,
                       recv_rows, recv_pairs, shards, self, pair_cap, row_words, packed);
    return hipGetLastError();
}

hipError_t launch_rowx_local_copy(const uint64_t *send_rows, const RowxRec *send_rec, uint64_t *recv_rows,
                                  RowxRec *recv_rec, const int32_t *cnt_all, int32_t shards, int32_t g,
                                  int32_t h, int64_t pair_cap, int64_t msg_cap, int32_t row_words,
                                  int32_t packed, hipStream_t st) {
    if (packed && (row_words < 1 || row_words > 256)) return hipErrorInvalidValue;
    const int64_t work = std::max<int64_t>(pair_cap * 64, msg_cap);
    hipLaunchKernelGGL(rowx_local_copy_kernel, dim3(blocks_for(work, 4096)), dim3(256), 0, st, send_rows,
                       send_rec, recv_rows, recv_rec, cnt_all, shards, g, h, pair_cap, msg_cap, row_words,
                       packed);
    return hipGetLastError();
}

hipError_t launch_rowx_recv_deg(const RowxRec *recv_rec, const int32_t *recv_msgs, int32_t shards,
                                int32_t self, int64_t msg_cap, int32_t row0, int32_t *deg,
                                hipStream_t st) {
    hipLaunchKernelGGL(rowx_recv_deg_kernel, dim3(blocks_for(msg_cap, 4096)), dim3(256), 0, st,
                       recv_rec, recv_msgs, shards, self, msg_cap, row0, deg);
    return hipGetLastError();
}

hipError_t launch_rowx_scatter_local(const int32_t *out_dst, int32_t rows, int32_t fanout,
                                     int32_t row0, const int32_t *off, int32_t *fill,
                                     int32_t *csr_src, int32_t *csr_slot, hipStream_t st) {
    hipLaunchKernelGGL(rowx_scatter_local_kernel, dim3(blocks_for(int64_t(rows) * fanout, 4096)),
                       dim3(256), 0, st, out_dst, rows, fanout, row0, off, fill, csr_src, csr_slot);
    return hipGetLastError();
}

hipError_t launch_rowx_scatter_remote(const RowxRec *recv_rec, const int32_t *recv_msgs,
                                      int32_t shards, int32_t self, int64_t msg_cap,
                                      int64_t pair_cap, const int32_t *off, int32_t *fill,
                                      int32_t *csr_src, int32_t *csr_slot, hipStream_t st) {
    hipLaunchKernelGGL(rowx_scatter_remote_kernel, dim3(blocks_for(msg_cap, 4096)), dim3(256), 0, st,
                       recv_rec, recv_msgs, shards, self, msg_cap, pair_cap, off, fill, csr_src,
                       csr_slot);
    return hipGetLastError();
}

}  // namespace gsp
