// gossip_protocol_amd/csrc/scale_kernels.hpp -- device side of the SCALE engine.
//
// HBM layout (full view, V = n columns):
//   table[2][rows][stride]  uint16 entries, ping-pong by tick parity:
//                           entry = hb << 5 | (ts mod 32), 0 = absent; hb in [1, 2047].
//                           One GPU: stride = n rounded up to 2048.  Column shard g of G:
//                           all n rows, columns [col0, col0 + stride), stride = width / G.
//   own_hb[rows], fail_tick[n], cnt[2][n] (member count by tick parity)
//   out_dst[rows * fanout]  this tick's messages (dst id or -1) of each sender slot
//   ping[rows]              swim: this tick's probe target (global id or -1)
//   deg[n], off[n + 1], fill[n], csr_src[n * fanout] (+ csr_slot)  next tick's receiver CSR
//   dig[ticks][kDigSlots][kDigFields]   sharded per-tick digest accumulators
// ts is kept modulo 32: every timestamp the protocol ever compares is within 20 ticks of
// the current tick ("Why 16-bit entries are exact").
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "event_ring.hpp"

namespace gsp {

constexpr int kScaleBlock = 256;          // 4 waves
constexpr int kEntriesPerLane = 8;        // 16 B per lane per row chunk
constexpr int kChunk = kScaleBlock * kEntriesPerLane;   // 2048 columns per block iteration
constexpr int kEvStage = 512;             // event stream: LDS-staged records per wave (one chunk's worst case)
constexpr int kMaxSegment = 1024;         // receiver segments sorted in LDS; longer ones are sorted in HBM
constexpr int kDigSlots = 64;             // atomic sharding of the per-tick digest
enum : int { kDigRounds = 0, kDigMerges, kDigSent, kDigDropped, kDigDelivered, kDigJoins,
             kDigRemoves, kDigHash, kDigFields };

struct ScaleTickArgs {
    const uint16_t *prev;        // table of tick t-1 (this shard's rows x stride)
    uint16_t *cur;               // table of tick t
    const uint16_t *remote;      // row mode: sender rows received from other shards
    int64_t stride;              // entries per row in this shard's table
    int32_t n;                   // nodes = global columns
    int32_t col0;                // first global column of this shard (column mode)
    int32_t row0;                // first global row of this shard (row mode)
    int32_t rows;                // rows of this shard
    int32_t tick;
    int32_t tremove;
    int32_t fanout;
    int32_t drop_pct;
    int32_t h0;
    int32_t nt_own, nt_src;      // non-temporal policy of the own-row / sender-row streams
    int32_t pipe;                // software-pipelined chunk loads (packed merge, policy 1)
    int32_t lds_pad;             // extra dynamic LDS bytes per workgroup (occupancy experiments)
    int32_t tfail;               // TFAIL suspicion: 0 off, else members this stale are not
                                 // gossiped / chosen / counted
    int32_t swim;                // SWIM probing: 0 off, else 1 direct + swim - 1 indirect paths
    int32_t count_rounds;        // this shard adds node-rounds / merges / sends to the digest
    uint64_t seed;
    const int32_t *fail_tick;    // [n] global
    const int32_t *start_tick;   // [n] global, or null: every node starts at tick 0 (policy.hpp)
    int32_t drop_prev;           // drop percentage of the sends of tick - 1 (SWIM probe paths)
    // JOINREPs (join_kernels.hpp): a receiver whose segment starts with kJoinRepSrc merges the
    // introducer's row of tick - 1 cut to intro_list Philox-chosen gossipable members
    const uint16_t *intro;       // node 0's row of tick - 1, this table's columns
    int32_t intro_list;          // B (gsp_policy.intro_list)
    const int32_t *intro_cnt;    // column shards: cnt_all ([shards][n]: node 0's slice counts at
                                 // intro_cnt[g * n]); null: one slice holds the whole row
    int32_t shards, shard;       // column shards: this slice's index among `shards`
    int32_t *own_hb;             // [rows]
    const int32_t *cnt_prev;     // [n] member counts at t-1 (global ids)
    int32_t *cnt_cur;            // [n] (fused: member count; slice: count in this slice)
    const int32_t *off;          // [rows + 1] receiver CSR
    int32_t *csr_src;            // sender ids (a segment longer than kMaxSegment is sorted in
                                 // place by its row's workgroup)
    int32_t *csr_slot;           // row mode: >= 0 local row, < 0 remote row -slot-1 (or null)
    int32_t *out_dst;            // [rows * fanout]
    int32_t *deg;                // [n] messages per destination (atomic)
    int32_t *ping;               // swim: [rows] probe target of the last send (-1 none)
    uint8_t *bitmap;             // slice mode: [rows][stride / 8] presence bits
    unsigned long long *dig;     // [kDigSlots][kDigFields] of this tick
    // event stream (gsp_scale_params.events): every join / remove as one 64-bit record
    // kind << 62 | t << 42 | r << 21 | x (event_record), appended in wave-compacted runs
    EvRingArgs ev;               // event stream (ev.buf null: off), event_ring.hpp
    int32_t *err;                // [1] capacity error: 0, else the first tick a receiver got
                                 // more than max_segment messages (every later tick is a no-op)
    int32_t max_segment;         // no bound (INT32_MAX) unless a test lowers it (GSP_TEST_MAX_SEGMENT)
    int32_t *long_list;          // [1 + rows] of this tick's parity: count, then the rows whose
                                 // segment is longer than kMaxSegment (deferred to
                                 // scale_long_kernel); null: the tile appends nothing (the other
                                 // tiles of a shared CSR)
};

__host__ __device__ inline unsigned long long event_record(uint32_t kind, uint32_t t, uint32_t r,
                                                           uint32_t x) {
    return (uint64_t(kind) << 62) | (uint64_t(t & 0xFFFFFu) << 42) | (uint64_t(r & 0x1FFFFFu) << 21) |
           uint64_t(x & 0x1FFFFFu);
}

// Reserve `cnt` ring slots for this lane: one wave prefix and one atomic per wave; returns
// the lane's first slot (slots >= cap are lost).  Call from converged code.
__device__ inline uint64_t wave_reserve_events(unsigned long long *count, uint32_t cnt) {
    if (!__ballot(cnt > 0)) return 0;                  // wave-uniform
    uint32_t incl = cnt;                               // inclusive wave scan (DPP-free form)
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(incl, d, 64);
        if ((threadIdx.x & 63) >= uint32_t(d)) incl += u;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    unsigned long long base = 0;
    if ((threadIdx.x & 63) == 63) base = atomicAdd(count, (unsigned long long)total);
    base = __shfl(base, 63, 64);
    return base + (incl - cnt);
}

// Append this lane's `cnt` records (rec(i), i < cnt) to the ring (wave_reserve_events).
template <typename Rec>
__device__ inline void wave_append_events(unsigned long long *buf, unsigned long long *count,
                                          int64_t cap, uint32_t cnt, Rec &&rec) {
    uint64_t p = wave_reserve_events(count, cnt);
    for (uint32_t i = 0; i < cnt; ++i, ++p)
        if (int64_t(p) < cap) buf[p] = rec(i);
}

// merge: 0 = per-entry scalar form, 1 = packed 16-bit form (v_pk_* / v_bfi_b32)
hipError_t launch_scale_init(const ScaleTickArgs &a, bool slice, hipStream_t st);
hipError_t launch_scale_tick(const ScaleTickArgs &a, bool slice, int merge, hipStream_t st);
// the rows every tick-kernel launch of this tick deferred (k > kMaxSegment): tpl[2 * g + parity]
// = local tile g's args at tick parity (dig at tick 0); a = tile 0's args of this tick
hipError_t launch_scale_long(const ScaleTickArgs &a, const ScaleTickArgs *tpl, int32_t ntiles, bool slice,
                             hipStream_t st);

// Column mode, after the all-gather of every shard's per-row slice counts:
//   resolve: per sender, Philox rank-select over the global order of its members; the
//            shard owning the chosen rank resolves the column from its bitmap slice.
//            picks[s * f + k] = column or -1; cnt_total[s] = member count of s.
//   finalize (after an all-reduce MAX of picks): drop draw, out_dst, deg.
struct ScaleResolveArgs {
    int32_t n, fanout, tick, drop_pct, shard, shards, count_rounds;
    const int32_t *start_tick;   // [n] or null
    int32_t swim;                // SWIM probing: picks hold fanout + 1 slots per sender, the
                                 // last one the probe target; finalize copies it to ping[]
    int64_t stride;              // slice width
    int32_t tiled;               // 1: local shards tile_lo .. tile_lo + tile_cnt - 1 keep their
                                 // bitmaps at bitmap + (g - tile_lo) * tile_bytes and this launch
                                 // resolves the ranks of all of them (shared shards)
    int32_t tile_lo, tile_cnt;
    int64_t tile_bytes;
    uint64_t seed;
    const int32_t *fail_tick;
    const int32_t *cnt_all;      // [shards][n]
    int32_t *cnt_total;          // [n]
    const uint8_t *bitmap;       // [n][stride / 8]
    int32_t *picks;              // [n * (fanout + (swim > 0))]
    int32_t *ping;               // swim: [n] probe target of each sender (or -1)
    int32_t *out_dst;            // [n * fanout]
    int32_t *deg;                // [n]
    unsigned long long *dig;
};
hipError_t launch_scale_resolve(const ScaleResolveArgs &a, hipStream_t st);
hipError_t launch_scale_finalize(const ScaleResolveArgs &a, hipStream_t st);
hipError_t launch_max_into(int32_t *dst, const int32_t *src, int64_t count, hipStream_t st);

// off[0..n] = exclusive scan of deg[0..n); tile_sum holds ceil(n / 4096) ints of scratch
hipError_t launch_exclusive_scan(const int32_t *deg, int32_t *off, int32_t n, int32_t *tile_sum,
                                 hipStream_t st);
// err = t (if 0) when a receiver segment of off[rows + 1] is longer than max_segment
hipError_t launch_segment_check(const int32_t *off, int32_t rows, int32_t max_segment, int32_t *err,
                                int32_t t, hipStream_t st);
// csr_src[off[d] + k] = sender, for every message slot i with out_dst[i] = d >= 0
hipError_t launch_scatter(const int32_t *out_dst, int64_t slots, int32_t fanout, int32_t row0,
                          const int32_t *off, int32_t *fill, int32_t *csr_src, hipStream_t st);
size_t scale_lds_bytes(int64_t stride, bool slice, bool events);

}  // namespace gsp
