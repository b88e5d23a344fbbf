// gossip_protocol_amd/csrc/scale_kernels.hpp -- device side of the SCALE engine.
//
// HBM layout (full view, V = n columns, stride = n rounded up to 2048 entries):
//   table[2][rows][stride]  uint16 entries, ping-pong by tick parity:
//                           entry = hb << 5 | (ts mod 32), 0 = absent; hb in [1, 2047]
//   own_hb[rows], fail_tick[rows], cnt[2][rows] (member count, by tick parity)
//   out_dst[rows * fanout]  this tick's messages (dst id or -1) from each sender slot
//   deg[n], off[n + 1], fill[n], csr_src[n * fanout]   next tick's receiver CSR
//   dig[ticks][kDigSlots][kDigFields]   sharded per-tick digest accumulators
// ts is kept modulo 32: every timestamp the protocol ever compares is within 20 ticks
// of the current tick ("Why 16 bits are exact").
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsp {

constexpr int kScaleBlock = 256;          // 4 waves
constexpr int kEntriesPerLane = 8;        // 16 B per lane per row chunk
constexpr int kChunk = kScaleBlock * kEntriesPerLane;   // 2048 columns per block iteration
constexpr int kMaxSegment = 1024;         // messages one receiver can merge per tick
constexpr int kDigSlots = 64;             // atomic sharding of the per-tick digest
enum : int { kDigRounds = 0, kDigMerges, kDigSent, kDigDropped, kDigDelivered, kDigJoins,
             kDigRemoves, kDigHash, kDigFields };

struct ScaleTickArgs {
    const uint16_t *prev;        // table of tick t-1
    uint16_t *cur;               // table of tick t
    int64_t stride;              // entries per row
    int32_t n;                   // nodes = columns
    int32_t row0;                // first global row of this shard (0 on one GPU)
    int32_t rows;                // rows of this shard
    int32_t tick;
    int32_t tremove;
    int32_t fanout;
    int32_t drop_pct;
    int32_t h0;
    uint64_t seed;
    const int32_t *fail_tick;    // [n] global
    int32_t *own_hb;             // [rows]
    const int32_t *cnt_prev;     // [n] member counts at t-1 (global ids)
    int32_t *cnt_cur;            // [n]
    const int32_t *off;          // [rows + 1] receiver CSR
    const int32_t *csr_src;      // sender ids
    int32_t *out_dst;            // [rows * fanout]
    int32_t *deg;                // [n] messages per destination (atomic)
    unsigned long long *dig;     // [kDigSlots][kDigFields] of this tick
    int32_t *err;                // [1] capacity error flag
};

hipError_t launch_scale_init(const ScaleTickArgs &a, hipStream_t st);
// policy: cache policy of the row streams (bit 0 own row non-temporal, bit 1 sender rows)
hipError_t launch_scale_tick(const ScaleTickArgs &a, int policy, hipStream_t st);
// off[0..n] = exclusive scan of deg[0..n); tile_sum holds ceil(n / 4096) ints of scratch
hipError_t launch_exclusive_scan(const int32_t *deg, int32_t *off, int32_t n, int32_t *tile_sum,
                                 hipStream_t st);
// csr_src[off[d] + k] = sender, for every message slot i with out_dst[i] = d >= 0
hipError_t launch_scatter(const int32_t *out_dst, int64_t slots, int32_t fanout, int32_t row0,
                          const int32_t *off, int32_t *fill, int32_t *csr_src, hipStream_t st);
size_t scale_lds_bytes(int64_t stride);

}  // namespace gsp
