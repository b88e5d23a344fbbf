// gossip_protocol_amd/csrc/rowx_kernels.hpp -- row-sharded gossip exchange (device side).
//
// Row shard g of G owns nodes [row0(g), row0(g + 1)), row0(g) = floor(g * n / G).  A message
// of tick t from a sender of shard g to a receiver of shard h != g needs the sender's view
// of tick t on shard h before tick t + 1 merges it.  Per tick:
//   pack     one lane per local sender: for every destination shard h != g it messages, one
//            PAIR (sender row shipped once per (sender, shard), however many of its messages
//            go there) and one MESSAGE RECORD per message {src id, dst - row0(h), pair};
//   gather   one wave per pair copies the sender's row into the contiguous send region of h;
//   (host)   counts all-gathered, then RCCL send/recv of rows and records (or device copies
//            between the shards of an in-process group);
//   csr      receiver CSR over the local rows: local messages (csr_slot = local row) and
//            received records (csr_slot = -(region * pair_cap + pair) - 1 into the remote rows).
// HBM layout per shard, one REGION per other shard (rowx_region; none for the shard itself):
// send_rows[G-1][pair_cap][wire_words], send_rec[G-1][msg_cap], recv_rows[G-1][pair_cap]
// [row_words] (what the tick kernels read), recv_wire[G-1][pair_cap][wire_words] (RCCL
// receives, packed rows only), recv_rec[G-1][msg_cap].  pair_cap = max rows of a shard
// makes every tick fit (a sender row goes to a shard at most once); an engine may size it
// smaller for large rows, in which case a count above the capacity fails the tick
// (GSP_ERR_CAPACITY, set on the device) and nothing is written out of bounds.
//
// Wire format.  A full-view row (u16 entries) travels as it is.  A partial-view row (V u64
// entries id << 32 | hb << 5 | ts5, sorted by id, empty slots last) travels PACKED: the low 16
// bits of each id (u16[V]), each value (u16[V]) and, because the ids ascend, their high 5 bits
// as 33 run boundaries: bound[h] = entries whose id >> 16 is below h (bound[32] = the entry
// count) -- 4 V + 66 bytes instead of 8 V (1,090 B instead of 2,048 B at V = 256).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsp {

struct RowxRec {
    int32_t src;     // global sender id
    int32_t dst;     // receiver, local to the destination shard
    int32_t pair;    // index of the sender's row in the (src shard -> dst shard) region
};

// 8-byte words of a packed partial-view row of V entries
__host__ __device__ inline int32_t rowx_packed_words(int32_t V) { return (4 * V + 66 + 7) / 8; }

struct RowxArgs {
    int32_t n, shards, shard, fanout;
    int32_t row0, rows;              // this shard's rows
    int64_t pair_cap, msg_cap;       // per (src shard, dst shard) region
    int32_t row_words;               // 8-byte words per row (packed: V, the entries per row)
    int32_t packed;                  // 1: send_rows holds packed rows (rowx_packed_words(V) each)
    const int32_t *out_dst;          // [rows * fanout] global destination ids, -1 = none
    const uint64_t *table;           // this shard's rows of the tick the messages were sent in
    int32_t *pair_cnt;               // [G] pairs per destination shard (zeroed before pack)
    int32_t *msg_cnt;                // [G] records per destination shard
    int32_t *pair_row;               // [G-1][pair_cap] local row of each pair
    uint64_t *send_rows;             // [G-1][pair_cap][row_words]
    RowxRec *send_rec;               // [G-1][msg_cap]
};

// owner shard of a global node id
__host__ __device__ inline int32_t rowx_owner(int32_t d, int32_t n, int32_t shards) {
    return int32_t(((int64_t(d) + 1) * shards - 1) / n);
}
__host__ __device__ inline int32_t rowx_row0(int32_t g, int32_t n, int32_t shards) {
    return int32_t(int64_t(g) * n / shards);
}

// region of peer shard h != self in a shard's send / receive buffers
__host__ __device__ inline int64_t rowx_region(int32_t h, int32_t self) {
    return h < self ? h : h - 1;
}

hipError_t launch_rowx_pack(const RowxArgs &a, hipStream_t st);
hipError_t launch_rowx_gather(const RowxArgs &a, hipStream_t st);

// After the counts all-gather (cnt_all[G][2G + 1]: pairs per destination, records per
// destination, capacity flag, of every shard): shard `self` checks every count against its
// capacity and -- RCCL path -- against the sizes the host posted for this exchange (bounds
// [2][G][G]: pairs, records; null: the capacities only), and any shard's capacity flag; the
// first failure sets *err = tick | kRowxErrBit (tick if a shard's receipt flag).  It writes the
// true counts this shard receives, clamped to what arrived, to recv_pairs[G] / recv_msgs[G]:
// the in-band counts every later kernel of the exchange reads.
constexpr int32_t kRowxErrBit = 1 << 24;
hipError_t launch_rowx_check(const int32_t *cnt_all, const int32_t *bounds, int32_t shards, int32_t self,
                             int64_t pair_cap, int64_t msg_cap, int32_t tick, int32_t *err,
                             int32_t *recv_pairs, int32_t *recv_msgs, hipStream_t st);
// Received rows of every source shard h != self (recv_pairs[h] of them) into recv_rows:
// packed rows decoded from recv_wire, raw rows copied from it.
hipError_t launch_rowx_unpack(const uint64_t *recv_wire, uint64_t *recv_rows, const int32_t *recv_pairs,
                              int32_t shards, int32_t self, int64_t pair_cap, int32_t row_words,
                              int32_t packed, hipStream_t st);
// In-process groups: shard g's send region for h -> shard h's receive region for g, rows
// (decoded when packed) and records, sized by the device counts (cnt_all row g).
hipError_t launch_rowx_local_copy(const uint64_t *send_rows, const RowxRec *send_rec, uint64_t *recv_rows,
                                  RowxRec *recv_rec, const int32_t *cnt_all, int32_t shards, int32_t g,
                                  int32_t h, int64_t pair_cap, int64_t msg_cap, int32_t row_words,
                                  int32_t packed, hipStream_t st);
// deg[row0 + rec.dst]++ for the received records of every source shard h != self
// (counts: recv_msgs[h])
hipError_t launch_rowx_recv_deg(const RowxRec *recv_rec, const int32_t *recv_msgs, int32_t shards,
                                int32_t self, int64_t msg_cap, int32_t row0, int32_t *deg,
                                hipStream_t st);
// local messages: csr_src = sender id, csr_slot = sender's local row
hipError_t launch_rowx_scatter_local(const int32_t *out_dst, int32_t rows, int32_t fanout,
                                     int32_t row0, const int32_t *off, int32_t *fill,
                                     int32_t *csr_src, int32_t *csr_slot, hipStream_t st);
// received records: csr_slot = -(rowx_region(h, self) * pair_cap + pair) - 1
hipError_t launch_rowx_scatter_remote(const RowxRec *recv_rec, const int32_t *recv_msgs,
                                      int32_t shards, int32_t self, int64_t msg_cap,
                                      int64_t pair_cap, const int32_t *off, int32_t *fill,
                                      int32_t *csr_src, int32_t *csr_slot, hipStream_t st);

}  // namespace gsp
