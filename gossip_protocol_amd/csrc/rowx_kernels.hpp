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
// send_rows[G-1][pair_cap][row_words], send_rec[G-1][msg_cap], recv_rows[G-1][pair_cap]
// [row_words], recv_rec[G-1][msg_cap].  pair_cap = max rows of a shard
// makes every tick fit (a sender row goes to a shard at most once); an engine may size it
// smaller for large rows, in which case a count above the capacity fails the tick
// (GSP_ERR_CAPACITY) and nothing is written out of bounds.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsp {

struct RowxRec {
    int32_t src;     // global sender id
    int32_t dst;     // receiver, local to the destination shard
    int32_t pair;    // index of the sender's row in the (src shard -> dst shard) region
};

struct RowxArgs {
    int32_t n, shards, shard, fanout;
    int32_t row0, rows;              // this shard's rows
    int64_t pair_cap, msg_cap;       // per (src shard, dst shard) region
    int32_t row_words;               // 8-byte words per row
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
