// gossip_protocol_amd/csrc/rowx_host.hpp -- host side of the row-shard exchange, shared by the
// partial-view and the full-view (row layout) engines.  Protocol and device layout:
// rowx_kernels.hpp.  One call moves tick t's cross-shard sender rows and message records and
// leaves every local shard with the receiver CSR (off, csr_src, csr_slot) of tick t + 1.
#pragma once
#include <rccl/rccl.h>

#include <vector>

#include "common.hpp"
#include "rowx_kernels.hpp"

namespace gsp {

// Exchange buffers of one shard.
struct RowxBufs {
    DevBuf<int32_t> cnt, cnt_all, recv_msgs, pair_row, csr_slot;
    DevBuf<uint64_t> send_rows, recv_rows;
    DevBuf<RowxRec> send_rec, recv_rec;

    hipError_t alloc(int32_t shards, int64_t pair_cap, int64_t msg_cap, int32_t row_words,
                     int64_t csr_cap, hipStream_t st);
    void release();
};

// What the exchange reads and writes of one local shard.
struct RowxShard {
    int32_t g, row0, rows;
    const int32_t *out_dst;       // [rows * fanout] messages of the tick being delivered
    const uint64_t *table;        // this shard's rows of that tick, row_words words each
    int32_t *deg;                 // [n] destination counts of that tick (zeroed on return)
    int32_t *off, *fill, *csr_src, *tile_sum;
    const int32_t *err;           // the shard's capacity flag (0, or the tick that overflowed)
    RowxBufs *x;
};

struct RowxJob {
    int32_t n, shards, fanout, row_words;
    int64_t pair_cap, msg_cap;
    ncclComm_t comm;              // one shard per process; null: every shard is local
    hipStream_t st;
    int32_t *h_cnt;               // pinned [G][2G + 1]: pairs, records, capacity flag per shard
    int32_t *h_recv;              // pinned [local shards][G]
};

// Counts per shard in the all-gather: G pair counts, G record counts, its capacity flag.
inline int32_t rowx_cnt_stride(int32_t shards) { return 2 * shards + 1; }

// Returns a gsp_status; *bytes += bytes the local shards sent to other shards.  Every shard's
// capacity flag travels with the counts, so every rank returns GSP_ERR_CAPACITY at the same
// point (before any send / receive) once any shard's receiver overflowed.
int rowx_exchange(const RowxJob &job, std::vector<RowxShard> &local, double *bytes);

}  // namespace gsp
