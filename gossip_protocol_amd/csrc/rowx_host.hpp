// gossip_protocol_amd/csrc/rowx_host.hpp -- host side of the row-shard exchange, shared by the
// partial-view and the full-view (row layout) engines.  Protocol and device layout:
// rowx_kernels.hpp.  One call moves tick t's cross-shard sender rows and message records and
// leaves every local shard with the receiver CSR (off, csr_src, csr_slot) of tick t + 1.
//
// No host wait on the stream: the counts are all-gathered and checked on the device, every
// kernel of the exchange reads the true counts from device memory (in-band), and RCCL -- which
// needs element counts when the call is posted -- is given sizes both sides derive from the
// counts of EARLIER exchanges: the largest count seen so far for that (sender shard, receiver
// shard) plus a margin (1/16 + 256 rows / 1,024 records), capped at the region's capacity.
// Those counts reach the host through pinned memory and one event per exchange; the host
// waits only for the previous exchange's event, so it stays at most one tick ahead of the
// device.  A count past the posted size (or a capacity) sets the job's error flag on the
// device (kRowxErrBit): that tick's tick kernels run no row and the engine reports
// GSP_ERR_CAPACITY -- never a silently truncated exchange.
#pragma once
#include <rccl/rccl.h>

#include <vector>

#include "common.hpp"
#include "rowx_kernels.hpp"

namespace gsp {

// Exchange buffers of one shard.
struct RowxBufs {
    DevBuf<int32_t> cnt, cnt_all, recv_msgs, recv_pairs, pair_row, csr_slot, bounds;
    DevBuf<uint64_t> send_rows, recv_rows, recv_wire;
    DevBuf<RowxRec> send_rec, recv_rec;

    // row_words: 8-byte words of a table row (packed: the view V); packed rows travel in
    // rowx_packed_words(V) words
    hipError_t alloc(int32_t shards, int64_t pair_cap, int64_t msg_cap, int32_t row_words,
                     bool packed, bool rccl, int64_t csr_cap, hipStream_t st);
    void release();
};

// What the exchange reads and writes of one local shard.
struct RowxShard {
    int32_t g, row0, rows;
    const int32_t *out_dst;       // [rows * fanout] messages of the tick being delivered
    const uint64_t *table;        // this shard's rows of that tick, row_words words each
    int32_t *deg;                 // [n] destination counts of that tick (zeroed on return)
    int32_t *off, *fill, *csr_src, *tile_sum;
    int32_t *err;                 // the job's capacity flag (0, or the tick that overflowed)
    RowxBufs *x;
};

// Host state of an engine's exchanges: the count ring, the sizes posted, the bytes accounted.
struct RowxState {
    static constexpr int kRing = 4;
    int32_t shards = 0;
    int32_t *h_cnt = nullptr;     // pinned [kRing][G][2G + 1]: all-gathered counts per exchange
    int32_t *h_bounds = nullptr;  // pinned [kRing][2][G][G]: pair / record sizes posted (RCCL)
    hipEvent_t ev[kRing] = {};
    int64_t seq = 0;              // exchanges posted
    int64_t seen = 0;             // exchanges whose counts the host has read
    std::vector<int64_t> max_pairs, max_msgs;   // [G][G] largest counts seen
    double wire_bytes_per_row = 0, rec_bytes = 12;
    bool rccl = false;
    bool tight = false;           // tests (GSP_TEST_ROWX_TIGHT=1): an in-process group posts and
                                  // checks sizes too, with no margin (the largest count seen)
    bool posted = false;          // tests (GSP_TEST_ROWX_POSTED=1): an in-process group posts and
                                  // checks the sizes a communicator would post (every margin)

    hipError_t init(int32_t shards, bool rccl);
    void release();
};

struct RowxJob {
    int32_t n, shards, fanout, row_words;
    bool packed;                  // partial-view rows, packed on the wire
    int64_t pair_cap, msg_cap;
    ncclComm_t comm;              // one shard per process; null: every shard is local
    hipStream_t st;
    int32_t tick;                 // the tick whose tick kernels read this exchange
    RowxState *state;
    // growth the host knows of between the last exchange whose counts it has read and this one
    // (the posted sizes must cover it): senders whose first sends these are (a join schedule's
    // nodes starting at the send tick), and the drop percentages of the sends of this exchange
    // and of the one before
    int64_t new_senders = 0;
    int32_t drop_now = 0, drop_before = 0;
};

// Counts per shard in the all-gather: G pair counts, G record counts, its capacity flag.
inline int32_t rowx_cnt_stride(int32_t shards) { return 2 * shards + 1; }

// Posts one exchange (no stream synchronisation).  *bytes += bytes accounted to the wire: the
// sizes posted to RCCL by this rank, or, for an in-process group, the true counts once the host
// has read them (rowx_collect adds the last exchange's).
int rowx_exchange(const RowxJob &job, std::vector<RowxShard> &local, double *bytes);
// Reads the counts of every posted exchange (waits for the last one's event) and accounts
// their bytes; call before reading *bytes.
int rowx_collect(RowxState &s, double *bytes);

}  // namespace gsp
