// gossip_protocol_amd/csrc/exact_kernels.hpp -- device side of the EXACT engine.
//
// Layout in HBM (N <= 1024 nodes, column x <-> node id x+1, EmulNet.cpp:72-77):
//   committed table   key[N][N] int64 (-1 = absent), hb[N][N] int32, ts[N][N] int32,
//                     rank[N][N] int32 (position in the member list, valid when present)
//   node state        inited[N], in_group[N], own_hb[N], nlist[N] (int32)
// A phase-P batch reads only the committed table (the send-time snapshot of every
// sender's list, MP1Node.cpp:357) and writes per-batch output rows, which a second
// kernel commits.  The member list order is carried by an insertion key
// (batch, queue index j, payload position p + 1): list order = ascending key.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsp {

enum : int32_t { kEvStartGroup = 0, kEvStartJoin = 1, kEvJoin = 2, kEvRemove = 3 };

struct ExactEvent {     // one dbg.log line produced by a batch node
    int32_t pos;        // position of the node in the batch (call order)
    int32_t kind;       // kEv*
    int32_t subject;    // column (node index) joined/removed
    int32_t pad;
    int64_t ord;        // order inside (pos, kind): join (j << 20 | p+1), remove -key
};

struct ExactTable {
    int64_t *key;
    int32_t *hb, *ts, *rank;
    int32_t *inited, *in_group, *own_hb, *nlist;
};

struct ExactBatchDev {
    int32_t n_batch;
    const int32_t *node, *op;          // [B]
    const int32_t *q_off;              // [B+1] CSR of each node's drained queue
    const int32_t *q_src, *q_type;     // [Q]  sender id, message type
    // payload of each queued message: q_prow[q] < 0 reads the sender's committed row of the
    // table (the normal case), >= 0 the row q_prow[q] of the p_* arrays, a list handed in by
    // the driver or kept from send time (gsp_queue_push / gsp_recv_callback / snapshots);
    // q_prow null: every payload is a committed row
    const int32_t *q_prow;             // [Q] or null
    const int64_t *p_key;              // [P][N] >= 0 present
    const int32_t *p_hb, *p_ts, *p_rank;   // [P][N]
    const int32_t *p_nlist;            // [P]
    // the list each JOINREP carries, as the reply is sent (MP1Node.cpp:225-229: after the
    // JOINREQ's addMember, before the rest of the queue): row rep_off[pos] + (reply index),
    // columns key (>= 0 present, list order) / hb / ts; rep_key null: not recorded
    const int32_t *rep_off;            // [B]
    int64_t *rep_key;
    int32_t *rep_hb, *rep_ts;
    const int32_t *send_off;           // [B+1] capacity offsets of the per-node send lists
    // outputs
    int64_t *o_key;                    // [B][N]
    int32_t *o_hb, *o_ts, *o_rank;     // [B][N]
    int32_t *o_state;                  // [B][4] inited, in_group, own_hb, nlist
    int32_t *send_dst, *send_type;     // [send_off[B]]
    int32_t *send_cnt;                 // [B]
    ExactEvent *events;                // [ev_cap]
    int32_t *ev_count;                 // [1]
    int32_t ev_cap;
    unsigned long long *merges;        // [1]
    int32_t intro_list;                // JOINREP payload bound (gsp_params.intro_list; 0 = off)
    uint64_t seed;                     // Philox key of the introducer-list draws
};

// Send builder: assigns global draw indices in batch order, draws, applies the drop
// window and the EmulNet buffer bound (EmulNet.cpp:87-118), compacts admitted sends.
struct ExactSendDev {
    int32_t n_batch;
    const int32_t *node, *send_off, *send_cnt, *send_dst, *send_type;
    int32_t rng_mode;                  // 0 glibc stream, 1 philox
    int32_t *adm_slot;                 // [admitted] send-list slot (send_off[pos] + k), or null
    const int32_t *glibc_stream;       // values of rand() by draw index
    int64_t stream_base;               // draw index of glibc_stream[0]
    int64_t g0;                        // global draw index of the batch's first send
    uint64_t seed;
    int32_t tick, dropmsg, drop_thr;   // drop iff dropmsg && draw % 100 < drop_thr
    int32_t buff_room;                 // EmulNet buffer slots still free
    int32_t size_reject;               // message bigger than MAX_MSG_SIZE: every send rejected
    int32_t *adm_src, *adm_dst, *adm_type;  // admitted sends, in draw order
    int32_t *adm_count;                // [1]
    int32_t *draws;                    // [1] draws consumed
    int32_t *sent_ctr;                 // [N+1][max_ticks] per-(id, tick) sent counters
    int32_t max_ticks;
};

hipError_t launch_exact_batch(const ExactTable &tab, const ExactBatchDev &b, int32_t n,
                              int32_t tick, int64_t batch_seq, int32_t tremove,
                              int32_t id_filter_limit, hipStream_t st);
hipError_t launch_exact_commit(const ExactTable &tab, const ExactBatchDev &b, int32_t n,
                               hipStream_t st);
hipError_t launch_exact_sends(const ExactSendDev &s, hipStream_t st);

}  // namespace gsp
