// gossip_protocol_amd/csrc/pview_kernels.hpp -- device side of the PARTIAL-VIEW engine.
//
// HBM layout (BASELINE config 5: n = 1,048,576 nodes, V = 256):
//   view[2][rows][V]   uint64 entry = id << 32 | hb << 5 | (ts mod 32); ~0 = empty slot.
//                      Each row is sorted by id with the empty slots last (2 KB at V = 256).
//   len[2][rows]       entries per row (by tick parity)
//   own_hb[rows], fail_tick[n], out_dst[rows * fanout], deg/off/fill/csr_src (receiver CSR)
//   rc_info[rows], rc_src/rc_slot[rows][8]   receipt records (K smallest senders)
//   rowdig[rows][4][4] per-row digest records of the current tick (one per wave)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "event_ring.hpp"

namespace gsp {

constexpr int kPvBlock = 256;
constexpr int kPvMaxView = 256;       // V <= 256: one entry per lane per list
constexpr int kPvMaxInbox = 7;        // K <= 7 messages merged per receiver per tick
constexpr uint64_t kPvEmpty = ~0ull;
enum : int { kPvRounds = 0, kPvMerges, kPvSent, kPvDropped, kPvDelivered, kPvOverflow,
             kPvJoins, kPvRemoves, kPvEvicts, kPvHash, kPvFields };
constexpr int kPvDigSlots = 256;   // spread the per-row digest atomics

// messages one receiver can be sent in one tick: the receipt kernel keeps the K smallest of any
// number, so the bound is only the 16-bit per-row overflow field of the digest record (round 2
// used 1024, which config 5's in-degree skew passes at tick ~73: the (age, -hb, id) eviction
// order favours low ids, so a few nodes end up in most views)
constexpr int kPvMaxSegment = 65535 + kPvMaxInbox;

struct PviewTickArgs {
    const uint64_t *prev;        // view table of tick t-1 (this shard's rows)
    uint64_t *cur;               // view table of tick t
    const uint64_t *remote;      // row mode: sender rows received from other shards
    int32_t n, view, inbox, fanout, tick, tremove, drop_pct, h0;
    int32_t row0, rows;
    uint64_t seed;
    const int32_t *fail_tick;    // [n]
    const int32_t *start_tick;   // [n], or null: every node starts at tick 0 (policy.hpp)
    int32_t drop_prev;           // drop percentage of the sends of tick - 1 (SWIM probe paths)
    int32_t tfail, swim;         // TFAIL suspicion / SWIM probing (0: off), as the full view
    int32_t *ping;               // swim: [rows] probe target chosen at the last send (-1 none)
    const uint64_t *intro;       // node 0's view of tick - 1: the JOINREP payload source
    int32_t intro_list;          // JOINREP payload bound B
    int32_t *own_hb;             // [rows]
    int32_t *len_cur;            // [rows] view length of this tick
    const int32_t *rc_info;      // [rows] receipt record: k | k_all << 3
    const int32_t *rc_src;       // [rows][8] the k smallest senders, ascending
    const int32_t *rc_slot;      // [rows][8] their rows: >= 0 local, < 0 remote (-slot - 1)
    int32_t *out_dst;            // [rows * fanout]
    int32_t *out_pos;            // [rows * fanout]: each message's slot in its receiver's CSR
                                 // segment (the send kernel's deg atomic), or null
    int32_t *deg;                // [n]
    unsigned long long *rowdig;  // [rows][4][4] per-row digest records of this tick
    unsigned long long *dig;     // [kPvDigSlots][kPvFields] of this tick
    int32_t *err;                // [1] capacity error: 0, else the first tick a receiver was
                                 // sent more than max_segment messages (the job stops there)
    int32_t max_segment;         // <= kPvMaxSegment (lowered only by tests)
    EvRingArgs ev;               // event stream (ev.buf null: off), event_ring.hpp
    const int32_t *kcount;       // [8] rows per merged-message count k (or null: row order)
    const int32_t *order;        // [8][rows]: the rows of each k; workgroup b runs the b-th row
                                 // of the k-descending order (one code variant per CU stretch)
    unsigned long long *prof;    // diagnostics: per-phase cycles of sampled rows (or null)
    int32_t split;               // with order set: rows bucketed by k into four kernels
    int32_t *kcount_host;        // pinned [8]: the split kernels' grids, the bucket sizes read
    hipEvent_t kcount_event;     // back behind this event after the receipt kernel
    int32_t evict_rot;           // evict_order 1: eviction ties by the rotated id (gossip.h)
    int32_t *rows_run;           // tests only (GSP_TEST_PV_COUNT_ROWS=1): [1] counter of this
                                 // tick, +1 per row a tick kernel runs (every row exactly once,
                                 // in every launch form), or null
    // drain-all (gsp_pview_params.inbox = 0, pview_drain.hip): a row sent more than
    // kPvMaxInbox messages is listed by the receipt kernel and merges them all there
    int32_t drain;               // 1: inbox 0 (the tick kernels skip the listed rows)
    const int32_t *long_list;    // [kDrainHead + kDrainClasses * rows]: counts, then the rows per class
    const int32_t *csr_off;      // [rows + 1] this tick's receiver CSR
    int32_t *csr_src, *csr_slot; // its senders (sorted in place) and rows (row mode, or null)
    uint32_t *scratch;           // [cus][2][scratch_cap] u64: HBM tuple buffers (hub rows)
    int64_t scratch_cap;         // tuples per buffer (>= 8192, a power of two)
    int32_t cus;                 // compute units: the hub kernel's persistent grid
    int32_t drain_lds;           // LDS tuple capacity in use (tests lower it to reach the hub
                                 // kernel, GSP_TEST_PV_DRAIN_LDS), <= kDrainLdsMax
    int32_t drain_wide;          // tests (GSP_TEST_PV_DRAIN_WIDE=w): the rows of classes < w run
                                 // in class w
    int32_t *drain_rows;         // pinned [kDrainHead]: long_list's head, copied back with the
                                 // split kernels' bucket sizes -- the drain classes' grids (a
                                 // class without rows is not launched), or null (persistent grids)
    int32_t nowait;              // 1 (row shards): no host wait for the bucket sizes -- every split
                                 // kernel launches on `rows` workgroups (those past their bucket
                                 // exit at once), the drain classes on persistent grids
    int32_t *dhead_async;        // nowait + drain all: pinned [kDrainHead], long_list's head copied
                                 // without a wait (the engine reads it after its next sync), or null
    hipStream_t drain_st;        // split form: the drain classes run on this stream beside the split
    hipEvent_t drain_fork, drain_join;   // kernels (fork after the receipt, join before the send
                                         // kernel), or null: on the tick's stream after them
    int32_t drain_side;          // with drain_st: 1 every drain class there, 2 the hub kernel only
    hipEvent_t *drain_ev;        // [kDrainClasses + 2]: recorded before the first drain class and
                                 // after each (the per-class kernel time; [kDrainClasses + 1]: the
                                 // hub kernel's start on its own stream), or null
};

// Drain-all row classes (pview_drain.hip), by the row's update tuples: own view + k payloads
// (Vp = pow2(V) slots each) + the senders' runs.  In LDS (k <= kDrainStage): 0: <= 3,072
// tuples, 192-lane rows, 5 per CU; 1: <= 4,096, 256-lane rows, 4 per CU; 2: <= 8,192, 512-lane
// rows, 2 per CU; 3: <= 16,384, 1024-lane rows, 1 per CU (k <= 10 / 14 / 30 / 62 at V = 256).
// Class 4 (kDrainHub): the rest, 1024-lane rows in two HBM buffers per workgroup (and every
// row of a view below 8 slots).  long_list: kDrainHead words -- the rows of each class at [c],
// their messages at [8 + c] -- then the rows of each class.
constexpr int kDrainClasses = 5;
constexpr int kDrainHub = 4;
constexpr int kDrainHead = 16;
constexpr int kDrainStage = 64;
constexpr int kDrainLdsMax = 16384;
// class 0: tuples, rows per CU, waves per SIMD (round 6: 2,560 / 6 / 5 -- the k <= 8 rows alone,
// 76 B of spills -- ran 5.05 ms of drain against 5.03)
constexpr int kDrainCap0 = 3072, kDrainPerCU0 = 5, kDrainWaves0 = 4;
// a hub row past its HBM buffers stops the job: err = tick | kDrainErrBit (kRowxErrBit: 1 << 24)
constexpr int32_t kDrainErrBit = 1 << 25;
__host__ __device__ inline int64_t pv_drain_need(int32_t k, int32_t view) {
    int32_t vp = 1;
    while (vp < view) vp <<= 1;
    return int64_t(vp) * (1 + k) + (int64_t(k) + vp - 1) / vp * vp;
}
__host__ __device__ inline int32_t pv_drain_class(int32_t k, int32_t view, int32_t lds, int32_t wide) {
    const int64_t need = pv_drain_need(k, view);
    if (view < 8 || k > kDrainStage || need > lds) return kDrainHub;
    if (wide < 1 && need <= kDrainCap0) return 0;
    if (wide < 2 && need <= 4096) return 1;
    if (wide < 3 && need <= 8192) return 2;
    return need <= kDrainLdsMax ? 3 : kDrainHub;
}
constexpr int kPvProfPhases = 16;   // per (slot, k): phases 0..14, rows sampled

struct PviewReceiptArgs {
    const int32_t *off;          // [rows + 1] receiver CSR
    const int32_t *csr_src;      // sender ids
    const int32_t *csr_slot;     // row mode: sender rows (null: local row = src - row0)
    int32_t rows, row0, inbox, tick, max_segment;
    int32_t *rc_info, *rc_src, *rc_slot;
    int32_t *kcount, *order;     // k-bucketed row order for the tick kernel (or null)
    int32_t *err;
    int32_t drain;               // inbox 0: rows sent more than kPvMaxInbox messages go to
    int32_t *long_list;          // long_list (by pv_drain_class), not into the buckets
    int32_t view, drain_lds, drain_wide;
};

hipError_t launch_pview_init(const PviewTickArgs &a, hipStream_t st);
hipError_t launch_pview_receipt(const PviewReceiptArgs &a, hipStream_t st);
// tick kernel, then the send kernel (peers, drops) and the digest reduction
hipError_t launch_pview_tick(const PviewTickArgs &a, hipStream_t st);
// drain-all rows (a.drain): launched by launch_pview_tick after the tick kernels
// parts: 1 the LDS classes, 2 the hub kernel, 3 both
hipError_t launch_pview_drain(const PviewTickArgs &a, hipStream_t st, int parts = 3);
// receiver CSR of one shard from the send kernel's positions: csr_src[off[d] + pos] = sender
hipError_t launch_pview_scatter(const int32_t *out_dst, const int32_t *out_pos, int64_t slots,
                                int32_t fanout, const int32_t *off, int32_t *csr_src, hipStream_t st);

}  // namespace gsp
