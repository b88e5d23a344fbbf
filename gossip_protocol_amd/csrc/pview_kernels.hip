// gossip_protocol_amd/csrc/pview_kernels.hip -- PARTIAL-VIEW tick kernels for gfx950.
//
// pview_receipt_kernel (one lane per receiver row): reads the row's CSR segment and keeps its
//   K smallest senders in ascending order (the canonical receipt order; the rest is inbox
//   overflow) as a fixed 8-slot record, so the tick kernel reaches the sender views after a
//   single dependent load instead of three (offsets -> CSR -> rows).
// pview_tick_split_kernel (the default form; rows bucketed by k, the number of messages a row
//   merges, heavy rows first): k = 6, 7 as 256-lane rows in 20 KB of LDS, k = 5 / k = 4 as
//   128-lane rows merged in place (one key buffer, 11.3 / 9.8 KB, PvSharedIP), k <= 3 as
//   128-lane rows in 10 KB; k = 0 rows of the plain protocol skip steps 2-5 (pv_own_only).
//   Each range's grid is its bucket size, read back behind an event after the receipt kernel.
//   pview_tick_kernel is the one-kernel form (GSP_TEST_PV_SPLIT=0: one 256-lane workgroup per row,
//   any k).  The row body:
//   1. loads: the own view is requested first; the receipt record is read by every wave
//      (no barrier) and the k sender views follow, one coalesced 2 KB row each;
//   2. keys: each view is a sorted block of 256 slots of 32-bit keys id << 11 | source << 8
//      | slot (source 0 = own view, j = the payload of message j; the 16-bit value
//      hb << 5 | ts5 stays behind in vals[source][slot]), so equal ids sort in message order;
//   3. union: a tree of merge-path merges (one co-rank binary search per lane per level, then
//      a register merge of the lane's kBlocks outputs): 256 -> 512 -> 1024 -> 2048 keys;
//   4. fold, in registers: each lane walks its kBlocks keys once, folding MP1Node::
//      recvCallBack's rules over every id run whose first key it holds (own entry, then for
//      j = 1..k the sender event of message j and payload entry j; MP1Node.cpp:234-301) and
//      the TREMOVE test (MP1Node.cpp:339-348); a run that continues into the next lane's
//      keys is finished from LDS.  A sender found in no list becomes a new (1, t) entry
//      ("orphan"); the lane whose id bracket holds it is the one that would hold its key,
//      so found / not found is decided locally;
//   5. survivors compacted in id order (one block scan); eviction to V by (age, -hb, id) with
//      one histogram over (age, hb) bins, an exact hb histogram only for a boundary in an
//      age's last bin, and an id-order tie prefix, resolved by a single packed block scan over
//      the lanes' survivors (kept in registers);
//   6. the new sorted view is written back (2 KB, coalesced); the row's digest counts go to a
//      per-row record (no global atomics), summed by pview_digest_kernel.
// pview_send_kernel (one lane per row): Philox rank-select peers over the new view, the drop
//   draw, and each message's slot in its receiver's CSR segment (the deg atomic's return), so
//   pview_scatter_kernel builds the next tick's receiver CSR without atomics.
// HBM bytes per node-round: 2 * V * 8 (own view read + write) + k * V * 8 (sender views).
#include <algorithm>
#include <type_traits>


#include "join_kernels.hpp"
#include "philox.hpp"
#include "pview_kernels.hpp"
#include "pview_rules.hpp"
#include "scale_kernels.hpp"
#include "wave_ops.hpp"

namespace gsp {
namespace {

constexpr int kSlots = kPvMaxView;                    // slots per source block
constexpr int kMaxBlocks = kPvMaxInbox + 1;           // own view + K sender views
constexpr int kMaxKeys = kSlots * kMaxBlocks;         // 2048
constexpr uint32_t kKeyMax = 0xFFFFFFFFu;             // id field 2^21 - 1: above every node id
constexpr uint32_t kNoId = 0xFFFFFFFFu;
static_assert(kMaxBlocks == 8, "the merge tree assumes 8 blocks of 256 keys");

// threadIdx.x as a value the compiler cannot see through: an opaque copy per use keeps the
// lane-position values derived from it (slot offsets, LDS addresses) short-lived temporaries
// instead of registers held across the row body (round 4: the looping overflow kernel spilled
// without it; kept since, as the measured code).  Its range [0, NT) is restated, so loops
// over a lane's slots still unroll.
template <int NT>
__device__ __forceinline__ int32_t pv_tid() {
    int32_t t = int32_t(threadIdx.x);
    asm volatile("" : "+v"(t));
    __builtin_assume(t >= 0 && t < NT);
    return t;
}

__device__ inline uint32_t key_id(uint32_t k) { return k >> 11; }
__device__ inline uint32_t key_src(uint32_t k) { return (k >> 8) & 7u; }
__device__ inline uint32_t key_slot(uint32_t k) { return k & 255u; }

// The row's barrier: a workgroup barrier for rows of several waves; for a one-wave row (NT =
// 64) only a wavefront-scope fence, which keeps the compiler from moving LDS accesses across
// it -- one wave's LDS operations execute in order, so no instruction is needed.
template <int NT>
__device__ __forceinline__ void pv_sync() {
    if constexpr (NT == 64) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    else __syncthreads();
}

// exclusive block scan over the NT lanes of a row; *total = sum of all lanes.  One barrier:
// the caller alternates between two s_wave buffers, so a buffer is rewritten only after a
// later scan's barrier has retired every read of it.  A one-wave row needs neither.
template <int NT = kPvBlock>
__device__ inline uint32_t block_scan(uint32_t v, uint32_t *total, uint32_t *s_wave) {
    const int32_t lane = pv_tid<NT>() & 63, wave = pv_tid<NT>() >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if constexpr (NT == 64) {
        *total = uint32_t(__builtin_amdgcn_readlane(int32_t(incl), 63));
        return incl - v;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int q = 0; q < NT / 64; ++q) {
        const uint32_t x = s_wave[q];
        before += q < wave ? x : 0u;
        all += x;
    }
    *total = all;
    return incl - v + before;
}

// N consecutive words at p: 16-B accesses when N % 4 == 0, 8-B when N % 2 == 0 (p is then
// 8-B aligned: word offset lane * N), else single words
template <int N>
__device__ inline void lds_store(uint32_t *p, const uint32_t (&v)[N]) {
    if constexpr (N % 4 == 0) {
#pragma unroll
        for (int i = 0; i < N; i += 4)
            *reinterpret_cast<uint4 *>(p + i) = make_uint4(v[i], v[i + 1], v[i + 2], v[i + 3]);
    } else if constexpr (N % 2 == 0) {
#pragma unroll
        for (int i = 0; i < N; i += 2) *reinterpret_cast<uint2 *>(p + i) = make_uint2(v[i], v[i + 1]);
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) p[i] = v[i];
    }
}

template <int N>
__device__ inline void lds_load(const uint32_t *p, uint32_t (&v)[N]) {
    if constexpr (N % 4 == 0) {
#pragma unroll
        for (int i = 0; i < N; i += 4) {
            const uint4 x = *reinterpret_cast<const uint4 *>(p + i);
            v[i] = x.x; v[i + 1] = x.y; v[i + 2] = x.z; v[i + 3] = x.w;
        }
    } else if constexpr (N % 2 == 0) {
#pragma unroll
        for (int i = 0; i < N; i += 2) {
            const uint2 x = *reinterpret_cast<const uint2 *>(p + i);
            v[i] = x.x; v[i + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = p[i];
    }
}

// LDS of one row: kKeys = 2048 (up to 8 sources, 20 KB: 8 rows per CU) or 1024 (up to 4
// sources, 10 KB: 16 rows of 128 lanes per CU).  keys[cur] (the sorted union C) is dead once
// the fold is done and then holds: the kept ids W [0, 256), the kept values (u16) at word
// 512, and before them the exact hb histogram of an e >= 31 boundary bin (2048 u16 bins,
// 1024 words at kHist; consumed before the scan that precedes the W writes).  keys[cur ^ 1]
// (the last merge level's source) is dead after the tree and holds the (age, hb) eviction
// bins (1024 u16 counters, words [512, 1024)), the block-scan buffers (8 words at kScan) and,
// when no eviction is needed, the survivor ids U (words [0, 256)).
// kKeys = 512 (up to 2 sources, one-wave rows only, 5 KB: 32 rows per CU): the bins take all
// of keys[cur ^ 1], the kept values follow the kept ids at word 256 of keys[cur], the exact
// hb histogram spans both halves (one wave: the bins are read before it is zeroed), and
// block scans need no buffer.
// Accessors (both layouts): kb(i) merge buffer i, bins / scanbuf the eviction histogram and
// block-scan words after the tree, pre() block-scan words before it, uids the survivor ids
// when nothing is evicted, wids / wvals the kept view, hist the exact hb histogram.
template <int kKeys>
struct alignas(16) PvShared {
    static_assert(kKeys == 512 || (kKeys >= 1024 && kKeys <= 2048 && kKeys % 256 == 0),
                  "2 (one-wave rows) or 4 to 8 sources of 256 keys");
    static constexpr bool kInPlace = false;
    static constexpr int kHist = kKeys == 512 ? 0 : kKeys - 1024,
                         kScan = kKeys == 512 ? 0 : kKeys > 1024 ? kKeys - 8 : 504,
                         kWValWord = kKeys == 512 ? 256 : 512, kBinWord = kKeys == 512 ? 0 : 512;
    uint32_t keys[2][kKeys];             // merge ping-pong; then the regions above
    uint16_t vals[kKeys];                // values by (source, slot); then survivor values
    __device__ uint32_t *hist(int cur) { return kKeys == 512 ? &keys[0][0] : keys[cur] + kHist; }
    __device__ uint32_t *kb(int i) { return keys[i]; }
    __device__ const uint32_t *base() const { return &keys[0][0]; }
    __device__ uint32_t *bins(int cur) { return keys[cur ^ 1] + kBinWord; }
    __device__ uint32_t *scanbuf(int cur) { return keys[cur ^ 1] + kScan; }
    __device__ uint32_t *pre() { return keys[1]; }
    __device__ uint32_t *uids(int cur) { return keys[cur ^ 1]; }
    __device__ uint32_t *wids(int cur) { return keys[cur]; }
    __device__ uint16_t *wvals(int cur) { return reinterpret_cast<uint16_t *>(keys[cur] + kWValWord); }
};

// One merge buffer, merged in place (a tree level reads its inputs into registers, then a
// barrier, then writes): 4 B + 2 B per key + 2 KB of bins and scan words -- 8.3 / 9.8 / 11.3 /
// 14.4 KB for 4 / 5 / 6 / 8 sources instead of 10 / 12.5 / 15 / 20 KB, so the rows merging 4
// or more messages fit more rows per CU, for one more barrier per tree level.  After the fold
// the key buffer holds the kept view (ids [0, 256), values at word 512) and, before them, the
// exact hb histogram (1024 words at kKeys - 1024).
template <int kKeys>
struct alignas(16) PvSharedIP {
    static_assert(kKeys >= 1024 && kKeys <= 2048 && kKeys % 256 == 0, "4 to 8 sources of 256 keys");
    static constexpr bool kInPlace = true;
    uint32_t keys[kKeys];
    uint16_t vals[kKeys];
    uint32_t aux[512 + 16];              // eviction bins (1024 u16), then 16 block-scan words
    __device__ uint32_t *hist(int) { return keys + (kKeys - 1024); }
    __device__ uint32_t *kb(int) { return keys; }
    __device__ const uint32_t *base() const { return keys; }
    __device__ uint32_t *bins(int) { return aux; }
    __device__ uint32_t *scanbuf(int) { return aux + 512; }
    __device__ uint32_t *pre() { return aux; }
    __device__ uint32_t *uids(int) { return keys; }
    __device__ uint32_t *wids(int) { return keys; }
    __device__ uint16_t *wvals(int) { return reinterpret_cast<uint16_t *>(keys + 512); }
};

template <class Sh>
__device__ inline int32_t lds_word(const Sh &sh, const uint32_t *p) {
    return int32_t(p - sh.base());
}
template <class Sh>
__device__ inline int32_t lds_half(const Sh &sh, const void *p) {
    return int32_t(reinterpret_cast<const uint16_t *>(p) - reinterpret_cast<const uint16_t *>(&sh));
}

// Diagnostics (GSP_PV_PROFILE=1): thread 0 of every 16th row adds the cycles since the last
// mark to prof[slot][k][phase] (phase kPvProfPhases - 1 counts the sampled rows); a scalar
// branch on a kernel argument when off.
struct PvMark {
    unsigned long long *out = nullptr;
    uint64_t last = 0;
    __device__ __forceinline__ void init(unsigned long long *prof, int32_t k) {
        if (prof && threadIdx.x == 0 && (blockIdx.x & 15u) == 0) {
            out = prof + ((blockIdx.x >> 4 & 63u) * 16 + uint32_t(k & 7)) * kPvProfPhases;
            atomicAdd(out + kPvProfPhases - 1, 1ull);
            last = clock64();
        }
    }
    __device__ __forceinline__ void mark(int phase) {
        if (out) {
            const uint64_t now = clock64();
            atomicAdd(out + phase, (unsigned long long)(now - last));
            last = now;
        }
    }
};

// The final view: ids and values as LDS offsets (words of keys[][], u16 units of the whole
// PvShared) -- plain integers, so the row's state never leaves registers.
struct RowOut {
    int32_t ids_off, vals_off;
    int32_t len;
    uint32_t joins, removes, evicts, merged;
    uint32_t hsum;                // sum of g(x) over the lane's events (pv_hash)
    bool written;                 // the view is already in HBM (pv_own_only)
};

// Steps 2-5 for a row with k <= kBlocks - 1 merged messages (kBlocks = 1, 2, 3, 4, 6 or 8).
// ent0: this lane's slot of the own view; ssrc/sslot: the receipt record (wave-uniform).
// kExt: the protocol extensions compiled in, a bit mask -- kExtPol: TFAIL payload filter, JOINREP (jrep:
// message 1 is a JOINREP whose payload is node 0's view cut to the bounded introducer list),
// SWIM (pcol / pok: the probe of t - 1, target id or kNoId, answered) and the event stream;
// the plain protocol (config 5) runs the kernel without them.
constexpr int kExtEv = 1, kExtPol = 2;   // kExt bits: event stream; TFAIL / SWIM / JOINREP
constexpr int kExtRot = 4;               // eviction ties by the rotated id (evict_order 1)
template <int kBlocks, int kExt, int NT, class Sh>
__device__ __forceinline__ void pv_merge_row(const PviewTickArgs &a, Sh &sh, int32_t r,
                                             int32_t k, const uint64_t (&ent0)[kSlots / NT],
                                             int32_t my_slot, const uint32_t (&ssrc)[kPvMaxInbox],
                                             bool jrep, uint32_t pcol, bool pok, RowOut &ro,
                                             PvMark &pm) {
    constexpr int SL = kSlots / NT;                      // slots of each source per lane
    constexpr int Q = kBlocks * SL;                      // keys per lane
    constexpr int kJ = kBlocks - 1;                      // k <= kJ messages in this variant
    constexpr int P = kBlocks * kSlots;
    static_assert(P <= int(sizeof(sh.vals) / 2), "row LDS too small for this variant");
    const int32_t tid = pv_tid<NT>();
    const int32_t V = a.view;
    const uint32_t t = uint32_t(a.tick), t5 = t & 31u, tr = uint32_t(a.tremove);
    const uint32_t th0 = t + uint32_t(a.h0);
    const int32_t Pe = (k + 1) * kSlots;                // keys that can be real
    const uint32_t S_join = uint32_t(pv_seed(1, t, uint32_t(r))), S_remove = uint32_t(pv_seed(2, t, uint32_t(r))),
                   S_evict = uint32_t(pv_seed(3, t, uint32_t(r)));

    // ---- 2. keys: one sorted block of 256 slots per source ------------------------------------
    // block 0 = the own view (loaded with the record), block m = message m's payload: the
    // sender's view (one coalesced 2 KB load) cut to what it gossiped at t - 1 (TFAIL), or for
    // a JOINREP node 0's view cut to the Philox-chosen members (bounded introducer list).
    // Lane tid holds slots [tid * SL, tid * SL + SL) of every block.
    const uint32_t tf = uint32_t(a.tfail), t5m1 = (t - 1u) & 31u;
    auto gossiped = [&](uint64_t v) {      // listed, and not suspected when sent at t - 1
        return v != kPvEmpty && (tf == 0 || ((t5m1 - uint32_t(v)) & 31u) < tf);
    };
    uint64_t ent[kBlocks][SL];
#pragma unroll
    for (int i = 0; i < SL; ++i) ent[0][i] = ent0[i];
#pragma unroll
    for (int m = 1; m < kBlocks; ++m) {
#pragma unroll
        for (int i = 0; i < SL; ++i) ent[m][i] = kPvEmpty;
        if (m <= k) {
            const int32_t sl = __builtin_amdgcn_readlane(my_slot, m - 1);
            const uint64_t *row = (m == 1 && jrep) ? a.intro
                                  : sl >= 0 ? a.prev + int64_t(sl) * V : a.remote + int64_t(-sl - 1) * V;
#pragma unroll
            for (int i = 0; i < SL; ++i) {
                const int32_t slot = tid * SL + i;
                if (slot < V) {
                    ent[m][i] = __builtin_nontemporal_load(row + slot);
                    if ((kExt & kExtPol) && !gossiped(ent[m][i])) ent[m][i] = kPvEmpty;
                }
            }
        }
    }
    if constexpr (kBlocks > 1 && (kExt & kExtPol)) if (jrep) {   // block-uniform: node 0's gossiped members
        uint32_t gl = 0;
#pragma unroll
        for (int i = 0; i < SL; ++i) gl += ent[1][i] != kPvEmpty ? 1u : 0u;
        uint32_t cnt0 = 0;
        uint32_t rank = block_scan<NT>(gl, &cnt0, sh.pre());     // free before the tree
        const int32_t B = a.intro_list < int32_t(cnt0) ? a.intro_list : int32_t(cnt0);
        uint64_t cm[4];
        pv_intro_mask(a.seed, t - 1u, uint32_t(r), int32_t(cnt0), B, cm);
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            const bool g = ent[1][i] != kPvEmpty;
            const uint32_t w = rank >> 6;
            const uint64_t word = w == 0 ? cm[0] : w == 1 ? cm[1] : w == 2 ? cm[2] : cm[3];
            if (!(g && ((word >> (rank & 63u)) & 1ull))) ent[1][i] = kPvEmpty;
            rank += g ? 1u : 0u;
        }
    }
    // A TFAIL- or introducer-filtered payload has holes: its keys are compacted to the front
    // of the block (the tree merges sorted blocks).  Block-uniform; one scan per message.
    int32_t kpos[kBlocks][SL];                           // slot of this lane's keys
    uint32_t kpad = 0;                                   // bit m * SL + i: slot i is padding
#pragma unroll
    for (int m = 0; m < kBlocks; ++m) {
#pragma unroll
        for (int i = 0; i < SL; ++i) kpos[m][i] = tid * SL + i;
        if ((kExt & kExtPol) && m >= 1 && (tf != 0 || (m == 1 && jrep)) && m <= k) {
            uint32_t cl = 0;
#pragma unroll
            for (int i = 0; i < SL; ++i) cl += ent[m][i] != kPvEmpty ? 1u : 0u;
            uint32_t cnt = 0;
            uint32_t pos = block_scan<NT>(cl, &cnt, sh.pre() + 16 + 8 * (m & 1));
#pragma unroll
            for (int i = 0; i < SL; ++i) {
                const bool ok = ent[m][i] != kPvEmpty;
                kpos[m][i] = ok ? int32_t(pos) : -1;
                pos += ok ? 1u : 0u;
                kpad |= uint32_t(tid * SL + i >= int32_t(cnt)) << (m * SL + i);
            }
        }
    }
    uint32_t merged = 0;                                 // payload entries (MP1Node.cpp:245 trips)
#pragma unroll
    for (int m = 0; m < kBlocks; ++m) {
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            const int32_t slot = tid * SL + i;
            const bool ok = ent[m][i] != kPvEmpty;
            merged += (m >= 1 && ok) ? 1u : 0u;
            if ((kExt & kExtPol) && ((kpad >> (m * SL + i)) & 1u)) sh.kb(0)[m * kSlots + slot] = kKeyMax;
            if (!(kExt & kExtPol) || kpos[m][i] >= 0)
                sh.kb(0)[m * kSlots + kpos[m][i]] =
                    ok ? (uint32_t(ent[m][i] >> 32) << 11) | (uint32_t(m) << 8) | uint32_t(slot) : kKeyMax;
            sh.vals[m * kSlots + slot] = uint16_t(ent[m][i]);
            if (!Sh::kInPlace && m > k) sh.kb(1)[m * kSlots + slot] = kKeyMax;   // padding for the ping-pong
        }
    }
    pv_sync<NT>();
    pm.mark(1);

    // ---- 3. merge-path tree: sorted union of every source, ties in message order ------------
    // Level s merges neighbouring segments of s keys (the last one of a level may be shorter
    // or alone when kBlocks is not a power of two).  The tree hands out Qt = 2^ceil(log2
    // kBlocks) * SL outputs per lane, so a lane's outputs never straddle two merges (P / Qt
    // lanes work).
    constexpr int Qt = (kBlocks <= 2 ? kBlocks : kBlocks <= 4 ? 4 : 8) * SL;
    constexpr bool kPow2 = (kBlocks & (kBlocks - 1)) == 0;
    const int32_t begt = tid * Qt;
    int cur = 0;
#pragma unroll
    for (int s = kSlots; s < P; s <<= 1) {
        uint32_t outk[Qt];
        const bool act = begt < Pe;
        if (act) {
            const uint32_t *X = sh.kb(cur);
            const int32_t b = begt / (2 * s), o = begt - b * 2 * s;
            const uint32_t *A = X + b * 2 * s, *B = A + s;
            int32_t sa = s, sb = s;
            if constexpr (!kPow2) {
                const int32_t rest = P - b * 2 * s;
                sa = rest < s ? rest : s;
                sb = rest - s < s ? (rest > s ? rest - s : 0) : s;
            }
            int32_t lo = o > sb ? o - sb : 0, hi = o < sa ? o : sa;
            while (lo < hi) {                                  // co-rank of output o
                const int32_t mid = (lo + hi) >> 1;
                if (A[mid] < B[o - mid - 1]) lo = mid + 1; else hi = mid;
            }
            int32_t i = lo, j = o - lo;
            uint32_t va = i < sa ? A[i] : kKeyMax, vb = j < sb ? B[j] : kKeyMax;
#pragma unroll
            for (int e = 0; e < Qt; ++e) {
                const bool ta = va <= vb;                      // equal only for padding
                outk[e] = ta ? va : vb;
                i += ta ? 1 : 0;
                j += ta ? 0 : 1;
                const int32_t ii = ta ? i : j;
                const uint32_t nv = ii < (ta ? sa : sb) ? (ta ? A : B)[ii] : kKeyMax;
                va = ta ? nv : va;
                vb = ta ? vb : nv;
            }
            if constexpr (!Sh::kInPlace) lds_store<Qt>(sh.kb(cur ^ 1) + begt, outk);
        }
        if constexpr (Sh::kInPlace) {            // one buffer: every input of the level is read
            pv_sync<NT>();                       // before any output is written over it
            if (act) lds_store<Qt>(sh.kb(0) + begt, outk);
        }
        pv_sync<NT>();
        if constexpr (!Sh::kInPlace) cur ^= 1;
        pm.mark(s == kSlots ? 12 : s == 2 * kSlots ? 13 : 14);
    }
    const int32_t beg = tid * Q;                               // the fold's Q keys per lane
    const uint32_t *C = sh.kb(cur);
    // the eviction histogram over (age, hb) bins (1024 u16 counters) and the block-scan words:
    // ping-pong layout, in keys[cur ^ 1] (the last level's source, dead after the tree) at
    // words [512, 1024) and Sh::kScan; in-place layout, in their own words
    uint32_t *const bins = sh.bins(cur);
    uint32_t *const scan_buf = sh.scanbuf(cur);
#pragma unroll
    for (int i = tid; i < 256; i += NT) reinterpret_cast<uint2 *>(bins)[i] = make_uint2(0u, 0u);

    pm.mark(2);
    // ---- 4. fold every id run that starts in this lane, in registers ------------------------
    uint32_t ck[Q], vv[Q];
    lds_load<Q>(C + beg, ck);
    const uint32_t prev_key = tid > 0 ? C[beg - 1] : 0u;
    const uint32_t next_key = beg + Q < P ? C[beg + Q] : kKeyMax;
#pragma unroll
    for (int e = 0; e < Q; ++e)                                // value gathers, all in flight
        vv[e] = ck[e] != kKeyMax ? uint32_t(sh.vals[key_src(ck[e]) * kSlots + key_slot(ck[e])]) : 0u;
    const uint32_t lo_id = tid > 0 ? key_id(prev_key) + 1u : 0u;   // this lane brackets ids
    const uint32_t hi_id = tid < NT - 1 ? key_id(ck[Q - 1]) : kKeyMax;  // [lo_id, hi_id]

    uint32_t res[Q], rid[Q];
    uint32_t nloc = 0, joins = 0, removes = 0, evicts = 0, found_mask = 0;
    uint32_t jmask = 0, rmask = 0;                       // event stream: join / remove keys
    uint32_t hsum = 0;
    // the run being folded: id, value, own-view value, sender event (message index, applied)
    uint32_t ax = kNoId, av = 0, ae0 = 0, ajs = 0;
    bool aown = false, adone = false;
#pragma unroll
    for (int e = 0; e < Q; ++e) {
        res[e] = 0;
        rid[e] = 0;
        const uint32_t key = ck[e];
        if (key == kKeyMax) continue;
        const uint32_t x = key_id(key), src = key_src(key);
        if (x != ax) {                                         // a run starts at key e
            ax = x;
            aown = e > 0 || x >= lo_id;                        // else the previous lane's run
            av = ae0 = 0;
            ajs = 0;
#pragma unroll
            for (int jj = 0; jj < kJ; ++jj) ajs = ssrc[jj] == x ? uint32_t(jj + 1) : ajs;
            adone = false;
            if (aown && ajs) found_mask |= 1u << (ajs - 1);
        }
        if (src == 0) {
            av = ae0 = vv[e];
        } else {
            if (ajs && !adone && ajs < src) { av = pv_event(av, t5); adone = true; }
            av = pv_merge(av, vv[e], t5, tr);
        }
        // does the run end here?
        uint32_t nxt = e + 1 < Q ? ck[e + 1 < Q ? e + 1 : e] : next_key;
        if (e + 1 == Q && nxt != kKeyMax && key_id(nxt) == x) {   // continues into the next lane
            // a run holds at most one key per source: at most kJ more keys, a fixed trip count
            bool go = true;
#pragma unroll
            for (int c2 = 0; c2 < kJ; ++c2) {
                const int32_t pos = beg + Q + c2;
                const uint32_t kk = (go && pos < P) ? C[pos < P ? pos : P - 1] : kKeyMax;
                go = go && kk != kKeyMax && key_id(kk) == x;
                if (go) {
                    const uint32_t s2 = key_src(kk);
                    if (ajs && !adone && ajs < s2) { av = pv_event(av, t5); adone = true; }
                    av = pv_merge(av, sh.vals[s2 * kSlots + key_slot(kk)], t5, tr);
                }
            }
            nxt = kKeyMax;
        }
        if (nxt != kKeyMax && key_id(nxt) == x) continue;
        if (!aown) continue;
        if (ajs && !adone) av = pv_event(av, t5);
        if (x == uint32_t(r) || !av) continue;                  // never list yourself
        if ((kExt & kExtPol) && x == pcol) av = (av & 0xFFE0u) | (pok ? t5 : ((t5 - tr) & 31u));   // SWIM answer
        if (!ae0) { joins++; hsum += pv_hash(S_join, x); if (kExt & kExtEv) jmask |= 1u << e; }
        if (((t5 - av) & 31u) >= tr) {                          // TREMOVE scan
            removes++;
            hsum += pv_hash(S_remove, x);
            if (kExt & kExtEv) rmask |= 1u << e;
            continue;
        }
        res[e] = av;
        rid[e] = x;
        nloc++;
    }
    // orphans: senders in this lane's bracket that no list holds (their key would be here)
    uint32_t adopt = 0;
    int32_t ains[kPvMaxInbox];
#pragma unroll
    for (int jj = 0; jj < kJ; ++jj) {
        ains[jj] = 0;
        const uint32_t x = ssrc[jj];
        if (jj < k && x >= lo_id && x <= hi_id && beg <= Pe && !((found_mask >> jj) & 1u)) {
            int32_t c = 0;
#pragma unroll
            for (int e = 0; e < Q; ++e) c += key_id(ck[e]) < x ? 1 : 0;
            ains[jj] = c;
            adopt |= 1u << jj;
            nloc++;
            joins++;
            hsum += pv_hash(S_join, x);
        }
    }

    if ((kExt & kExtEv) && a.ev.buf) {                   // event stream: joins and removes
        if (!(a.ev.kinds & GSP_EVENTS_JOIN)) jmask = 0;
        if (!(a.ev.kinds & GSP_EVENTS_REMOVE)) rmask = 0;
        const uint32_t amask = (a.ev.kinds & GSP_EVENTS_JOIN) ? adopt : 0u;
        uint64_t p = wave_reserve_events(ev_stripe_count(a.ev),
                                         uint32_t(__popc(jmask) + __popc(rmask) + __popc(amask)));
        unsigned long long *const eb = ev_stripe_buf(a.ev);
        auto put = [&](uint32_t kind, uint32_t x) {
            if (int64_t(p) < a.ev.cap) eb[p] = event_record(kind, t, uint32_t(r), x);
            ++p;
        };
#pragma unroll
        for (int e = 0; e < Q; ++e) {
            if ((jmask >> e) & 1u) put(1u, key_id(ck[e]));
            if ((rmask >> e) & 1u) put(2u, key_id(ck[e]));
        }
#pragma unroll
        for (int jj = 0; jj < kJ; ++jj)
            if ((amask >> jj) & 1u) put(1u, ssrc[jj]);
    }
    pm.mark(3);
    // ---- 5a. survivors (and adopted orphans), compacted in id order -------------------------
    // for_each visits this lane's survivors in id order as (value, id)
    const uint32_t fresh = (1u << 5) | t5;                     // an orphan: (hb 1, ts t)
    // Almost every sender is an orphan (views are tiny next to n), but a lane brackets more
    // than one only rarely: one orphan per lane takes the short path, a wave with any lane
    // holding two or more takes the general one.
    const int32_t n_orph = __popc(adopt);
    uint32_t o_x = 0;
    int32_t o_p = -1;
    if (n_orph == 1) {
#pragma unroll
        for (int jj = 0; jj < kJ; ++jj)
            if ((adopt >> jj) & 1u) { o_x = ssrc[jj]; o_p = ains[jj]; }
    }
    const bool multi = __ballot(n_orph > 1) != 0ull;          // wave-uniform
    // rb[e]: the eviction bin of res[e] (filled on the eviction path, computed once per slot)
    uint32_t rb[Q];
#pragma unroll
    for (int e = 0; e < Q; ++e) rb[e] = 0;
    const uint32_t fresh_bin = pv_bin(fresh, t5, th0);
    auto for_each = [&](auto &&f) {                            // f(value, id, bin)
        if (!multi) {
#pragma unroll
            for (int e = 0; e <= Q; ++e) {
                if (o_p == e) f(fresh, o_x, fresh_bin);
                if (e < Q && res[e]) f(res[e], rid[e], rb[e]);
            }
        } else {
#pragma unroll
            for (int e = 0; e <= Q; ++e) {
#pragma unroll
                for (int jj = 0; jj < kJ; ++jj)
                    if (((adopt >> jj) & 1u) && ains[jj] == e) f(fresh, ssrc[jj], fresh_bin);
                if (e < Q && res[e]) f(res[e], rid[e], rb[e]);
            }
        }
    };
    uint32_t total = 0;
    const uint32_t base = block_scan<NT>(nloc, &total, scan_buf);
    const bool evict = int32_t(total) > V;
    if (!evict) {                                              // the survivors are the view
        uint32_t *Uid = sh.uids(cur);
        uint16_t *Uval = sh.vals;                              // the gathered values are dead
        uint32_t w = base;
        for_each([&](uint32_t v, uint32_t x, uint32_t) {
            Uid[w] = x;
            Uval[w] = uint16_t(v);
            w++;
        });
        ro.ids_off = lds_word(sh, Uid);
        ro.vals_off = lds_half(sh, Uval);
        ro.len = int32_t(total);
    } else {
#pragma unroll
        for (int e = 0; e < Q; ++e) rb[e] = pv_bin(res[e], t5, th0);
        for_each([&](uint32_t, uint32_t, uint32_t b) {
            atomicAdd(&bins[b >> 1], 1u << ((b & 1u) * 16u));
        });
    }

    pm.mark(4);
    // ---- 5b. eviction to V by (age, -hb, id) ------------------------------------------------
    // Order key (age, -hb) as one bin index age * 32 + e, e = h0 + t - age - hb: every entry
    // satisfies hb <= h0 + ts (a heartbeat grows by at most one per tick from h0, and every
    // rule that sets ts = t sets hb <= h0 + t), so e >= 0, and within an age e ascends as hb
    // descends.  Kept: every bin below the boundary bin, then boundary-bin entries in id
    // order.  A boundary bin e < 31 holds one (age, hb); the last bin of an age (e >= 31)
    // can hold several hb values -- then the exact boundary hb comes from an hb histogram.
    if (evict) {
        pv_sync<NT>();                                   // bin histogram complete
        const int32_t lane = tid & 63;
        uint32_t bstar, need, at;
        {   // every wave: lane l sums bins [16 l, 16 l + 16), the lane holding the V-th entry
            // walks its bins
            const uint16_t *b16 = reinterpret_cast<const uint16_t *>(bins);
            const uint4 *bw = reinterpret_cast<const uint4 *>(bins + 8 * lane);
            uint32_t loc = 0;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint4 x = bw[q];
                loc += (x.x & 0xFFFFu) + (x.x >> 16) + (x.y & 0xFFFFu) + (x.y >> 16) +
                       (x.z & 0xFFFFu) + (x.z >> 16) + (x.w & 0xFFFFu) + (x.w >> 16);
            }
            const uint32_t incl = wave_incl_scan(loc);
            const int32_t lb = __builtin_ffsll(__ballot(incl >= uint32_t(V))) - 1;
            const uint32_t before = lane_of(incl - loc, lb);
            const uint32_t c = lane < 16 ? uint32_t(b16[16 * lb + lane]) : 0u;
            const uint32_t ci = wave_incl_scan(c);      // c = 0 beyond lane 15
            const int32_t lh = __builtin_ffsll(__ballot(lane < 16 && before + ci >= uint32_t(V))) - 1;
            bstar = uint32_t(16 * lb + lh);
            at = lane_of(c, lh);
            need = uint32_t(V) - (before + lane_of(ci, lh) - at);   // kept from the bin
        }
        pm.mark(7);
        const bool tie = at > need;
        const uint32_t astar = bstar >> 5;
        uint32_t hstar = th0 - astar - (bstar & 31u), need2 = need;
        if (tie && (bstar & 31u) == 31u) {                               // block-uniform: exact hb boundary
            uint32_t *hist = sh.hist(cur);                 // 2048 hb bins, u16 pairs; C is dead
            for (int32_t i = tid; i < 1024; i += NT) hist[i] = 0;
            pv_sync<NT>();
            for_each([&](uint32_t v, uint32_t, uint32_t b) {
                if (b == bstar)
                    atomicAdd(&hist[(v >> 5) >> 1], 1u << (((v >> 5) & 1u) * 16u));
            });
            pv_sync<NT>();
            // every wave: lane l sums hb bins 2047 - 32l - 31 .. 2047 - 32l (descending lanes),
            // the lane holding the need-th largest walks its bins
            const uint16_t *h16 = reinterpret_cast<const uint16_t *>(hist);
            const uint4 *hw = reinterpret_cast<const uint4 *>(hist + 1024 - 16 * (lane + 1));
            uint32_t loc = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 x = hw[q];
                loc += (x.x & 0xFFFFu) + (x.x >> 16) + (x.y & 0xFFFFu) + (x.y >> 16) +
                       (x.z & 0xFFFFu) + (x.z >> 16) + (x.w & 0xFFFFu) + (x.w >> 16);
            }
            const uint32_t incl = wave_incl_scan(loc);
            const unsigned long long hit = __ballot(incl >= need);
            const int32_t lb = __builtin_ffsll(hit) - 1;
            // lanes 0..31 take the boundary lane's 32 bins (descending hb) and scan them
            const uint32_t before = lane_of(incl - loc, lb);
            const uint32_t c = lane < 32 ? uint32_t(h16[2047 - 32 * lb - lane]) : 0u;
            const uint32_t ci = wave_incl_scan(c);      // c = 0 beyond lane 31
            const unsigned long long hit2 = __ballot(lane < 32 && before + ci >= need);
            const int32_t lh = __builtin_ffsll(hit2) - 1;
            hstar = uint32_t(2047 - 32 * lb - lh);
            need2 = need - before - (lane_of(ci, lh) - lane_of(c, lh));  // kept among ties
        }
        pm.mark(8);
        // one packed scan: ties before this lane (low 16) and plain keeps before it (high 16)
        uint32_t nt = 0, nk = 0, nth = 0;
        // evict_order 1 (kExtRot): the ties are kept in the order of the rotated id (x - m) mod
        // n -- the ties with x >= m in id order, then those below m -- so nth counts the ties
        // at or above m; m = Philox(EVICT; t, r) mod n (oracle/pview_oracle.c pv_rot)
        const uint32_t mrot = (kExt & kExtRot) ? draw_u31(kDomainEvict, a.seed, t, uint32_t(r), 0u, 0u) %
                                                     uint32_t(a.n)
                                               : 0u;
        // ties: the boundary bin's entries with hb == hstar (all of them unless e >= 31);
        // plain keeps: lower bins, and boundary-bin entries with a larger hb or without a tie
        for_each([&](uint32_t v, uint32_t x, uint32_t b) {
            const uint32_t hb = v >> 5;
            const bool is_tie = tie && b == bstar && hb == hstar;
            nt += is_tie ? 1u : 0u;
            if (kExt & kExtRot) nth += (is_tie && x >= mrot) ? 1u : 0u;
            nk += (!is_tie && (b < bstar || (b == bstar && (!tie || hb > hstar)))) ? 1u : 0u;
        });
        pm.mark(9);
        uint32_t sums = 0;
        const uint32_t ex = block_scan<NT>(nt | (nk << 16), &sums, scan_buf + 4);
        pm.mark(10);
        uint32_t tie_before = ex & 0xFFFFu;
        uint32_t ties_kept_before = tie_before < need2 ? tie_before : need2;
        // rotated order: keep_hi of the ties at or above m, keep_lo below it; before this lane
        // in id order come lo_before ties below m, then hi_before at or above it
        uint32_t hi_before = 0, keep_hi = 0, keep_lo = 0;
        if ((kExt & kExtRot) && tie) {                       // block-uniform
            uint32_t A = 0;
            hi_before = block_scan<NT>(nth, &A, scan_buf);   // scan_buf's last reads retired
            keep_hi = need2 < A ? need2 : A;
            keep_lo = need2 - keep_hi;
            const uint32_t lo_before = tie_before - hi_before;
            ties_kept_before = (lo_before < keep_lo ? lo_before : keep_lo) + (hi_before < keep_hi ? hi_before : keep_hi);
        }
        uint32_t w = (ex >> 16) + (tie ? ties_kept_before : 0u);
        uint32_t *Wid = sh.wids(cur);
        uint16_t *Wval = sh.wvals(cur);
        uint64_t evp = 0;                                  // event stream: this lane's evictions
        const bool ev_on = (kExt & kExtEv) && a.ev.buf && (a.ev.kinds & GSP_EVENTS_EVICT);
        if (ev_on) {
            uint32_t kept_t;
            if ((kExt & kExtRot) && tie) {
                const uint32_t lo_before = tie_before - hi_before, ntl = nt - nth;
                const int32_t kl = int32_t(keep_lo) - int32_t(lo_before), kh = int32_t(keep_hi) - int32_t(hi_before);
                kept_t = uint32_t(kl <= 0 ? 0 : (kl >= int32_t(ntl) ? int32_t(ntl) : kl)) +
                         uint32_t(kh <= 0 ? 0 : (kh >= int32_t(nth) ? int32_t(nth) : kh));
            } else {
                const int32_t tk = int32_t(need2) - int32_t(tie_before);
                kept_t = uint32_t(tk <= 0 ? 0 : (tk >= int32_t(nt) ? int32_t(nt) : tk));
            }
            evp = wave_reserve_events(ev_stripe_count(a.ev), nloc - (nk + kept_t));
        }
        uint32_t lo_rank = tie_before - hi_before;           // kExtRot: ranks among the ties
        for_each([&](uint32_t v, uint32_t x, uint32_t b) {
            const uint32_t hb = v >> 5;
            bool keep = b < bstar || (b == bstar && (!tie || hb > hstar));
            if (tie && b == bstar && hb == hstar) {
                if (kExt & kExtRot) keep = x >= mrot ? hi_before++ < keep_hi : lo_rank++ < keep_lo;
                else keep = tie_before++ < need2;
            }
            if (keep) {
                Wid[w] = x;
                Wval[w] = uint16_t(v);
                w++;
            } else {
                evicts++;
                hsum += pv_hash(S_evict, x);
                if (ev_on) {
                    if (int64_t(evp) < a.ev.cap) ev_stripe_buf(a.ev)[evp] = event_record(3u, t, uint32_t(r), x);
                    ++evp;
                }
            }
        });
        ro.ids_off = lds_word(sh, Wid);
        ro.vals_off = lds_half(sh, Wval);
        ro.len = V;
        pm.mark(11);
    }
    ro.joins = joins;
    ro.removes = removes;
    ro.evicts = evicts;
    ro.merged = merged;
    ro.hsum = hsum;
    pv_sync<NT>();
}

// ---- 6. write the view and the row's digest record (peers: pview_send_kernel) -------------
// rowdig[lr][wave][4]: w0 = merges | delivered << 32 | sent << 40 | dropped << 48 | round << 56,
// w1 = joins | removes << 16 | evicts << 32 | overflow << 48, w2 = event hash, w3 = 0; each
// wave writes its own partial record (no barrier; a 128-lane row's two waves also zero the
// records of waves 2 and 3); sent / dropped come from the send kernel.
template <int NT, class Sh>
__device__ __forceinline__ void pv_finish(const PviewTickArgs &a, Sh &sh, int32_t lr,
                                          int32_t k, int32_t k_all, bool init, const RowOut &ro) {
    const int32_t tid = pv_tid<NT>(), lane = tid & 63, wave = tid >> 6;
    const int32_t V = a.view, len = ro.len;
    const uint32_t t = uint32_t(a.tick);
    const uint32_t *ids = sh.base() + ro.ids_off;
    const uint16_t *vals = reinterpret_cast<const uint16_t *>(&sh) + ro.vals_off;
    uint64_t *out = a.cur + int64_t(lr) * V;
    if (!ro.written)
        for (int32_t i = tid; i < V; i += NT)
            __builtin_nontemporal_store(
                i < len ? (uint64_t(ids[i]) << 32) | uint64_t(vals[i]) : kPvEmpty, out + i);
    if (init) {
        if (tid == 0) a.len_cur[lr] = len;
        return;
    }
    // per-lane counts are <= 15, so two 16-bit fields per word cannot carry in a wave sum
    const uint32_t jrs = wave_sum32(ro.joins | (ro.removes << 16));
    const uint32_t evm = wave_sum32(ro.evicts | (ro.merged << 16));
    const uint64_t jr = jrs;                          // joins | removes << 16
    const uint64_t ev = evm & 0xFFFFu;
    uint64_t mg = evm >> 16;
    // the wave's event hash: its g(x) sum plus its event counts times the row's kind seeds
    const uint32_t r = uint32_t(a.row0 + lr);
    const uint64_t h = wave_sum64(ro.hsum) + uint64_t(jrs & 0xFFFFu) * pv_seed(1, t, r) +
                       uint64_t(jrs >> 16) * pv_seed(2, t, r) + uint64_t(ev) * pv_seed(3, t, r);
    if (lane == 0) {
        uint64_t w0 = mg, w1 = jr | (ev << 32);
        if (wave == 0) {
            a.len_cur[lr] = len;
            // alive at every tick since it started (pre-joined: ticks 1..t)
            const int32_t st = a.start_tick ? a.start_tick[a.row0 + lr] : 0;
            a.own_hb[lr] = int32_t(t) - (st > 0 ? st - 1 : 0);
            w0 += uint64_t(k) | (uint64_t(k) << 32) | (1ull << 56);
            w1 |= uint64_t(k_all - k) << 48;
        }
        ulonglong2 *rec = reinterpret_cast<ulonglong2 *>(a.rowdig + (int64_t(lr) * 4 + wave) * 4);
        rec[0] = make_ulonglong2(w0, w1);
        if (wave == 0) rec[1].x = h;                  // w3 belongs to the send kernel
        else rec[1] = make_ulonglong2(h, 0ull);
#pragma unroll
        for (int w = NT / 64; w < 4; w += NT / 64) {     // the records of waves this row lacks
            ulonglong2 *z = reinterpret_cast<ulonglong2 *>(a.rowdig + (int64_t(lr) * 4 + wave + w) * 4);
            z[0] = z[1] = make_ulonglong2(0ull, 0ull);
        }
    }
}

// A row that merges no message (k = 0, ~30 % of config 5's rows), plain protocol: its view is
// its own view minus the entries TREMOVE drops (MP1Node.cpp:339-348) -- no union, no fold
// state, nothing to evict -- so the kept entries go from registers straight to HBM in id order
// (one block scan for their positions), byte for byte the entries they were.
template <int NT, class Sh>
__device__ __forceinline__ void pv_own_only(const PviewTickArgs &a, Sh &sh, int32_t r, int32_t lr,
                                            const uint64_t (&ent0)[kSlots / NT], RowOut &ro) {
    constexpr int SL = kSlots / NT;
    const int32_t tid = pv_tid<NT>();
    const int32_t V = a.view;
    const uint32_t t = uint32_t(a.tick), t5 = t & 31u, tr = uint32_t(a.tremove);
    const uint32_t S_remove = uint32_t(pv_seed(2, t, uint32_t(r)));
    uint32_t keep = 0, removes = 0;
    uint32_t hsum = 0;
    bool kp[SL];
#pragma unroll
    for (int i = 0; i < SL; ++i) {
        const uint64_t e = ent0[i];
        const uint32_t x = uint32_t(e >> 32), v = uint32_t(e) & 0xFFFFu;
        const bool skip = e == kPvEmpty || x == uint32_t(r) || v == 0u;   // never list yourself
        const bool rem = !skip && ((t5 - v) & 31u) >= tr;
        kp[i] = !skip && !rem;
        keep += kp[i] ? 1u : 0u;
        removes += rem ? 1u : 0u;
        if (rem) hsum += pv_hash(S_remove, x);
    }
    uint32_t total = 0;
    uint32_t w = block_scan<NT>(keep, &total, sh.pre());
    uint64_t *out = a.cur + int64_t(lr) * V;
#pragma unroll
    for (int i = 0; i < SL; ++i)
        if (kp[i]) __builtin_nontemporal_store(ent0[i], out + w++);
    for (int32_t i = int32_t(total) + tid; i < V; i += NT) __builtin_nontemporal_store(kPvEmpty, out + i);
    ro.len = int32_t(total);
    ro.removes = removes;
    ro.hsum = hsum;
    ro.written = true;
}

// workgroup-order index b -> row: b itself, or the b-th row of the k-descending order of
// the buckets k in [kQlo, kQhi]
template <int kQlo = 0, int kQhi = 7>
__device__ __forceinline__ int32_t pv_row_of(const PviewTickArgs &a, int32_t b) {
    if (!a.order) return b;
    int32_t q = kQhi;
    for (; q > kQlo; --q) {
        const int32_t c = a.kcount[q];
        if (b < c) break;
        b -= c;
    }
    return a.order[int64_t(q) * a.rows + b];
}

// One non-init row: the own view slot and the receipt record are requested first (their
// latencies overlap), then merge, ops, eviction, view write and digest record.
// NT lanes per row; the row's k (merged messages) lies in [kQlo, kQhi] -- only those
// variants are compiled in.
template <int kExt, int NT, int kQlo, int kQhi, class Sh>
__device__ __forceinline__ void pv_row(const PviewTickArgs &a, Sh &sh, int32_t lr) {
    constexpr int SL = kSlots / NT;
    const int32_t tid = pv_tid<NT>(), lane = tid & 63;
    const int32_t r = a.row0 + lr;
    // drain-all: a row sent more than kPvMaxInbox messages is pview_drain_kernel's (only the
    // one-kernel form without row order reaches it here)
    if (a.drain && (a.rc_info[lr] >> 3) > kPvMaxInbox) return;
    if (a.rows_run && tid == 0) atomicAdd(a.rows_run, 1);     // tests: each row exactly once
    uint64_t ent0[SL];
#pragma unroll
    for (int i = 0; i < SL; ++i)
        ent0[i] = tid * SL + i < a.view ? __builtin_nontemporal_load(a.prev + int64_t(lr) * a.view + tid * SL + i)
                                        : kPvEmpty;
    const int32_t info_v = a.rc_info[lr];
    const int32_t my_src = lane < 8 ? a.rc_src[int64_t(lr) * 8 + lane] : 0;
    const int32_t my_slot = lane < 8 ? a.rc_slot[int64_t(lr) * 8 + lane] : 0;
    // crashed (no recv, no ops, no send), not started yet, or a capacity error stopped the job
    if (a.tick > a.fail_tick[r] || (a.start_tick && a.tick < a.start_tick[r]) || *a.err) {
        if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
        return;
    }
    PvMark pm;
    RowOut ro{};
    const int32_t info = __builtin_amdgcn_readfirstlane(info_v);
    const int32_t k = info & 7, k_all = info >> 3;
    pm.init(a.prof, k);
    // a JOINREP (sender kJoinRepSrc) sorts first; its sender event is node 0's
    const bool jrep = (kExt & kExtPol) && k > 0 && __builtin_amdgcn_readfirstlane(my_src) == kJoinRepSrc;
    uint32_t ssrc[kPvMaxInbox];
#pragma unroll
    for (int jj = 0; jj < kPvMaxInbox; ++jj)
        ssrc[jj] = jj < k ? uint32_t(__builtin_amdgcn_readlane(my_src, jj)) : kNoId;
    if (jrep) ssrc[0] = 0u;
    // SWIM: the probe this row sent at t - 1, answered iff its target is alive now and one of
    // the swim paths survived its drop draw (paths sent at t - 1)
    uint32_t pcol = kNoId;
    bool pok = false;
    if constexpr ((kExt & kExtPol) != 0) pv_swim_probe(a, lr, uint32_t(r), pcol, pok);
    pm.mark(0);
    if constexpr ((kExt & ~kExtRot) == 0 && kQlo == 0) {   // (a row without messages evicts nothing)
        if (k == 0) {
            pv_own_only<NT>(a, sh, r, lr, ent0, ro);
            pm.mark(5);
            pv_finish<NT>(a, sh, lr, k, k_all, false, ro);
            pm.mark(6);
            return;
        }
    }
    // one variant per key count (own view + k sender views)
#define GSP_PV_VARIANT(K)                                                                        \
    else if (kQlo <= K && K <= kQhi && k == K)                                                  \
        pv_merge_row<(K < kQlo ? kQlo : K > kQhi ? kQhi : K) + 1, kExt, NT>(a, sh, r, k, ent0, my_slot, \
                                                                          ssrc, jrep, pcol, pok, ro, pm);
    if (false) {}
    GSP_PV_VARIANT(0) GSP_PV_VARIANT(1) GSP_PV_VARIANT(2) GSP_PV_VARIANT(3)
    GSP_PV_VARIANT(4) GSP_PV_VARIANT(5) GSP_PV_VARIANT(6) GSP_PV_VARIANT(7)
#undef GSP_PV_VARIANT
    pm.mark(5);
    pv_finish<NT>(a, sh, lr, k, k_all, false, ro);
    pm.mark(6);
}

// Tick 0: every row writes its pre-joined bounded view {(r + 1 + j * (n / V)) mod n} (or
// everyone if n - 1 <= V) with hb = h0, ts = 0.
__global__ void __launch_bounds__(kPvBlock) pview_init_kernel(PviewTickArgs a) {
    __shared__ PvShared<kMaxKeys> sh;
    const int32_t tid = threadIdx.x;
    const int32_t lr = blockIdx.x, r = a.row0 + lr, V = a.view, n = a.n;
    if (a.tick > a.fail_tick[r]) {
        if (tid < 16) a.rowdig[int64_t(lr) * 16 + tid] = 0ull;
        return;
    }
    RowOut ro{};
    uint32_t *ids = sh.keys[0];
    if (n - 1 <= V) {
        for (int32_t x = tid; x < n; x += kPvBlock)
            if (x != r) ids[x < r ? x : x - 1] = uint32_t(x);
        ro.len = n - 1;
    } else {
        const int64_t stride = n / V;
        const int64_t first_wrap = (int64_t(n) - r - 1 + stride - 1) / stride;
        const int32_t J = int32_t(first_wrap < V ? first_wrap : V);
        for (int32_t j = tid; j < V; j += kPvBlock) {
            int64_t x = int64_t(r) + 1 + int64_t(j) * stride;
            int32_t p;
            if (x >= n) { x -= n; p = j - J; } else { p = j + (V - J); }
            ids[p] = uint32_t(x);
        }
        ro.len = V;
    }
    ro.ids_off = 0;
    if (a.start_tick) {        // join schedule: only the nodes that start at tick 0 are listed
        __syncthreads();
        const bool late = a.start_tick[r] > 0;
        const uint32_t x = tid < ro.len ? ids[tid] : 0u;
        const bool keep = tid < ro.len && !late && a.start_tick[x] == 0;
        uint32_t total = 0;
        const uint32_t pos = block_scan(keep ? 1u : 0u, &total, sh.keys[1]);
        if (keep) sh.keys[1][8 + pos] = x;
        ro.len = int32_t(total);
        ro.ids_off = lds_word(sh, sh.keys[1] + 8);       // keys[1][8 ..): the kept ids
    }
    for (int32_t i = tid; i < ro.len; i += kPvBlock) sh.vals[i] = uint16_t(a.h0 << 5);
    ro.vals_off = lds_half(sh, sh.vals);
    __syncthreads();
    pv_finish<kPvBlock>(a, sh, lr, 0, 0, true, ro);
}

// The one-kernel form (GSP_TEST_PV_SPLIT=0; every row a 256-lane row in 20 KB, any k).  One row
// per workgroup: a software-pipelined variant (the next row's record, own view and first
// sender views requested while the current row merged, two rows per workgroup) measured 4-8 %
// slower -- other resident rows already hide the HBM round trips.
template <int kExt>
__global__ void __launch_bounds__(kPvBlock, 8) pview_tick_kernel(PviewTickArgs a) {
    __shared__ PvShared<kMaxKeys> sh;
    if (a.order && a.drain) {                // the bucketed rows only (drain: long rows are not)
        int32_t total = 0;
#pragma unroll
        for (int q = 0; q <= kPvMaxInbox; ++q) total += a.kcount[q];
        if (int32_t(blockIdx.x) >= total) return;
    }
    pv_row<kExt, kPvBlock, 0, 7>(a, sh, pv_row_of(a, int32_t(blockIdx.x)));
}

// Split form (rows bucketed by k, a.order set): the rows that merge at most 3 messages
// (kQhi = 3: at most 4 sources, 1024 keys) run as 128-lane rows in 10 KB of LDS -- 16 rows
// per CU instead of 8, two waves per row instead of four, each lane holding two slots of
// every source -- k = 4 and k = 5 as 128-lane rows merged in place in 9.8 / 11.3 KB, k = 6, 7
// as 256-lane rows in 20 KB.  One kernel per k range, heavy rows first; workgroup b runs the
// b-th row of the range's k-descending order, the grid is the range's bucket size (read back
// by the host after the receipt kernel: launch_pview_tick).
template <int kExt, int NT, int kQlo, int kQhi, int kMinWaves = 8, bool kIP = false>
__global__ void __launch_bounds__(NT, kMinWaves) pview_tick_split_kernel(PviewTickArgs a) {
    constexpr int kKeys = NT == 64 ? 512 : kQhi <= 3 ? 1024 : (kQhi + 1) * kSlots;
    __shared__ std::conditional_t<kIP, PvSharedIP<kKeys>, PvShared<kKeys>> sh;
    static_assert(NT != 64 || kQhi <= 1, "one-wave rows hold at most 2 sources");
    int32_t tot = 0;                             // the range's rows: a grid past them (a.nowait)
#pragma unroll
    for (int q = kQlo; q <= kQhi; ++q) tot += a.kcount[q];
    if (int32_t(blockIdx.x) >= tot) return;
    pv_row<kExt, NT, kQlo, kQhi>(a, sh, pv_row_of<kQlo, kQhi>(a, int32_t(blockIdx.x)));
}

// The K smallest senders of every receiver's CSR segment, ascending (the canonical receipt
// order; the rest is inbox overflow), as a fixed 8-slot record.  One lane per row, keeping a
// sorted best 8: a sender not below the current 8th costs one compare (early reject), loads 4
// at a time.  Rows past kPvWaveSegment senders (the hubs the eviction order makes: thousands of
// senders at config 5 past tick ~70) are left to their wave, which runs them one after the
// other: every lane keeps a best 8 of its stride of the segment, then 8 rounds of a wave
// minimum pop the row's 8 smallest.  With a.kcount set, the rows are also bucketed by k (how
// many messages they merge): the tick kernel then runs them k-descending.
constexpr int32_t kPvWaveSegment = 64;

// sender i of a segment and its row (>= 0 local, < 0 remote -slot - 1)
__device__ __forceinline__ void pv_sender(const PviewReceiptArgs &a, int32_t o, int32_t &s, int32_t &sl) {
    s = a.csr_src[o];
    sl = a.csr_slot ? a.csr_slot[o] : s - a.row0;
}

// insertion into the ascending best 8 (bs, bl); a sender >= bs[7] changes nothing
__device__ __forceinline__ void pv_best8(int32_t (&bs)[8], int32_t (&bl)[8], int32_t s, int32_t sl) {
    if (s >= bs[7]) return;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const bool lt = s < bs[q];
        const int32_t ts = bs[q], tl = bl[q];
        bs[q] = lt ? s : ts;
        bl[q] = lt ? sl : tl;
        s = lt ? ts : s;
        sl = lt ? tl : sl;
    }
}

// the best 8 of senders [i0, k) with stride `step` of the segment at o0
__device__ __forceinline__ void pv_best8_scan(const PviewReceiptArgs &a, int32_t o0, int32_t i0, int32_t k,
                                              int32_t step, int32_t (&bs)[8], int32_t (&bl)[8]) {
    int32_t i = i0;
    for (; i + 3 * step < k; i += 4 * step) {        // four loads in flight
        int32_t s[4], sl[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pv_sender(a, o0 + i + u * step, s[u], sl[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) pv_best8(bs, bl, s[u], sl[u]);
    }
    for (; i < k; i += step) {
        int32_t s, sl;
        pv_sender(a, o0 + i, s, sl);
        pv_best8(bs, bl, s, sl);
    }
}

__device__ __forceinline__ int32_t wave_min_i32(int32_t x) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x = min(x, __shfl_xor(x, d, 64));
    return x;
}

__global__ void __launch_bounds__(256) pview_receipt_kernel(PviewReceiptArgs a) {
    const int32_t lr = int32_t(blockIdx.x) * 256 + int32_t(threadIdx.x);
    const int32_t lane = int32_t(threadIdx.x) & 63;
    const bool valid = lr < a.rows;
    int32_t k = 0, k_all = 0, o0 = 0;
    int32_t bs[8], bl[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) { bs[q] = 0x7FFFFFFF; bl[q] = 0; }
    bool wide = false, lng = false;
    if (valid) {
        o0 = a.off[lr];
        k_all = a.off[lr + 1] - o0;
        if (k_all > a.max_segment) atomicCAS(a.err, 0, a.tick);   // this tick's tick kernel runs no row
        else if (a.drain && k_all > kPvMaxInbox) lng = true;        // pview_drain_kernel's
        else if (k_all > kPvWaveSegment) wide = true;
        else pv_best8_scan(a, o0, 0, k_all, 1, bs, bl);
        k = (k_all > a.max_segment || lng) ? 0 : (k_all < a.inbox ? k_all : a.inbox);
    }
    if (a.drain) {           // the long rows by drain class: one global atomic per class and
                             // workgroup (per wave, 16 K waves per tick on 4 counters, cost 0.17 ms)
        __shared__ int32_t cls_cnt[kDrainClasses][4], cls_msg[kDrainClasses][4], cls_base[kDrainClasses];
        const int32_t wave = int32_t(threadIdx.x) >> 6;
        const int32_t c = lng ? pv_drain_class(k_all, a.view, a.drain_lds, a.drain_wide) : -1;
        unsigned long long mine = 0;
#pragma unroll
        for (int q = 0; q < kDrainClasses; ++q) {
            const unsigned long long lm = __ballot(c == q);
            const uint32_t msgs = wave_sum32(c == q ? uint32_t(k_all) : 0u);
            if (lane == 0) { cls_cnt[q][wave] = __popcll(lm); cls_msg[q][wave] = int32_t(msgs); }
            mine = c == q ? lm : mine;
        }
        __syncthreads();
        if (threadIdx.x < kDrainClasses) {       // rows of each class at [c], messages at [8 + c]
            const int32_t q = int32_t(threadIdx.x);
            const int32_t tot = cls_cnt[q][0] + cls_cnt[q][1] + cls_cnt[q][2] + cls_cnt[q][3];
            cls_base[q] = tot ? atomicAdd(&a.long_list[q], tot) : 0;
            if (tot) atomicAdd(&a.long_list[8 + q], cls_msg[q][0] + cls_msg[q][1] + cls_msg[q][2] + cls_msg[q][3]);
        }
        __syncthreads();
        if (c >= 0) {
            int32_t at = cls_base[c] + __popcll(mine & ((1ull << lane) - 1ull));
            for (int32_t w = 0; w < wave; ++w) at += cls_cnt[c][w];
            a.long_list[kDrainHead + c * a.rows + at] = lr;
        }
    }
    // the wave's wide rows, one after the other (wave-uniform loop)
    for (unsigned long long m = __ballot(wide); m; m &= m - 1) {
        const int32_t l = __builtin_ffsll(m) - 1;
        const int32_t wo = __builtin_amdgcn_readlane(o0, l), wk = __builtin_amdgcn_readlane(k_all, l);
        int32_t ws[8], wl[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) { ws[q] = 0x7FFFFFFF; wl[q] = 0; }
        pv_best8_scan(a, wo, lane, wk, 64, ws, wl);
        // 8 rounds: the smallest head of the lanes' sorted lists (senders are distinct, so one
        // lane holds it) goes to lane l's record, and that lane pops it
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int32_t mn = wave_min_i32(ws[0]);
            const unsigned long long who = __ballot(ws[0] == mn && mn != 0x7FFFFFFF);
            const int32_t src_slot = who ? __builtin_amdgcn_readlane(wl[0], __builtin_ffsll(who) - 1) : 0;
            if (lane == l) { bs[q] = mn; bl[q] = src_slot; }
            if (who && lane == __builtin_ffsll(who) - 1) {
#pragma unroll
                for (int z = 0; z < 7; ++z) { ws[z] = ws[z + 1]; wl[z] = wl[z + 1]; }
                ws[7] = 0x7FFFFFFF;
            }
        }
    }
    if (valid) {
        int4 *ps = reinterpret_cast<int4 *>(a.rc_src + int64_t(lr) * 8);
        int4 *pl = reinterpret_cast<int4 *>(a.rc_slot + int64_t(lr) * 8);
        ps[0] = make_int4(bs[0], bs[1], bs[2], bs[3]);
        ps[1] = make_int4(bs[4], bs[5], bs[6], bs[7]);
        pl[0] = make_int4(bl[0], bl[1], bl[2], bl[3]);
        pl[1] = make_int4(bl[4], bl[5], bl[6], bl[7]);
        a.rc_info[lr] = k | (k_all << 3);
    }
    if (a.kcount) {        // block histogram of k, one global atomic per non-empty bucket
        __shared__ int32_t s_cnt[8], s_base[8];
        if (threadIdx.x < 8) s_cnt[threadIdx.x] = 0;
        __syncthreads();
        const bool bucket = valid && !lng;       // drain: a long row is in no bucket
        const int32_t pos = bucket ? atomicAdd(&s_cnt[k], 1) : 0;
        __syncthreads();
        if (threadIdx.x < 8 && s_cnt[threadIdx.x])
            s_base[threadIdx.x] = atomicAdd(&a.kcount[threadIdx.x], s_cnt[threadIdx.x]);
        __syncthreads();
        if (bucket) a.order[int64_t(k) * a.rows + s_base[k] + pos] = lr;
    }
}

// Peers and sends of every row (one lane per row), after the tick kernel wrote the views:
// min(F, len) distinct members by Philox rank-select over the id order, then the drop draw.
// kF: the fan-out bound the peer arrays are sized for (4 covers config 5's f = 3 in a quarter of
// the registers and compares of the general 16)
template <int kF>
__global__ void __launch_bounds__(256) pview_send_kernel(PviewTickArgs a) {
    const int32_t lr = int32_t(blockIdx.x) * 256 + int32_t(threadIdx.x);
    const uint32_t t = uint32_t(a.tick);
    // TFAIL: peers and the probe target are chosen among the members not suspected at t, by
    // rank in id order (an 8-word bitmap of the gossipable slots).  The wave builds its 64 rows'
    // bitmaps together, every lane still active: row j is read coalesced (lane l takes slots
    // l, l + 64, ...) and four ballots give its bitmap to lane j -- one lane reading its own 2 KB
    // row slot by slot made every load touch 64 rows' lines (3.7 ms per tick at config 5)
    uint32_t gmask[kPvMaxView / 32];
#pragma unroll
    for (int w = 0; w < kPvMaxView / 32; ++w) gmask[w] = 0u;
    if (a.tfail > 0) {
        const uint32_t t5 = t & 31u, tf = uint32_t(a.tfail);
        const int32_t lane = int32_t(threadIdx.x) & 63, lr0 = lr - lane;
        for (int32_t j0 = 0; j0 < 64; j0 += 4) {                 // 4 rows' loads in flight
            uint64_t e[4][kPvMaxView / 64];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int c = 0; c < kPvMaxView / 64; ++c) {
                    const int32_t lj = lr0 + j0 + u, i = c * 64 + lane;
                    e[u][c] = lj < a.rows && i < a.view ? a.cur[int64_t(lj) * a.view + i] : kPvEmpty;
                }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int c = 0; c < kPvMaxView / 64; ++c) {
                    const uint64_t b = __ballot(e[u][c] != kPvEmpty && ((t5 - uint32_t(e[u][c])) & 31u) < tf);
                    if (lane == j0 + u) {
                        gmask[2 * c] = uint32_t(b);
                        gmask[2 * c + 1] = uint32_t(b >> 32);
                    }
                }
        }
    }
    if (lr >= a.rows) return;
    const int32_t r = a.row0 + lr, F = a.fanout;
    unsigned long long *w3 = a.rowdig + int64_t(lr) * 16 + 3;
    const bool dead = a.tick > a.fail_tick[r] || (a.start_tick && a.tick < a.start_tick[r]) ||
                      (a.tick > 0 && *a.err);
    int32_t *od = a.out_dst + int64_t(lr) * F;
    if (dead) {
        for (int32_t q = 0; q < F; ++q) od[q] = -1;
        if (a.swim > 0) a.ping[lr] = -1;
        *w3 = 0ull;
        return;
    }
    const int32_t len = a.len_cur[lr];
    const uint64_t *row = a.cur + int64_t(lr) * a.view;
    int32_t cnt = len;
    if (a.tfail > 0) {
        cnt = 0;
#pragma unroll
        for (int w = 0; w < kPvMaxView / 32; ++w) {              // slots past len are empty
            const int32_t lo = w * 32;
            const uint32_t keep = len >= lo + 32 ? ~0u : len <= lo ? 0u : (1u << (len - lo)) - 1u;
            gmask[w] &= keep;
            cnt += __builtin_popcount(gmask[w]);
        }
    }
    auto slot_of = [&](int32_t rk) -> int32_t {     // rank among the gossipable -> slot
        if (a.tfail <= 0) return rk;
#pragma unroll
        for (int w = 0; w < kPvMaxView / 32; ++w) {
            const int32_t c = __builtin_popcount(gmask[w]);
            if (rk < c) {
                uint32_t m = gmask[w];
                for (int32_t z = 0; z < rk; ++z) m &= m - 1;
                return w * 32 + __builtin_ffs(m) - 1;
            }
            rk -= c;
        }
        return 0;
    };
    const int32_t keff = F < cnt ? F : cnt;
    int32_t ch[kF], dst[kF];
#pragma unroll
    for (int q = 0; q < kF; ++q) { ch[q] = 0x7FFFFFFF; dst[q] = -1; }
#pragma unroll
    for (int kk = 0; kk < kF; ++kk) {
        if (kk >= keff) continue;
        const uint32_t u = draw_u31(kDomainPeer, a.seed, t, uint32_t(r), uint32_t(kk), 0u);
        int32_t rk = int32_t(u % uint32_t(cnt - kk));
#pragma unroll
        for (int q = 0; q < kF; ++q) rk += (q < kk && rk >= ch[q]) ? 1 : 0;   // ch ascending
        int32_t x = rk;
#pragma unroll
        for (int q = 0; q < kF; ++q) {                   // insert rk, keeping ch ascending
            const bool lt = x < ch[q];
            const int32_t c = ch[q];
            ch[q] = lt ? x : c;
            x = lt ? c : x;
        }
        dst[kk] = int32_t(row[slot_of(rk)] >> 32);
    }
    uint32_t dropped = 0;
#pragma unroll
    for (int kk = 0; kk < kF; ++kk) {
        if (kk >= F) continue;
        int32_t d = dst[kk];
        if (d >= 0) {
            const uint32_t dr = draw_u31(kDomainSend, a.seed, t, uint32_t(r), uint32_t(d), 3u);
            if (int32_t(dr % 100u) < a.drop_pct) { d = -1; dropped++; }
        }
        od[kk] = d;
        if (d >= 0) {
            const int32_t pos = atomicAdd(&a.deg[d], 1);
            if (a.out_pos) a.out_pos[int64_t(lr) * F + kk] = pos;
        }
    }
    if (a.swim > 0) {          // this tick's probe target: one more rank over the same order
        int32_t p = -1;
        if (cnt > 0)
            p = int32_t(row[slot_of(int32_t(draw_u31(kDomainPing, a.seed, t, uint32_t(r), 0u, 0x100u) %
                                            uint32_t(cnt)))] >> 32);
        a.ping[lr] = p;
    }
    *w3 = uint64_t(keff) | (uint64_t(dropped) << 8);
}

// Per-tick digest: sums the per-row records (4 per row, one per wave of the tick kernel:
// w0 = merges | delivered << 32 | round << 56, w1 = joins | removes << 16 | evicts << 32 |
// overflow << 48, w2 = event hash, w3 = sent | dropped << 8 from the send kernel).
__global__ void __launch_bounds__(256) pview_digest_kernel(const unsigned long long *rowdig,
                                                           int64_t records, unsigned long long *dig) {
    unsigned long long f[kPvFields] = {0};
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < records;
         i += int64_t(gridDim.x) * 256) {
        const ulonglong2 x = reinterpret_cast<const ulonglong2 *>(rowdig)[i * 2];
        const ulonglong2 y = reinterpret_cast<const ulonglong2 *>(rowdig)[i * 2 + 1];
        f[kPvMerges] += x.x & 0xFFFFFFFFull;
        f[kPvDelivered] += (x.x >> 32) & 0xFFull;
        f[kPvRounds] += (x.x >> 56) & 1ull;
        f[kPvJoins] += x.y & 0xFFFFull;
        f[kPvRemoves] += (x.y >> 16) & 0xFFFFull;
        f[kPvEvicts] += (x.y >> 32) & 0xFFFFull;
        f[kPvOverflow] += x.y >> 48;
        f[kPvHash] += y.x;
        f[kPvSent] += y.y & 0xFFull;
        f[kPvDropped] += (y.y >> 8) & 0xFFull;
    }
    __shared__ unsigned long long part[4][kPvFields];
    const int32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < kPvFields; ++q) {
        const unsigned long long s = wave_sum64(f[q]);
        if (lane == 0) part[wave][q] = s;
    }
    __syncthreads();
    if (threadIdx.x < kPvFields) {
        const int q = threadIdx.x;
        const unsigned long long s = part[0][q] + part[1][q] + part[2][q] + part[3][q];
        if (s) atomicAdd(&dig[(blockIdx.x % kPvDigSlots) * kPvFields + q], s);
    }
}

// Receiver CSR of one shard without atomics: message i of sender row i / F goes to slot
// out_pos[i] of its receiver's segment (MP1Node's queue order is not kept by any scatter: the
// receipt kernel sorts each segment's senders).
__global__ void pview_scatter_kernel(const int32_t *out_dst, const int32_t *out_pos, int64_t slots,
                                     int32_t fanout, const int32_t *off, int32_t *csr_src) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < slots;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int32_t d = out_dst[i];
        if (d >= 0) csr_src[off[d] + out_pos[i]] = int32_t(i / fanout);
    }
}

bool pv_args_ok(const PviewTickArgs &a) {
    return a.view >= 1 && a.view <= kPvMaxView && a.inbox >= 1 && a.inbox <= kPvMaxInbox &&
           a.fanout >= 1 && a.fanout <= 16 && a.n < (1 << 21) && a.rows >= 0;
}

unsigned digest_blocks(int64_t records) {
    return unsigned(records < 262144 ? (records + 255) / 256 : 1024);
}

void launch_send_and_digest(const PviewTickArgs &a, hipStream_t st) {
    if (a.fanout <= 4)
        hipLaunchKernelGGL(pview_send_kernel<4>, dim3(unsigned((a.rows + 255) / 256)), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(pview_send_kernel<16>, dim3(unsigned((a.rows + 255) / 256)), dim3(256), 0, st, a);
    // the init tick's records hold only w3 (sends) -- its rowdig was zeroed by the host
    const int64_t records = int64_t(a.rows) * 4;
    hipLaunchKernelGGL(pview_digest_kernel, dim3(digest_blocks(records)), dim3(256), 0, st, a.rowdig,
                       records, a.dig);
}

}  // namespace

hipError_t launch_pview_init(const PviewTickArgs &a, hipStream_t st) {
    if (!pv_args_ok(a)) return hipErrorInvalidValue;
    if (a.rows == 0) return hipSuccess;
    hipLaunchKernelGGL(pview_init_kernel, dim3(a.rows), dim3(kPvBlock), 0, st, a);
    launch_send_and_digest(a, st);
    return hipGetLastError();
}

hipError_t launch_pview_scatter(const int32_t *out_dst, const int32_t *out_pos, int64_t slots,
                                int32_t fanout, const int32_t *off, int32_t *csr_src, hipStream_t st) {
    if (slots <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((slots + 255) / 256, 8192);
    hipLaunchKernelGGL(pview_scatter_kernel, dim3(unsigned(blocks)), dim3(256), 0, st, out_dst, out_pos,
                       slots, fanout, off, csr_src);
    return hipGetLastError();
}

hipError_t launch_pview_receipt(const PviewReceiptArgs &a, hipStream_t st) {
    if (a.inbox < 1 || a.inbox > kPvMaxInbox || a.rows < 0) return hipErrorInvalidValue;
    if (a.rows == 0) return hipSuccess;
    hipLaunchKernelGGL(pview_receipt_kernel, dim3(unsigned((a.rows + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_pview_tick(const PviewTickArgs &a, hipStream_t st) {
    if (!pv_args_ok(a)) return hipErrorInvalidValue;
    if (a.rows == 0) return hipSuccess;
    const dim3 g(unsigned(a.rows)), blk(kPvBlock);
    // the protocol extensions in use select the kernel: kExtPol for TFAIL / SWIM / joins,
    // kExtEv for the event stream (the plain protocol runs neither)
    const int ext = ((a.tfail > 0 || a.swim > 0 || a.start_tick != nullptr) ? kExtPol : 0) |
                    (a.ev.buf != nullptr ? kExtEv : 0) | (a.evict_rot ? kExtRot : 0);
    if (a.order && a.split) {
        // split form: k = 6, 7 / k = 5 / k = 4 / k <= 3 (pview_tick_split_kernel), in this order
        // (the heavy rows first), each on a grid of exactly its bucket's rows: the bucket sizes
        // are copied back behind an event after the receipt kernel and the host waits for it
        // (round 5: on one box, ticks 6-25, 5.36 ms against 5.42 for round 3's grids predicted
        // without a wait plus an overflow kernel, and 6.7-13 ms for persistent kernels pulling
        // row chunks from per-XCD heads -- DESIGN.md 4b)
        // Row shards (a.nowait) skip that wait: every range launches on `rows` workgroups, those
        // past the range's bucket exit after reading its counts (pview_tick_split_kernel), so
        // the host queues tick after tick behind the exchange's collectives.
        PviewTickArgs b = a;
        int32_t c[8];
        if (a.nowait) {
            for (int q = 0; q < 8; ++q) c[q] = q == 0 ? a.rows : 0;
            b.drain_rows = nullptr;
            if (a.drain && a.dhead_async &&
                hipMemcpyAsync(a.dhead_async, a.long_list, kDrainHead * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
                return hipGetLastError();
        } else {
            if (!a.kcount_host || !a.kcount_event) return hipErrorInvalidValue;
            if (hipMemcpyAsync(a.kcount_host, a.kcount, 8 * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                (a.drain && a.drain_rows &&
                 hipMemcpyAsync(a.drain_rows, a.long_list, kDrainHead * 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
                hipEventRecord(a.kcount_event, st) != hipSuccess || hipEventSynchronize(a.kcount_event) != hipSuccess)
                return hipGetLastError();
            for (int q = 0; q < 8; ++q) c[q] = a.kcount_host[q];
        }
        const unsigned g67 = a.nowait ? unsigned(a.rows) : unsigned(c[6] + c[7]),
                       g5 = a.nowait ? unsigned(a.rows) : unsigned(c[5]),
                       g4 = a.nowait ? unsigned(a.rows) : unsigned(c[4]),
                       g03 = unsigned(c[0] + c[1] + c[2] + c[3]);
        // k = 6, 7: 256-lane rows in 20 KB, 8 waves per SIMD (8 rows per CU); k = 5 / k = 4:
        // 128-lane rows merged in place (PvSharedIP, 11.3 / 9.8 KB) at 6 / 7 waves per SIMD (12 /
        // 14 rows; 8 / 7 spill 24 / 20 B); k <= 3: 128-lane rows in 10 KB (16 rows per CU).
        // DESIGN.md 4b records the A/Bs behind each choice.
#define GSP_PV_RANGE(E, NT, LO, HI, W, IP, G) \
        if (G) hipLaunchKernelGGL((pview_tick_split_kernel<E, NT, LO, HI, W, IP>), dim3(G), dim3(NT), 0, st, b);
#define GSP_PV_SPLIT_LAUNCH(E)                                                                            \
    do {                                                                                                  \
        GSP_PV_RANGE(E, 256, 6, 7, 8, false, g67)                                                       \
        GSP_PV_RANGE(E, 128, 5, 5, 6, true, g5)                                                         \
        GSP_PV_RANGE(E, 128, 4, 4, 7, true, g4)                                                         \
        GSP_PV_RANGE(E, 128, 0, 3, 8, false, g03)                                                       \
    } while (0)
        // drain all: the hub kernel goes first on a stream of its own (its rows and the others'
        // are disjoint): a tick's few hub rows run one per CU and would leave the rest of the GPU
        // idle behind them; every drain class there (drain_side 1) was slower
        const bool side = a.drain && a.drain_st && a.drain_fork && a.drain_join;
        if (side) {
            if (hipEventRecord(a.drain_fork, st) != hipSuccess ||
                hipStreamWaitEvent(a.drain_st, a.drain_fork, 0) != hipSuccess)
                return hipGetLastError();
            const hipError_t e = launch_pview_drain(b, a.drain_st, a.drain_side == 2 ? 2 : 3);
            if (e != hipSuccess) return e;
        }
        switch (ext) {      // evict_order 1: the plain protocol's kernel, or the superset one
            case 0: GSP_PV_SPLIT_LAUNCH(0); break;
            case kExtEv: GSP_PV_SPLIT_LAUNCH(kExtEv); break;
            case kExtPol: GSP_PV_SPLIT_LAUNCH(kExtPol); break;
            case kExtPol | kExtEv: GSP_PV_SPLIT_LAUNCH(kExtPol | kExtEv); break;
            case kExtRot: GSP_PV_SPLIT_LAUNCH(kExtRot); break;
            default: GSP_PV_SPLIT_LAUNCH(kExtRot | kExtPol | kExtEv); break;
        }
#undef GSP_PV_SPLIT_LAUNCH
#undef GSP_PV_RANGE
        if (side && a.drain_side == 2) {                 // the LDS classes after the split kernels
            const hipError_t e = launch_pview_drain(b, st, 1);
            if (e != hipSuccess) return e;
        }
        if (side) {
            if (hipEventRecord(a.drain_join, a.drain_st) != hipSuccess ||
                hipStreamWaitEvent(st, a.drain_join, 0) != hipSuccess)
                return hipGetLastError();
        } else if (a.drain) {
            const hipError_t e = launch_pview_drain(b, st);
            if (e != hipSuccess) return e;
        }
        launch_send_and_digest(b, st);
        return hipGetLastError();
    }
    switch (ext) {
        case 0: hipLaunchKernelGGL((pview_tick_kernel<0>), g, blk, 0, st, a); break;
        case kExtEv: hipLaunchKernelGGL((pview_tick_kernel<kExtEv>), g, blk, 0, st, a); break;
        case kExtPol: hipLaunchKernelGGL((pview_tick_kernel<kExtPol>), g, blk, 0, st, a); break;
        case kExtPol | kExtEv: hipLaunchKernelGGL((pview_tick_kernel<kExtPol | kExtEv>), g, blk, 0, st, a); break;
        default: hipLaunchKernelGGL((pview_tick_kernel<kExtRot | kExtPol | kExtEv>), g, blk, 0, st, a); break;
    }
    if (a.drain) {
        PviewTickArgs b = a;
        b.drain_rows = nullptr;                  // not copied back in this form: persistent grids
        const hipError_t e = launch_pview_drain(b, st);
        if (e != hipSuccess) return e;
    }
    launch_send_and_digest(a, st);
    return hipGetLastError();
}

}  // namespace gsp
