// gossip_protocol_amd/csrc/event_ring.hpp -- the device event ring of the scale engines.
//
// The tick kernels append join / remove / evict records (event_record, scale_kernels.hpp) --
// the reference's Log::logNodeAdd / logNodeRemove lines (Log.cpp:116-130) at scale.  The ring
// is striped: kEvStripes sub-rings of equal capacity, each with its own counter on its own
// 128-byte line, and a workgroup appends to stripe blockIdx.x % kEvStripes.  One counter for
// the whole job serialises every reservation of a tick on one address (config 3: +7 % kernel
// time with one reservation per row, config 5: x9 with two per wave); 256 counters, hit from a
// fixed XCD each (workgroups go round-robin over the 8 XCDs), take that away.
#pragma once

#include <cstdint>

#include "common.hpp"
#include "gossip/gossip.h"

namespace gsp {

constexpr int kEvStripes = 256;
constexpr int kEvCounterStride = 16;      // u64 words between counters (128 B)

// What a kernel needs: stripe s of the ring is buf[s * cap, (s + 1) * cap), its counter
// count[s * kEvCounterStride]; kinds: bit k set = record kind k (1 join, 2 remove, 3 evict).
struct EvRingArgs {
    unsigned long long *buf;               // null: events off
    unsigned long long *count;
    int64_t cap;                           // records per stripe
    uint32_t kinds;
};

#if defined(__HIPCC__)
// this workgroup's stripe
__device__ inline unsigned long long *ev_stripe_buf(const EvRingArgs &e) {
    return e.buf + int64_t(blockIdx.x % kEvStripes) * e.cap;
}
__device__ inline unsigned long long *ev_stripe_count(const EvRingArgs &e) {
    return e.count + (blockIdx.x % kEvStripes) * kEvCounterStride;
}
#endif

// host side: one shard's ring
struct EvRing {
    DevBuf<unsigned long long> buf, count;
    int64_t stripe_cap = 0;
    uint32_t kinds = 0;

    // events: the params' field (0 off, 1 every kind, else an OR of GSP_EVENTS_JOIN / REMOVE /
    // EVICT); total_cap: records (0: 2^24), rounded up to a multiple of kEvStripes
    hipError_t alloc(int32_t events, int64_t total_cap, hipStream_t st);
    EvRingArgs args() const { return EvRingArgs{buf.p, count.p, stripe_cap, kinds}; }
    // copies at most `cap` records (every stripe in order) into out (null: count only, the
    // ring is kept), adds the held / lost records to *n / *lost, and empties the ring when out
    // is given
    hipError_t drain(uint64_t *out, int64_t cap, int64_t *n, int64_t *lost);
    void release() {
        buf.release();
        count.release();
    }
};

}  // namespace gsp
