// gossip_protocol_amd/csrc/event_ring.cpp -- host side of the striped event ring
// (event_ring.hpp); drained by gsp_scale_drain_events / gsp_pview_drain_events.
#include "event_ring.hpp"

#include <algorithm>
#include <vector>

#include "gossip/gossip.h"

namespace gsp {

hipError_t EvRing::alloc(int32_t events, int64_t total_cap, hipStream_t st) {
    kinds = events == 1 ? (GSP_EVENTS_JOIN | GSP_EVENTS_REMOVE | GSP_EVENTS_EVICT) : uint32_t(events);
    const int64_t total = total_cap > 0 ? total_cap : (int64_t(1) << 24);
    stripe_cap = (total + kEvStripes - 1) / kEvStripes;
    if (hipError_t e = buf.alloc(size_t(stripe_cap) * kEvStripes)) return e;
    if (hipError_t e = count.alloc(size_t(kEvStripes) * kEvCounterStride)) return e;
    return hipMemsetAsync(count.p, 0, size_t(kEvStripes) * kEvCounterStride * 8, st);
}

hipError_t EvRing::drain(uint64_t *out, int64_t cap, int64_t *n, int64_t *lost) {
    std::vector<unsigned long long> c(size_t(kEvStripes) * kEvCounterStride);
    if (hipError_t e = hipMemcpy(c.data(), count.p, c.size() * 8, hipMemcpyDeviceToHost)) return e;
    for (int s = 0; s < kEvStripes; ++s) {
        const int64_t got = int64_t(c[size_t(s) * kEvCounterStride]);
        const int64_t have = std::min(got, stripe_cap);
        *lost += got - have;
        if (!out) {                        // counting only: the ring is kept
            *n += have;
            continue;
        }
        // the records past cap are dropped with the ring: counted as lost, never in *n
        const int64_t take = std::max<int64_t>(0, std::min(have, cap - *n));
        if (take > 0)
            if (hipError_t e = hipMemcpy(out + *n, buf.p + int64_t(s) * stripe_cap, size_t(take) * 8,
                                         hipMemcpyDeviceToHost))
                return e;
        *n += take;
        *lost += have - take;
    }
    if (out) return hipMemset(count.p, 0, size_t(kEvStripes) * kEvCounterStride * 8);
    return hipSuccess;
}

}  // namespace gsp
