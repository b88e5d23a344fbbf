// gossip_protocol_amd/csrc/pview_rules.hpp -- the partial view's per-entry rules on packed
// 16-bit values (hb << 5 | ts mod 32, 0 = absent) and its digest hash, shared by the tick
// kernels (pview_kernels.hip) and the drain-all kernel (pview_drain.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsp {

// Event digest term (oracle/pview_oracle.c gsp_pv_event_mix): S + g(x) per event, S a row seed
// per kind (1 join, 2 remove, 3 evict) and g(x) = ((x ^ lo32(S)) * 0x9E3779B1) >> 5.  A row
// hashes ~1000 events per tick, so the per-event part is one multiply (round 4; it was a
// three-multiply 64-bit finaliser): lanes sum g(x) in 32 bits (< 2^27 each, at most 30 per
// lane) and pv_finish adds the S terms once per wave, as the wave's event counts times S.
__device__ inline uint64_t pv_seed(uint32_t kind, uint32_t t, uint32_t r) {
    uint64_t z = (uint64_t(kind) << 62) | (uint64_t(t & 0xFFFFF) << 42) | (uint64_t(r & 0x1FFFFF) << 21);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ inline uint32_t pv_hash(uint32_t s, uint32_t x) {
    return ((x ^ s) * 0x9E3779B1u) >> 5;
}

// the reference's merge of one payload entry (packed hb << 5 | ts5, 0 = absent)
__device__ inline uint32_t pv_merge(uint32_t e, uint32_t v, uint32_t t5, uint32_t tr) {
    const uint32_t upd = ((v >> 5) > (e >> 5)) ? ((v & 0xFFE0u) | t5) : e;
    const uint32_t add = (v != 0u && ((t5 - v) & 31u) < tr) ? v : 0u;
    return e ? upd : add;
}
// eviction order bin of a surviving entry: age * 32 + min(h0 + t - age - hb, 31), th0 = h0 + t
__device__ inline uint32_t pv_bin(uint32_t v, uint32_t t5, uint32_t th0) {
    const uint32_t age = (t5 - v) & 31u;
    const int32_t e = int32_t(th0 - age) - int32_t(v >> 5);
    return (age << 5) | uint32_t(e < 0 ? 0 : e > 31 ? 31 : e);
}
// the sender entry of a GOSSIP: hb + 1 and ts = t, or (1, t) when absent (MP1Node.cpp:237-243)
__device__ inline uint32_t pv_event(uint32_t v, uint32_t t5) { return (((v >> 5) + 1u) << 5) | t5; }

}  // namespace gsp
