// gossip_protocol_amd/csrc/pview_rules.hpp -- the partial view's per-entry rules on packed
// 16-bit values (hb << 5 | ts mod 32, 0 = absent) and its digest hash, shared by the tick
// kernels (pview_kernels.hip) and the drain-all kernel (pview_drain.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "philox.hpp"
#include "pview_kernels.hpp"

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

// The bounded introducer list (block-uniform): bit q of m = rank q of node 0's gossiped members
// is carried -- B sequential distinct Philox ranks (next_distinct_rank, philox.hpp) kept as a
// 256-bit mask instead of a sorted array, so nothing is indexed dynamically (no scratch).
__device__ inline void pv_intro_mask(uint64_t seed, uint32_t t_send, uint32_t r, int32_t cnt,
                                     int32_t B, uint64_t (&m)[4]) {
    m[0] = m[1] = m[2] = m[3] = 0ull;
    for (int32_t i = 0; i < B; ++i) {
        int32_t rk = int32_t(draw_u31(kDomainJoin, seed, t_send, 0u, r, uint32_t(i)) % uint32_t(cnt - i));
        bool done = false;
#pragma unroll
        for (int w = 0; w < 4; ++w) {                    // the rk-th rank not chosen yet
            const int32_t zeros = 64 - __popcll(m[w]);
            if (!done && rk < zeros) {
                uint64_t z = ~m[w];
                for (int32_t q = 0; q < rk; ++q) z &= z - 1;
                m[w] |= z & (~z + 1);
                done = true;
            }
            if (!done) rk -= zeros;
        }
    }
}

// SWIM: the probe row lr (node r) sent at t - 1 -- its target pcol (0xFFFFFFFF: none) and
// whether it was answered (pok): the target is alive now and one of the swim paths survived
// its drop draw (the drop percentage of the sends of t - 1).  Resolved after the merges, before
// TREMOVE (oracle/pview_oracle.c pv_row_step).  Row-uniform.
__device__ inline void pv_swim_probe(const PviewTickArgs &a, int32_t lr, uint32_t r, uint32_t &pcol, bool &pok) {
    pcol = 0xFFFFFFFFu;
    pok = false;
    if (a.swim <= 0) return;
    const int32_t p = __builtin_amdgcn_readfirstlane(a.ping[lr]);
    if (p < 0) return;
    pcol = uint32_t(p);
    for (int32_t i = 0; i < a.swim; ++i)
        pok = pok || int32_t(draw_u31(kDomainPing, a.seed, uint32_t(a.tick - 1), r, uint32_t(p), uint32_t(i)) %
                             100u) >= a.drop_prev;
    pok = pok && a.tick <= a.fail_tick[p] && (!a.start_tick || a.tick >= a.start_tick[p]);
}
// a TFAIL payload holds the sender's members gossipable at t - 1 ((t - 1) - ts < tfail)
__device__ inline bool pv_gossiped(uint64_t v, uint32_t tf, uint32_t t5m1) {
    return v != ~0ull && (tf == 0 || ((t5m1 - uint32_t(v)) & 31u) < tf);
}

}  // namespace gsp
