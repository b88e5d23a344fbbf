// gossip_protocol_amd/csrc/philox.hpp -- counter-based Philox4x32-10 for host and device.
//
// The build replaces the reference's stateful rand() (EmulNet.cpp:89, Application.cpp:182/189)
// with a draw addressed by (domain, seed; a, b, c, d), so any message's drop decision and any
// peer choice can be computed by whichever lane owns it, in any order.  Algorithm: Salmon et
// al., SC'11 (Random123).  Key = (seed_lo, seed_hi ^ domain), counter = (a, b, c, d); the
// rand()-shaped value is word 0 >> 1, in [0, 2^31).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsp {

enum : uint32_t {
    kDomainSend = 0x53454E44u,  // "SEND": drop draw of one message
    kDomainFail = 0x4641494Cu,  // "FAIL": failure injection
    kDomainPeer = 0x50454552u,  // "PEER": scale-mode peer choice
    kDomainPing = 0x50494E47u,  // "PING": SWIM probe target and probe paths
    kDomainJoin = 0x4A4F494Eu,  // "JOIN": the members a JOINREP carries (bounded introducer list)
    kDomainEvict = 0x45564354u, // "EVCT": the eviction tie rotation of a row (evict_order 1)
};

// Sequential sampling without replacement: draw k maps u % (cnt - k) onto the ranks not
// chosen yet, in ascending order (chosen[] kept sorted).  Used for peers, probe targets and
// the bounded introducer list alike; identical on host and device, in every lane.
__host__ __device__ inline int32_t next_distinct_rank(uint32_t u, int32_t cnt, int32_t k,
                                                      int32_t *chosen, int32_t &nch) {
    int32_t rk = int32_t(u % uint32_t(cnt - k));
    int32_t pos = 0;
    while (pos < nch && rk >= chosen[pos]) { rk++; pos++; }
    for (int32_t q = nch; q > pos; --q) chosen[q] = chosen[q - 1];
    chosen[pos] = rk;
    nch++;
    return rk;
}

__host__ __device__ inline uint32_t philox_word0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = uint64_t(0xD2511F53u) * c0;
        const uint64_t p1 = uint64_t(0xCD9E8D57u) * c2;
        const uint32_t n0 = uint32_t(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = uint32_t(p0 >> 32) ^ c3 ^ k1;
        c1 = uint32_t(p1);
        c3 = uint32_t(p0);
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c0;
}

__host__ __device__ inline void philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = uint64_t(0xD2511F53u) * c0;
        const uint64_t p1 = uint64_t(0xCD9E8D57u) * c2;
        const uint32_t n0 = uint32_t(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = uint32_t(p0 >> 32) ^ c3 ^ k1;
        c1 = uint32_t(p1);
        c3 = uint32_t(p0);
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// rand()-shaped draw in [0, 2^31).
__host__ __device__ inline uint32_t draw_u31(uint32_t domain, uint64_t seed, uint32_t a, uint32_t b,
                                             uint32_t c, uint32_t d) {
    return philox_word0(a, b, c, d, uint32_t(seed), uint32_t(seed >> 32) ^ domain) >> 1;
}

}  // namespace gsp
