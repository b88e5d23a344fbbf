/*
 * oracle/gsp_philox.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C Philox4x32-10 (Salmon et al., SC'11, "Parallel random numbers: as easy
 * as 1, 2, 3"; the Random123 reference algorithm) and the counter layout that the
 * build uses to replace the reference's stateful glibc rand() draws:
 *
 *   EmulNet::ENsend   rand() % 100           (/root/reference/EmulNet.cpp:89)
 *   Application::fail rand() % N             (/root/reference/Application.cpp:182)
 *                     rand() % N / 2         (/root/reference/Application.cpp:189)
 *
 * The product has its own independent device implementation
 * (gossip_protocol_amd/csrc/philox.cuh); tests check the two agree and check this
 * one against the published Random123 known-answer vectors.
 */
#ifndef GSP_ORACLE_PHILOX_H
#define GSP_ORACLE_PHILOX_H
#include <stdint.h>

#define GSP_DOMAIN_SEND 0x53454E44u /* "SEND": per-message drop draw      */
#define GSP_DOMAIN_FAIL 0x4641494Cu /* "FAIL": failure-injection draw     */
#define GSP_DOMAIN_PEER 0x50454552u /* "PEER": scale-mode peer choice     */
#define GSP_DOMAIN_PING 0x50494E47u /* "PING": SWIM probe target / paths  */
#define GSP_DOMAIN_JOIN 0x4A4F494Eu /* "JOIN": bounded introducer list     */
#define GSP_DOMAIN_EVICT 0x45564354u /* "EVCT": eviction tie rotation (evict_order 1) */

static inline void gsp_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2],
                                     uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* A rand()-shaped draw in [0, 2^31): word 0 of Philox(ctr, key) shifted right once. */
static inline uint32_t gsp_philox_u31(uint32_t domain, uint64_t seed, uint32_t a,
                                      uint32_t b, uint32_t c, uint32_t d) {
    uint32_t ctr[4] = {a, b, c, d};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32) ^ domain};
    uint32_t out[4];
    gsp_philox4x32_10(ctr, key, out);
    return out[0] >> 1;
}

#endif
