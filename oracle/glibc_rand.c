/*
 * oracle/glibc_rand.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Restatement of glibc 2.35's default rand()/srand() (random_r.c, TYPE_3: additive
 * feedback generator, degree 31, separation 3; seeded by the Park-Miller minimal
 * standard LCG through Schrage's method, then 310 outputs discarded).  The reference
 * draws from it at /root/reference/EmulNet.cpp:89 and Application.cpp:182/189 after
 * srand(time(NULL)) at Application.cpp:50/96.  glibc is a system dependency, not part
 * of the reference tree; tests pin this restatement against the real libc rand().
 *
 *   r[0]      = seed (0 -> 1)
 *   r[i]      = 16807 * r[i-1] mod (2^31 - 1)          i = 1..30
 *   r[i]      = r[i-31]                                 i = 31..33
 *   r[i]      = r[i-31] + r[i-3]  (mod 2^32)            i >= 34
 *   rand()_k  = r[344 + k] >> 1                         k = 0, 1, ...
 */
#include "gsp_oracle.h"

void gsp_glibc_srand(gsp_glibc_rng *g, uint32_t seed) {
    int32_t r[34];
    int32_t s = (int32_t)seed;
    if (s == 0) s = 1;
    r[0] = s;
    for (int i = 1; i < 31; ++i) {
        long hi = r[i - 1] / 127773;
        long lo = r[i - 1] % 127773;
        long w = 16807 * lo - 2836 * hi;
        if (w < 0) w += 2147483647;
        r[i] = (int32_t)w;
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    for (int i = 0; i < 34; ++i) g->ring[i] = (uint32_t)r[i];
    g->pos = 34;
    for (int k = 0; k < 310; ++k) (void)gsp_glibc_rand(g);
}

int gsp_glibc_rand(gsp_glibc_rng *g) {
    /* ring of the last 34 values; slot for index i is i % 34 */
    uint32_t v = g->ring[(g->pos - 31) % 34] + g->ring[(g->pos - 3) % 34];
    g->ring[g->pos % 34] = v;
    g->pos++;
    return (int)(v >> 1);
}

/* Fill out[0..n) with the first n outputs after srand(seed). */
void gsp_glibc_stream(uint32_t seed, int32_t *out, int64_t n) {
    gsp_glibc_rng g;
    gsp_glibc_srand(&g, seed);
    for (int64_t i = 0; i < n; ++i) out[i] = gsp_glibc_rand(&g);
}
