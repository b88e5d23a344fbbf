/*
 * oracle/schedule.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * The driver policies of the build-defined scale protocols, restated once for both
 * restatements (scale_oracle.c, pview_oracle.c).  The reference hard-codes them in its driver:
 *   join schedule   node i starts at tick (int)(STEP_RATE * i)     Application.cpp:143, Params.cpp:30
 *   drop window     dropmsg on at t = 50, off at t = 300           Application.cpp:177, 198
 *   failures        one random node, or N/2 contiguous, at t = 100 Application.cpp:180-196
 * Here they are data: a start tick and a crash tick per node, and a drop percentage per send
 * tick.  A node is alive at tick t iff start <= t <= crash.
 */
#include <limits.h>
#include <string.h>

#include "gsp_oracle.h"
#include "gsp_philox.h"

void gsp_sched_start_ticks(const gsp_oracle_policy *p, int32_t n, int32_t *start) {
    for (int32_t i = 0; i < n; ++i) start[i] = p->step_rate > 0 ? (int32_t)(p->step_rate * i) : 0;
}

/* event index d enters every draw, so two events of the same tick choose independently; the
 * legacy (mode0, tick0, ppm0) event is index 0 (the draws of the single-event protocol) */
static void apply_event(int32_t n, uint64_t seed, int32_t d, int32_t mode, int32_t tick,
                        int32_t ppm, int32_t *fail) {
    const uint32_t T = (uint32_t)tick;
    if (mode == GSP_OFAIL_RANDOM) {
        for (int32_t r = 0; r < n; ++r)
            if (gsp_philox_u31(GSP_DOMAIN_FAIL, seed, T, (uint32_t)r, 0, (uint32_t)d) % 1000000u <
                (uint32_t)ppm && tick < fail[r])
                fail[r] = tick;
    } else if (mode == GSP_OFAIL_BLOCK) {
        int64_t m = (int64_t)n * ppm / 1000000;
        uint32_t start = gsp_philox_u31(GSP_DOMAIN_FAIL, seed, T, 0xFFFFFFFFu, 0, (uint32_t)d) % (uint32_t)n;
        for (int64_t i = 0; i < m; ++i) {
            int32_t r = (int32_t)((start + i) % (uint32_t)n);
            if (tick < fail[r]) fail[r] = tick;
        }
    } else if (mode == GSP_OFAIL_SINGLE) {         /* rand() % N, Application.cpp:182 */
        int32_t r = (int32_t)(gsp_philox_u31(GSP_DOMAIN_FAIL, seed, T, 0xFFFFFFFEu, 0, (uint32_t)d) %
                              (uint32_t)n);
        if (tick < fail[r]) fail[r] = tick;
    } else if (mode == GSP_OFAIL_HALF) {           /* (rand() % N) / 2 .. + N/2, :189-195 */
        int32_t first = (int32_t)(gsp_philox_u31(GSP_DOMAIN_FAIL, seed, T, 0xFFFFFFFDu, 0, (uint32_t)d) %
                                  (uint32_t)n) / 2;
        for (int32_t r = first; r < first + n / 2; ++r)
            if (tick < fail[r]) fail[r] = tick;
    }
}

void gsp_sched_fail_ticks(const gsp_oracle_policy *p, int32_t n, uint64_t seed, int32_t mode0,
                          int32_t tick0, int32_t ppm0, int32_t *fail) {
    for (int32_t r = 0; r < n; ++r) fail[r] = INT_MAX;
    apply_event(n, seed, 0, mode0, tick0, ppm0, fail);
    for (int32_t e = 0; e < p->n_fail_events && e < GSP_ORACLE_MAX_FAIL_EVENTS; ++e)
        apply_event(n, seed, e + 1, p->fail_events[e].mode, p->fail_events[e].tick,
                    p->fail_events[e].ppm, fail);
}

int32_t gsp_sched_drop(const gsp_oracle_policy *p, int32_t drop_pct, int32_t t) {
    if (t < p->drop_from) return 0;
    if (p->drop_until > 0 && t >= p->drop_until) return 0;
    return drop_pct;
}

int32_t gsp_sched_intro_ranks(const gsp_oracle_policy *p, uint64_t seed, int32_t t, int32_t j,
                              int32_t cnt, int32_t *ranks) {
    const int32_t b = p->intro_list < cnt ? p->intro_list : cnt;
    int32_t nch = 0;
    for (int32_t i = 0; i < b; ++i) {   /* sequential sampling without replacement, as peers */
        int32_t rk = (int32_t)(gsp_philox_u31(GSP_DOMAIN_JOIN, seed, (uint32_t)t, 0, (uint32_t)j,
                                              (uint32_t)i) % (uint32_t)(cnt - i));
        int32_t pos = 0;
        while (pos < nch && rk >= ranks[pos]) { rk++; pos++; }
        memmove(&ranks[pos + 1], &ranks[pos], sizeof(int32_t) * (size_t)(nch - pos));
        ranks[pos] = rk;
        nch++;
    }
    return b;
}
