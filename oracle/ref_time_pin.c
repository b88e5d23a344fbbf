/*
 * oracle/ref_time_pin.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Linked into the reference build under oracle/_ref/ so that the reference's
 * `srand(time(NULL))` (/root/reference/Application.cpp:50 and :96) becomes an input:
 * with GSP_SEED set, time() returns that value; otherwise it returns the wall clock
 * exactly as libc would.  The reference sources themselves are compiled unmodified.
 */
#include <stdlib.h>
#include <time.h>

time_t time(time_t *tloc) {
    const char *s = getenv("GSP_SEED");
    time_t v;
    if (s && *s) {
        v = (time_t)strtoll(s, NULL, 10);
    } else {
        struct timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        v = ts.tv_sec;
    }
    if (tloc) *tloc = v;
    return v;
}
