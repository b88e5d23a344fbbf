/*
 * oracle/scale_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Sequential restatement of the build-defined scale protocol (DESIGN.md "Scale mode"),
 * full view, int32 heartbeat + ABSOLUTE int32 timestamp per entry.  The per-entry rules
 * are the reference's (paths under /root/reference):
 *   sender entry:   present -> hb += 1, ts = t; absent -> add (1, t)     MP1Node.cpp:237-243
 *   payload entry:  present -> if v.hb > hb: hb = v.hb, ts = t           MP1Node.cpp:247-251
 *                   absent  -> add a copy of v if v.id != self and
 *                              t - v.ts < TREMOVE                        MP1Node.cpp:282-301
 *   ops:            own hb += 1; remove entries with t - ts >= TREMOVE   MP1Node.cpp:337-348
 * What the reference leaves undefined at scale (it asserts N <= 1000, EmulNet.h:10, and
 * filters ids >= 10, MP1Node.cpp:245) is fixed by the build: pre-joined start, no id
 * filter, receipt in ascending sender order, Philox peer choice (fanout f, distinct
 * peers) and Philox drop/failure draws.
 * TFAIL suspicion (the reference defines TFAIL = 5, MP1Node.h:22, and never
 * uses it): with cfg.tfail > 0 a member whose heartbeat is tfail or more ticks old is
 * SUSPECTED -- still listed until TREMOVE, but left out of the payload a node gossips, of its
 * peer choice and of its member count.  The GPU engine stores entries packed
 * (hb:11 | ts mod 32:5); this restatement keeps absolute values so that parity tests
 * prove the packing loses nothing observable.
 * SWIM ping/ack probing (mp1_specifications.pdf p.3 allows it, the reference
 * does not implement it): with cfg.swim = s >= 1, every alive node r also picks ONE probe
 * target p per tick -- Philox(PING; t, r, 0, 0x100) % cnt over the same member order as its
 * gossip peers.  The probe (ping + ack, one round trip) is resolved in r's tick t + 1, after
 * r's gossip merges and before its TREMOVE scan: it is answered iff p is alive at t + 1 and
 * at least one of s paths survives its drop draw (Philox(PING; t, r, p, i) % 100 >=
 * drop_pct, i = 0 direct, 1..s-1 indirect ping-req relays).  Answered: r refreshes p's
 * timestamp (ts = t + 1, hb unchanged, so hb <= h0 + t still holds).  Unanswered: r declares
 * p failed -- ts = (t + 1) - TREMOVE, so the scan of the same tick removes it (one remove
 * event).  The probe target was listed when chosen and merges never remove, so it is listed
 * at resolution time.
 */
#include <stdlib.h>
#include <string.h>

#include "gsp_oracle.h"
#include "gsp_philox.h"

struct gsp_scale_oracle {
    gsp_scale_cfg c;
    int32_t t;
    int cur;
    uint8_t *pres[2];
    int32_t *hb[2], *ts[2];
    int32_t *own_hb, *fail_tick, *cnt;
    int32_t *ping;                  /* swim: probe target of each node's last send, or -1 */
    int32_t *msrc, *mdst;
    int64_t nmsg, mcap;
};

uint64_t gsp_event_mix(int kind, int64_t t, int64_t r, int64_t x) {
    uint64_t z = ((uint64_t)kind << 62) | ((uint64_t)(t & 0xFFFFF) << 42) |
                 ((uint64_t)(r & 0x1FFFFF) << 21) | (uint64_t)(x & 0x1FFFFF);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int alive_at(const gsp_scale_oracle *o, int32_t r, int32_t t) { return t <= o->fail_tick[r]; }

/* a listed member with timestamp ts is gossiped / chosen / counted at tick t */
static int gossipable(const gsp_scale_cfg *c, int32_t t, int32_t ts) {
    return c->tfail <= 0 || t - ts < c->tfail;
}

static void compute_fail_ticks(gsp_scale_oracle *o) {
    const gsp_scale_cfg *c = &o->c;
    for (int32_t r = 0; r < c->n; ++r) o->fail_tick[r] = 0x7FFFFFFF;
    if (c->fail_mode == 1) {
        for (int32_t r = 0; r < c->n; ++r)
            if (gsp_philox_u31(GSP_DOMAIN_FAIL, c->seed, (uint32_t)c->fail_tick, (uint32_t)r, 0, 0) %
                    1000000u < (uint32_t)c->fail_ppm)
                o->fail_tick[r] = c->fail_tick;
    } else if (c->fail_mode == 2) {
        int64_t m = (int64_t)c->n * c->fail_ppm / 1000000;
        uint32_t start = gsp_philox_u31(GSP_DOMAIN_FAIL, c->seed, (uint32_t)c->fail_tick,
                                        0xFFFFFFFFu, 0, 0) % (uint32_t)c->n;
        for (int64_t i = 0; i < m; ++i) o->fail_tick[(start + i) % c->n] = c->fail_tick;
    }
}

/* Phase SEND of tick t for every alive node, reading table `tab`. */
static void send_all(gsp_scale_oracle *o, int tab, int32_t t, gsp_tick_digest *d) {
    const gsp_scale_cfg *c = &o->c;
    const int32_t n = c->n;
    o->nmsg = 0;
    int32_t chosen[64];
    for (int32_t s = 0; s < n; ++s) {
        if (!alive_at(o, s, t)) continue;
        const uint8_t *ps = o->pres[tab] + (size_t)s * n;
        const int32_t *tss = o->ts[tab] + (size_t)s * n;
        int32_t cnt = o->cnt[s];
        int32_t keff = c->fanout < cnt ? c->fanout : cnt;
        int32_t nch = 0;
        for (int32_t k = 0; k < keff; ++k) {
            uint32_t u = gsp_philox_u31(GSP_DOMAIN_PEER, c->seed, (uint32_t)t, (uint32_t)s,
                                        (uint32_t)k, 0);
            int32_t rk = (int32_t)(u % (uint32_t)(cnt - k));
            int32_t pos = 0;
            while (pos < nch && rk >= chosen[pos]) { rk++; pos++; }
            memmove(&chosen[pos + 1], &chosen[pos], sizeof(int32_t) * (nch - pos));
            chosen[pos] = rk;
            nch++;
            /* rank -> column: rk-th gossipable column in ascending order */
            int32_t seen = -1, dst = -1;
            for (int32_t x = 0; x < n; ++x)
                if (ps[x] && gossipable(c, t, tss[x]) && ++seen == rk) { dst = x; break; }
            if (d) d->sent++;
            uint32_t dr = gsp_philox_u31(GSP_DOMAIN_SEND, c->seed, (uint32_t)t, (uint32_t)s,
                                         (uint32_t)dst, 3u);
            if ((int32_t)(dr % 100u) < c->drop_pct) {
                if (d) d->dropped++;
                continue;
            }
            if (o->nmsg == o->mcap) {
                o->mcap = o->mcap ? o->mcap * 2 : 1024;
                o->msrc = realloc(o->msrc, sizeof(int32_t) * o->mcap);
                o->mdst = realloc(o->mdst, sizeof(int32_t) * o->mcap);
            }
            o->msrc[o->nmsg] = s;
            o->mdst[o->nmsg] = dst;
            o->nmsg++;
        }
        if (c->swim > 0) {      /* the probe target: one more rank-select over the same order */
            o->ping[s] = -1;
            if (cnt > 0) {
                int32_t rk = (int32_t)(gsp_philox_u31(GSP_DOMAIN_PING, c->seed, (uint32_t)t,
                                                      (uint32_t)s, 0, 0x100) % (uint32_t)cnt);
                int32_t seen = -1;
                for (int32_t x = 0; x < n; ++x)
                    if (ps[x] && gossipable(c, t, tss[x]) && ++seen == rk) { o->ping[s] = x; break; }
            }
        }
    }
}

/* ---- the per-row rules, exported (tests/test_scale_rules_vs_reference.py feeds them the
 * reference's own rows and message order) ---- */

/* Receiver row r merges ONE GOSSIP sent by s at tick t - 1, at tick t.  P/H/S: r's row
 * (presence, hb, absolute ts) over n columns; Ps/Hs/Ss: s's row as s sent it.
 *   sender entry:  present -> hb += 1, ts = t; absent -> add (1, t)     MP1Node.cpp:237-243
 *   payload entry: present -> if v.hb > hb: hb = v.hb, ts = t           MP1Node.cpp:247-251
 *                  absent  -> add a copy of v if v.id != r, t - v.ts < T MP1Node.cpp:282-301
 * With tfail > 0 the payload holds only what s could gossip at t - 1.  Join events are
 * counted into *joins and hashed into *hash. */
void gsp_scale_oracle_merge_msg(int32_t n, int32_t t, int32_t T, int32_t tfail, int32_t r,
                                uint8_t *P, int32_t *H, int32_t *S, int32_t s, const uint8_t *Ps,
                                const int32_t *Hs, const int32_t *Ss, int64_t *joins,
                                uint64_t *hash) {
    if (P[s]) { H[s] += 1; S[s] = t; }
    else {
        P[s] = 1; H[s] = 1; S[s] = t;
        (*joins)++; *hash += gsp_event_mix(1, t, r, s);
    }
    for (int32_t x = 0; x < n; ++x) {
        if (!Ps[x] || x == s || !(tfail <= 0 || (t - 1) - Ss[x] < tfail)) continue;
        if (P[x]) {
            if (Hs[x] > H[x]) { H[x] = Hs[x]; S[x] = t; }
        } else if (x != r && t - Ss[x] < T) {
            P[x] = 1; H[x] = Hs[x]; S[x] = Ss[x];
            (*joins)++; *hash += gsp_event_mix(1, t, r, x);
        }
    }
}

/* nodeLoopOps' TREMOVE scan of row r at tick t (MP1Node.cpp:339-348): entries with
 * t - ts >= T are removed (events counted / hashed); returns the gossipable member count. */
int32_t gsp_scale_oracle_remove_scan(int32_t n, int32_t t, int32_t T, int32_t tfail, int32_t r,
                                     uint8_t *P, int32_t *H, int32_t *S, int64_t *removes,
                                     uint64_t *hash) {
    int32_t live = 0;
    for (int32_t x = 0; x < n; ++x) {
        if (!P[x]) continue;
        if (t - S[x] >= T) {
            P[x] = 0; H[x] = 0; S[x] = 0;
            (*removes)++; *hash += gsp_event_mix(2, t, r, x);
        } else {
            live += tfail <= 0 || t - S[x] < tfail;
        }
    }
    return live;
}

gsp_scale_oracle *gsp_scale_oracle_create(const gsp_scale_cfg *cfg) {
    if (!cfg || cfg->n < 2 || cfg->fanout < 1 || cfg->fanout > 60 ||
        cfg->swim < 0 || cfg->swim > 8) return NULL;
    gsp_scale_oracle *o = calloc(1, sizeof *o);
    o->c = *cfg;
    const int32_t n = cfg->n;
    size_t nn = (size_t)n * n;
    for (int b = 0; b < 2; ++b) {
        o->pres[b] = calloc(nn, 1);
        o->hb[b] = calloc(nn, sizeof(int32_t));
        o->ts[b] = calloc(nn, sizeof(int32_t));
    }
    o->own_hb = calloc(n, sizeof(int32_t));
    o->fail_tick = calloc(n, sizeof(int32_t));
    o->cnt = calloc(n, sizeof(int32_t));
    o->ping = malloc(sizeof(int32_t) * n);
    for (int32_t r = 0; r < n; ++r) o->ping[r] = -1;
    compute_fail_ticks(o);
    /* tick 0: pre-joined, every other node present with (h0, 0) */
    for (int32_t r = 0; r < n; ++r) {
        for (int32_t x = 0; x < n; ++x) {
            size_t i = (size_t)r * n + x;
            o->pres[0][i] = (x != r);
            o->hb[0][i] = (x != r) ? cfg->h0 : 0;
            o->ts[0][i] = 0;
        }
        o->cnt[r] = n - 1;
    }
    o->cur = 0;
    o->t = 0;
    send_all(o, 0, 0, NULL);
    return o;
}

void gsp_scale_oracle_destroy(gsp_scale_oracle *o) {
    if (!o) return;
    for (int b = 0; b < 2; ++b) { free(o->pres[b]); free(o->hb[b]); free(o->ts[b]); }
    free(o->own_hb); free(o->fail_tick); free(o->cnt); free(o->msrc); free(o->mdst);
    free(o->ping);
    free(o);
}

int gsp_scale_oracle_step(gsp_scale_oracle *o, gsp_tick_digest *d) {
    const gsp_scale_cfg *c = &o->c;
    const int32_t n = c->n, T = c->tremove;
    const int32_t t = o->t + 1;
    const int prev = o->cur, next = 1 - o->cur;
    memset(d, 0, sizeof *d);
    d->tick = t;

    /* bucket last tick's surviving messages by destination, ascending sender */
    int32_t *deg = calloc((size_t)n + 1, sizeof(int32_t));
    for (int64_t m = 0; m < o->nmsg; ++m) deg[o->mdst[m] + 1]++;
    for (int32_t r = 0; r < n; ++r) deg[r + 1] += deg[r];
    int32_t *fill = calloc(n, sizeof(int32_t));
    int32_t *bucket = malloc(sizeof(int32_t) * (o->nmsg ? o->nmsg : 1));
    for (int64_t m = 0; m < o->nmsg; ++m) {
        int32_t r = o->mdst[m];
        bucket[deg[r] + fill[r]++] = o->msrc[m];
    }
    for (int32_t r = 0; r < n; ++r) { /* insertion sort each (tiny) bucket */
        int32_t *b = bucket + deg[r];
        int32_t k = deg[r + 1] - deg[r];
        for (int32_t i = 1; i < k; ++i) {
            int32_t v = b[i], j = i - 1;
            while (j >= 0 && b[j] > v) { b[j + 1] = b[j]; j--; }
            b[j + 1] = v;
        }
    }

    int32_t *cnt_next = malloc(sizeof(int32_t) * n);
    for (int32_t r = 0; r < n; ++r) {
        const size_t row = (size_t)r * n;
        uint8_t *P = o->pres[next] + row;
        int32_t *H = o->hb[next] + row, *S = o->ts[next] + row;
        memcpy(P, o->pres[prev] + row, n);
        memcpy(H, o->hb[prev] + row, sizeof(int32_t) * n);
        memcpy(S, o->ts[prev] + row, sizeof(int32_t) * n);
        if (!alive_at(o, r, t)) { cnt_next[r] = o->cnt[r]; continue; }
        d->node_rounds++;
        for (int32_t j = deg[r]; j < deg[r + 1]; ++j) {
            const int32_t s = bucket[j];
            const size_t srow = (size_t)s * n;
            const uint8_t *Ps = o->pres[prev] + srow;
            const int32_t *Hs = o->hb[prev] + srow, *Ss = o->ts[prev] + srow;
            d->delivered++;
            d->merges += 1 + o->cnt[s];
            /* the payload: s's members gossipable when s sent it (tick t - 1) */
            gsp_scale_oracle_merge_msg(n, t, T, c->tfail, r, P, H, S, s, Ps, Hs, Ss, &d->joins,
                                       &d->event_hash);
        }
        if (c->swim > 0 && o->ping[r] >= 0) {   /* resolve the probe sent at t - 1 */
            const int32_t p = o->ping[r];
            int ok = 0;
            for (int32_t i = 0; i < c->swim; ++i)
                ok |= (int32_t)(gsp_philox_u31(GSP_DOMAIN_PING, c->seed, (uint32_t)(t - 1), (uint32_t)r,
                                               (uint32_t)p, (uint32_t)i) % 100u) >= c->drop_pct;
            if (P[p]) S[p] = (ok && alive_at(o, p, t)) ? t : t - T;
        }
        o->own_hb[r] += 1;
        cnt_next[r] = gsp_scale_oracle_remove_scan(n, t, T, c->tfail, r, P, H, S, &d->removes,
                                                   &d->event_hash);
    }
    memcpy(o->cnt, cnt_next, sizeof(int32_t) * n);
    free(cnt_next); free(deg); free(fill); free(bucket);
    o->cur = next;
    o->t = t;
    send_all(o, next, t, d);
    return 0;
}

int gsp_scale_oracle_row(const gsp_scale_oracle *o, int32_t r, uint8_t *present, int32_t *hb,
                         int32_t *ts) {
    if (r < 0 || r >= o->c.n) return -1;
    size_t row = (size_t)r * o->c.n;
    if (present) memcpy(present, o->pres[o->cur] + row, o->c.n);
    if (hb) memcpy(hb, o->hb[o->cur] + row, sizeof(int32_t) * o->c.n);
    if (ts) memcpy(ts, o->ts[o->cur] + row, sizeof(int32_t) * o->c.n);
    return 0;
}

int gsp_scale_oracle_own_hb(const gsp_scale_oracle *o, int32_t r) { return o->own_hb[r]; }
int32_t gsp_scale_oracle_fail_tick(const gsp_scale_oracle *o, int32_t r) { return o->fail_tick[r]; }

int64_t gsp_scale_oracle_messages(const gsp_scale_oracle *o, int32_t *src, int32_t *dst,
                                  int64_t cap) {
    int64_t k = o->nmsg < cap ? o->nmsg : cap;
    if (src) memcpy(src, o->msrc, sizeof(int32_t) * k);
    if (dst) memcpy(dst, o->mdst, sizeof(int32_t) * k);
    return o->nmsg;
}

/* exported for the known-answer tests */
void gsp_oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    gsp_philox4x32_10(ctr, key, out);
}
uint32_t gsp_oracle_draw(uint32_t domain, uint64_t seed, uint32_t a, uint32_t b, uint32_t c,
                         uint32_t d) {
    return gsp_philox_u31(domain, seed, a, b, c, d);
}
