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
 * Driver policies (schedule.c; the reference's Application.cpp:143, 177-200 as data): a node
 * is alive from its start tick to its crash tick; sends are dropped only inside the drop
 * window.  Nodes starting at tick 0 are pre-joined (they list each other).  A later node j
 * starts with an empty list; at tick start_j - 1 the introducer (node 0, MP1Node.cpp:378-386),
 * if alive, sends it a JOINREP (drop draw: Philox(SEND; t, 0, j, 1), msgType JOINREP) whose
 * payload is a bounded introducer list -- intro_list members of the introducer's gossipable
 * list chosen by Philox (gsp_sched_intro_ranks; MP1Node.cpp:221-230 sends the whole list, and
 * its receiver ignores it, :231-233).  The receiver handles a JOINREP like a GOSSIP from
 * node 0 with that payload: the introducer enters as (1, t), the chosen members are copied if
 * fresh.  It is always node 0's only message that tick, so it merges first.
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
 * drop(t), i = 0 direct, 1..s-1 indirect ping-req relays).  Answered: r refreshes p's
 * timestamp (ts = t + 1, hb unchanged, so hb <= h0 + t still holds).  Unanswered: r declares
 * p failed -- ts = (t + 1) - TREMOVE, so the scan of the same tick removes it (one remove
 * event).  The probe target was listed when chosen and merges never remove, so it is listed
 * at resolution time.
 * Every join / remove event of the last step is kept (gsp_scale_oracle_events) for the
 * device event stream's parity tests.
 */
#include <stdlib.h>
#include <string.h>

#include <omp.h>

#include "gsp_oracle.h"
#include "gsp_philox.h"

enum { MSG_JOINREP = 1, MSG_GOSSIP = 3 };

struct gsp_scale_oracle {
    gsp_scale_cfg c;
    int32_t t;
    int cur;
    uint8_t *pres[2];
    int32_t *hb[2], *ts[2];
    int32_t *own_hb, *fail_tick, *start_tick, *cnt;
    int32_t *ping;                  /* swim: probe target of each node's last send, or -1 */
    int32_t *msrc, *mdst, *mtype;   /* messages of the last send phase (GOSSIP and JOINREP) */
    int64_t nmsg, mcap;
    int32_t *ev_kind, *ev_r, *ev_x; /* events of the last step */
    int64_t nev, evcap;
};

/* Rows are independent within a phase (every row reads only the previous tick's table), so
 * the step and the send phase run over contiguous row blocks, one per OpenMP thread; each
 * block keeps its own messages / events and the blocks are concatenated in row order, so the
 * result is the sequential one, bit for bit.  gsp_oracle_set_threads(1) gives the
 * single-threaded restatement (bench.py's CPU baseline). */
static int g_threads = 0;     /* 0: OpenMP's default */
void gsp_oracle_set_threads(int nt) { g_threads = nt > 0 ? nt : 0; }
static int oracle_threads(void) { return g_threads > 0 ? g_threads : omp_get_max_threads(); }

typedef struct { int32_t *a, *b, *c; int64_t n, cap; } triples;
static void triples_push(triples *v, int32_t a, int32_t b, int32_t c) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 1024;
        v->a = realloc(v->a, sizeof(int32_t) * v->cap);
        v->b = realloc(v->b, sizeof(int32_t) * v->cap);
        v->c = realloc(v->c, sizeof(int32_t) * v->cap);
    }
    v->a[v->n] = a; v->b[v->n] = b; v->c[v->n] = c;
    v->n++;
}
static void triples_free(triples *v) { free(v->a); free(v->b); free(v->c); }

uint64_t gsp_event_mix(int kind, int64_t t, int64_t r, int64_t x) {
    uint64_t z = ((uint64_t)kind << 62) | ((uint64_t)(t & 0xFFFFF) << 42) |
                 ((uint64_t)(r & 0x1FFFFF) << 21) | (uint64_t)(x & 0x1FFFFF);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int alive_at(const gsp_scale_oracle *o, int32_t r, int32_t t) {
    return o->start_tick[r] <= t && t <= o->fail_tick[r];
}

/* a listed member with timestamp ts is gossiped / chosen / counted at tick t */
static int gossipable(const gsp_scale_cfg *c, int32_t t, int32_t ts) {
    return c->tfail <= 0 || t - ts < c->tfail;
}

static void push_msg(gsp_scale_oracle *o, int32_t s, int32_t d, int32_t type) {
    if (o->nmsg == o->mcap) {
        o->mcap = o->mcap ? o->mcap * 2 : 1024;
        o->msrc = realloc(o->msrc, sizeof(int32_t) * o->mcap);
        o->mdst = realloc(o->mdst, sizeof(int32_t) * o->mcap);
        o->mtype = realloc(o->mtype, sizeof(int32_t) * o->mcap);
    }
    o->msrc[o->nmsg] = s;
    o->mdst[o->nmsg] = d;
    o->mtype[o->nmsg] = type;
    o->nmsg++;
}

static void push_event(gsp_scale_oracle *o, int32_t kind, int32_t r, int32_t x) {
    if (o->nev == o->evcap) {
        o->evcap = o->evcap ? o->evcap * 2 : 1024;
        o->ev_kind = realloc(o->ev_kind, sizeof(int32_t) * o->evcap);
        o->ev_r = realloc(o->ev_r, sizeof(int32_t) * o->evcap);
        o->ev_x = realloc(o->ev_x, sizeof(int32_t) * o->evcap);
    }
    o->ev_kind[o->nev] = kind;
    o->ev_r[o->nev] = r;
    o->ev_x[o->nev] = x;
    o->nev++;
}

/* rank -> column: the rk-th gossipable column of row (ps, tss) at tick t, ascending */
static int32_t column_of_rank(const gsp_scale_cfg *c, const uint8_t *ps, const int32_t *tss,
                              int32_t t, int32_t rk) {
    int32_t seen = -1;
    for (int32_t x = 0; x < c->n; ++x)
        if (ps[x] && gossipable(c, t, tss[x]) && ++seen == rk) return x;
    return -1;
}

/* Phase SEND of tick t for every alive node, reading table `tab`; then the JOINREPs the
 * introducer sends at t to the nodes that start at t + 1. */
static void send_all(gsp_scale_oracle *o, int tab, int32_t t, gsp_tick_digest *d) {
    const gsp_scale_cfg *c = &o->c;
    const int32_t n = c->n;
    const int32_t drop = gsp_sched_drop(&c->pol, c->drop_pct, t);
    o->nmsg = 0;
    const int nt = oracle_threads();
    triples *blk = calloc((size_t)nt, sizeof(triples));
    int64_t sent = 0, dropped = 0;
#pragma omp parallel num_threads(nt) reduction(+ : sent, dropped)
    {
        const int tid = omp_get_thread_num(), nth = omp_get_num_threads();
        triples *mine = &blk[tid];
        int32_t chosen[64];
        for (int32_t s = (int32_t)((int64_t)n * tid / nth); s < (int32_t)((int64_t)n * (tid + 1) / nth); ++s) {
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
                int32_t dst = column_of_rank(c, ps, tss, t, rk);
                sent++;
                uint32_t dr = gsp_philox_u31(GSP_DOMAIN_SEND, c->seed, (uint32_t)t, (uint32_t)s,
                                             (uint32_t)dst, 3u);
                if ((int32_t)(dr % 100u) < drop) {
                    dropped++;
                    continue;
                }
                triples_push(mine, s, dst, MSG_GOSSIP);
            }
            if (c->swim > 0) {  /* the probe target: one more rank-select over the same order */
                o->ping[s] = -1;
                if (cnt > 0) {
                    int32_t rk = (int32_t)(gsp_philox_u31(GSP_DOMAIN_PING, c->seed, (uint32_t)t,
                                                          (uint32_t)s, 0, 0x100) % (uint32_t)cnt);
                    o->ping[s] = column_of_rank(c, ps, tss, t, rk);
                }
            }
        }
    }
    for (int i = 0; i < nt; ++i) {       /* the blocks in row order: the sequential list */
        for (int64_t m = 0; m < blk[i].n; ++m) push_msg(o, blk[i].a[m], blk[i].b[m], blk[i].c[m]);
        triples_free(&blk[i]);
    }
    free(blk);
    if (d) { d->sent += sent; d->dropped += dropped; }
    if (!alive_at(o, 0, t)) return;             /* JOINREPs to the nodes starting at t + 1 */
    for (int32_t j = 1; j < n; ++j) {
        if (o->start_tick[j] != t + 1) continue;
        if (d) d->sent++;
        uint32_t dr = gsp_philox_u31(GSP_DOMAIN_SEND, c->seed, (uint32_t)t, 0, (uint32_t)j, 1u);
        if ((int32_t)(dr % 100u) < drop) {
            if (d) d->dropped++;
            continue;
        }
        push_msg(o, 0, j, MSG_JOINREP);
    }
}

gsp_scale_oracle *gsp_scale_oracle_create(const gsp_scale_cfg *cfg) {
    if (!cfg || cfg->n < 2 || cfg->fanout < 1 || cfg->fanout > 60 ||
        cfg->swim < 0 || cfg->swim > 8 || cfg->pol.intro_list < 0 || cfg->pol.intro_list > 16)
        return NULL;
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
    o->start_tick = calloc(n, sizeof(int32_t));
    o->cnt = calloc(n, sizeof(int32_t));
    o->ping = malloc(sizeof(int32_t) * n);
    for (int32_t r = 0; r < n; ++r) o->ping[r] = -1;
    gsp_sched_start_ticks(&cfg->pol, n, o->start_tick);
    gsp_sched_fail_ticks(&cfg->pol, n, cfg->seed, cfg->fail_mode, cfg->fail_tick, cfg->fail_ppm,
                         o->fail_tick);
    /* tick 0: the nodes that start at 0 are pre-joined: each lists the others with (h0, 0) */
    for (int32_t r = 0; r < n; ++r) {
        int32_t cnt = 0;
        for (int32_t x = 0; x < n; ++x) {
            size_t i = (size_t)r * n + x;
            const int on = x != r && o->start_tick[r] == 0 && o->start_tick[x] == 0;
            o->pres[0][i] = (uint8_t)on;
            o->hb[0][i] = on ? cfg->h0 : 0;
            o->ts[0][i] = 0;
            cnt += on;
        }
        o->cnt[r] = cnt;
    }
    o->cur = 0;
    o->t = 0;
    send_all(o, 0, 0, NULL);
    return o;
}

void gsp_scale_oracle_destroy(gsp_scale_oracle *o) {
    if (!o) return;
    for (int b = 0; b < 2; ++b) { free(o->pres[b]); free(o->hb[b]); free(o->ts[b]); }
    free(o->own_hb); free(o->fail_tick); free(o->start_tick); free(o->cnt);
    free(o->msrc); free(o->mdst); free(o->mtype); free(o->ping);
    free(o->ev_kind); free(o->ev_r); free(o->ev_x);
    free(o);
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

int gsp_scale_oracle_step(gsp_scale_oracle *o, gsp_tick_digest *d) {
    const gsp_scale_cfg *c = &o->c;
    const int32_t n = c->n, T = c->tremove;
    const int32_t t = o->t + 1;
    const int prev = o->cur, next = 1 - o->cur;
    memset(d, 0, sizeof *d);
    d->tick = t;
    o->nev = 0;

    /* bucket last tick's surviving messages by destination, ascending sender (message index
     * carried along; a JOINREP comes from node 0, which sends no GOSSIP to a joiner) */
    int32_t *deg = calloc((size_t)n + 1, sizeof(int32_t));
    for (int64_t m = 0; m < o->nmsg; ++m) deg[o->mdst[m] + 1]++;
    for (int32_t r = 0; r < n; ++r) deg[r + 1] += deg[r];
    int32_t *fill = calloc(n, sizeof(int32_t));
    int32_t *bucket = malloc(sizeof(int32_t) * (o->nmsg ? o->nmsg : 1));
    for (int64_t m = 0; m < o->nmsg; ++m) {
        int32_t r = o->mdst[m];
        bucket[deg[r] + fill[r]++] = (int32_t)m;
    }
    for (int32_t r = 0; r < n; ++r) { /* insertion sort each (tiny) bucket by sender */
        int32_t *b = bucket + deg[r];
        int32_t k = deg[r + 1] - deg[r];
        for (int32_t i = 1; i < k; ++i) {
            int32_t v = b[i], j = i - 1;
            while (j >= 0 && o->msrc[b[j]] > o->msrc[v]) { b[j + 1] = b[j]; j--; }
            b[j + 1] = v;
        }
    }

    int32_t *cnt_next = malloc(sizeof(int32_t) * n);
    const int nt = oracle_threads();
    triples *evb = calloc((size_t)nt, sizeof(triples));
    gsp_tick_digest *part = calloc((size_t)nt, sizeof(gsp_tick_digest));
#pragma omp parallel num_threads(nt)
    {
    const int tid = omp_get_thread_num(), nth = omp_get_num_threads();
    gsp_tick_digest *pd = &part[tid];
    uint8_t *Pj = malloc((size_t)n), *P0 = malloc((size_t)n);
    int32_t ranks[16];
    for (int32_t r = (int32_t)((int64_t)n * tid / nth); r < (int32_t)((int64_t)n * (tid + 1) / nth); ++r) {
        const size_t row = (size_t)r * n;
        uint8_t *P = o->pres[next] + row;
        int32_t *H = o->hb[next] + row, *S = o->ts[next] + row;
        memcpy(P, o->pres[prev] + row, n);
        memcpy(H, o->hb[prev] + row, sizeof(int32_t) * n);
        memcpy(S, o->ts[prev] + row, sizeof(int32_t) * n);
        if (!alive_at(o, r, t)) { cnt_next[r] = o->cnt[r]; continue; }
        pd->node_rounds++;
        memcpy(P0, P, n);
        for (int32_t j = deg[r]; j < deg[r + 1]; ++j) {
            const int32_t m = bucket[j], s = o->msrc[m];
            const size_t srow = (size_t)s * n;
            const uint8_t *Ps = o->pres[prev] + srow;
            const int32_t *Hs = o->hb[prev] + srow, *Ss = o->ts[prev] + srow;
            pd->delivered++;
            if (o->mtype[m] == MSG_JOINREP) {
                /* the bounded introducer list: the chosen ranks among node 0's gossipable
                 * members of tick t - 1 */
                const int32_t b = gsp_sched_intro_ranks(&c->pol, c->seed, t - 1, r, o->cnt[0], ranks);
                memset(Pj, 0, (size_t)n);
                for (int32_t i = 0; i < b; ++i) {
                    const int32_t x = column_of_rank(c, Ps, Ss, t - 1, ranks[i]);
                    if (x >= 0) Pj[x] = 1;
                }
                pd->merges += 1 + b;
                gsp_scale_oracle_merge_msg(n, t, T, 0, r, P, H, S, s, Pj, Hs, Ss, &pd->joins,
                                           &pd->event_hash);
            } else {
                pd->merges += 1 + o->cnt[s];
                /* the payload: s's members gossipable when s sent it (tick t - 1) */
                gsp_scale_oracle_merge_msg(n, t, T, c->tfail, r, P, H, S, s, Ps, Hs, Ss,
                                           &pd->joins, &pd->event_hash);
            }
        }
        if (c->swim > 0 && o->ping[r] >= 0) {   /* resolve the probe sent at t - 1 */
            const int32_t p = o->ping[r];
            const int32_t drop = gsp_sched_drop(&c->pol, c->drop_pct, t - 1);
            int ok = 0;
            for (int32_t i = 0; i < c->swim; ++i)
                ok |= (int32_t)(gsp_philox_u31(GSP_DOMAIN_PING, c->seed, (uint32_t)(t - 1), (uint32_t)r,
                                               (uint32_t)p, (uint32_t)i) % 100u) >= drop;
            if (P[p]) S[p] = (ok && alive_at(o, p, t)) ? t : t - T;
        }
        o->own_hb[r] += 1;
        for (int32_t x = 0; x < n; ++x)         /* the row's join events, then its removes */
            if (P[x] && !P0[x]) triples_push(&evb[tid], 1, r, x);
        for (int32_t x = 0; x < n; ++x)
            if (P[x] && t - S[x] >= T) triples_push(&evb[tid], 2, r, x);
        cnt_next[r] = gsp_scale_oracle_remove_scan(n, t, T, c->tfail, r, P, H, S, &pd->removes,
                                                   &pd->event_hash);
    }
    free(Pj);
    free(P0);
    }
    for (int i = 0; i < nt; ++i) {       /* digest sums; events in row order */
        d->node_rounds += part[i].node_rounds;
        d->delivered += part[i].delivered;
        d->merges += part[i].merges;
        d->joins += part[i].joins;
        d->removes += part[i].removes;
        d->event_hash += part[i].event_hash;
        for (int64_t e = 0; e < evb[i].n; ++e) push_event(o, evb[i].a[e], evb[i].b[e], evb[i].c[e]);
        triples_free(&evb[i]);
    }
    free(evb);
    free(part);
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
int32_t gsp_scale_oracle_start_tick(const gsp_scale_oracle *o, int32_t r) { return o->start_tick[r]; }

/* GOSSIP messages of the last send phase: (src, dst) pairs; JOINREPs are not listed */
int64_t gsp_scale_oracle_messages(const gsp_scale_oracle *o, int32_t *src, int32_t *dst,
                                  int64_t cap) {
    int64_t k = 0;
    for (int64_t m = 0; m < o->nmsg; ++m) {
        if (o->mtype[m] != MSG_GOSSIP) continue;
        if (k < cap) {
            if (src) src[k] = o->msrc[m];
            if (dst) dst[k] = o->mdst[m];
        }
        k++;
    }
    return k;
}

/* The JOINREPs of the last send phase (their destinations, ascending). */
int64_t gsp_scale_oracle_joinreps(const gsp_scale_oracle *o, int32_t *dst, int64_t cap) {
    int64_t k = 0;
    for (int64_t m = 0; m < o->nmsg; ++m)
        if (o->mtype[m] == MSG_JOINREP) {
            if (dst && k < cap) dst[k] = o->mdst[m];
            k++;
        }
    return k;
}

/* The join (kind 1) / remove (kind 2) events of the last step, rows ascending, joins of a
 * row before its removes, members ascending. */
int64_t gsp_scale_oracle_events(const gsp_scale_oracle *o, int32_t *kind, int32_t *r, int32_t *x,
                                int64_t cap) {
    const int64_t k = o->nev < cap ? o->nev : cap;
    if (kind) memcpy(kind, o->ev_kind, sizeof(int32_t) * (size_t)k);
    if (r) memcpy(r, o->ev_r, sizeof(int32_t) * (size_t)k);
    if (x) memcpy(x, o->ev_x, sizeof(int32_t) * (size_t)k);
    return o->nev;
}

/* exported for the known-answer tests */
void gsp_oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    gsp_philox4x32_10(ctr, key, out);
}
uint32_t gsp_oracle_draw(uint32_t domain, uint64_t seed, uint32_t a, uint32_t b, uint32_t c,
                         uint32_t d) {
    return gsp_philox_u31(domain, seed, a, b, c, d);
}
