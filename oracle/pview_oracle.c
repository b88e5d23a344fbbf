/*
 * oracle/pview_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Sequential restatement of the build-defined PARTIAL-VIEW scale protocol (DESIGN.md
 * "Partial view", BASELINE config 5): every node keeps at most V member entries
 * (id, hb, ts) sorted by id.  Per-entry rules are the reference's (MP1Node.cpp:234-301,
 * 335-348) applied per id; the bounded-state choices are the build's:
 *   init      view of r = {(r + 1 + j * (n / V)) mod n : j < V} (all others if n - 1 <= V),
 *             hb = h0, ts = 0 -- among the nodes that start at tick 0;
 *   inbox     a receiver merges at most K messages per tick, in ascending sender order; the
 *             rest are counted as overflow and ignored.  K = 0 drains every message, as the
 *             reference's checkMessages does (MP1Node.cpp:200-212);
 *   evict     after the TREMOVE scan, a view larger than V keeps the V entries with the
 *             smallest (age, -hb, id);
 *   send      min(f, cnt) distinct members by Philox rank-select over the id order of the
 *             cnt gossipable members.
 * The driver policies (join schedule + bounded introducer list, drop window, failure events),
 * TFAIL suspicion and SWIM probing follow scale_oracle.c's definitions with "column order"
 * read as "id order of the view":
 *   JOINREP   node 0 -> a node starting at t + 1, payload = intro_list of node 0's gossipable
 *             members (Philox ranks, gsp_sched_intro_ranks); merged like a GOSSIP from 0;
 *   TFAIL     a payload holds the sender's members gossipable at t - 1 ((t - 1) - ts < tfail);
 *             peers, probe targets and the count are over gossipable members;
 *   SWIM      the probe target p chosen at t - 1 is resolved after the merges of t, before
 *             the TREMOVE scan: present p gets ts = t (answered) or t - TREMOVE (not).
 * Absolute int32 timestamps (the device stores ts mod 32).  The join / remove / evict events
 * of the last step are kept for the event-stream parity tests.
 */
#include <stdlib.h>
#include <string.h>

#include "gsp_oracle.h"
#include "gsp_philox.h"

enum { MSG_JOINREP = 1, MSG_GOSSIP = 3 };

typedef struct { int32_t id, hb, ts; } pv_ent;

struct gsp_pview_oracle {
    gsp_pview_cfg c;
    int32_t t;
    int cur;
    pv_ent *tab[2];      /* [n][V] */
    int32_t *len[2];     /* [n] */
    int32_t *own_hb, *fail_tick, *start_tick, *ping;
    int32_t *msrc, *mdst, *mtype;
    int64_t nmsg, mcap;
    int32_t *ev_kind, *ev_r, *ev_x;
    int64_t nev, evcap;
};

static int alive_at(const gsp_pview_oracle *o, int32_t r, int32_t t) {
    return o->start_tick[r] <= t && t <= o->fail_tick[r];
}
static int gossipable(const gsp_pview_cfg *c, int32_t t, int32_t ts) {
    return c->tfail <= 0 || t - ts < c->tfail;
}

/* Event digest term of the partial view (kinds: 1 join, 2 remove, 3 evict): S + g(x), a row
 * seed S = gsp_event_mix(kind, t, r, 0) and g(x) = ((x ^ lo32(S)) * 0x9E3779B1) >> 5 -- the
 * kernel hashes ~1000 events per row per tick, so the per-event part is one multiply (round 4;
 * the sum over a row's events is still a 64-bit checksum: the S terms are 64-bit). */
uint64_t gsp_pv_event_mix(int kind, int64_t t, int64_t r, int64_t x) {
    const uint64_t S = gsp_event_mix(kind, t, r, 0);
    return S + ((((uint32_t)x ^ (uint32_t)S) * 0x9E3779B1u) >> 5);
}

static const pv_ent *find_id(const pv_ent *l, int32_t len, int32_t id) {
    int32_t lo = 0, hi = len;
    while (lo < hi) {
        int32_t mid = (lo + hi) >> 1;
        if (l[mid].id < id) lo = mid + 1; else hi = mid;
    }
    return (lo < len && l[lo].id == id) ? &l[lo] : NULL;
}

static void push_msg(gsp_pview_oracle *o, int32_t s, int32_t d, int32_t type) {
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

/* event sink of one row step (NULL in the exported per-row helper) */
typedef struct { gsp_pview_oracle *o; } ev_sink;
static void push_event(ev_sink *sk, int32_t kind, int32_t r, int32_t x) {
    if (!sk) return;
    gsp_pview_oracle *o = sk->o;
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

/* the gossipable members of view l at tick t, in id order, and their count */
static int32_t gossip_list(const gsp_pview_cfg *c, const pv_ent *l, int32_t len, int32_t t,
                           pv_ent *out) {
    int32_t m = 0;
    for (int32_t i = 0; i < len; ++i)
        if (gossipable(c, t, l[i].ts)) {
            if (out) out[m] = l[i];
            m++;
        }
    return m;
}

static void pv_send_all(gsp_pview_oracle *o, int tab, int32_t t, gsp_pview_digest *d) {
    const gsp_pview_cfg *c = &o->c;
    const int32_t drop = gsp_sched_drop(&c->pol, c->drop_pct, t);
    o->nmsg = 0;
    int32_t chosen[64];
    pv_ent *g = malloc(sizeof(pv_ent) * (size_t)c->view);
    for (int32_t s = 0; s < c->n; ++s) {
        if (!alive_at(o, s, t)) continue;
        const pv_ent *l = o->tab[tab] + (size_t)s * c->view;
        const int32_t cnt = gossip_list(c, l, o->len[tab][s], t, g);
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
            int32_t dst = g[rk].id;
            if (d) d->sent++;
            uint32_t dr = gsp_philox_u31(GSP_DOMAIN_SEND, c->seed, (uint32_t)t, (uint32_t)s,
                                         (uint32_t)dst, 3u);
            if ((int32_t)(dr % 100u) < drop) { if (d) d->dropped++; continue; }
            push_msg(o, s, dst, MSG_GOSSIP);
        }
        if (c->swim > 0) {
            o->ping[s] = -1;
            if (cnt > 0)
                o->ping[s] = g[gsp_philox_u31(GSP_DOMAIN_PING, c->seed, (uint32_t)t, (uint32_t)s, 0,
                                              0x100) % (uint32_t)cnt].id;
        }
    }
    free(g);
    if (!alive_at(o, 0, t)) return;             /* JOINREPs to the nodes starting at t + 1 */
    for (int32_t j = 1; j < c->n; ++j) {
        if (o->start_tick[j] != t + 1) continue;
        if (d) d->sent++;
        uint32_t dr = gsp_philox_u31(GSP_DOMAIN_SEND, c->seed, (uint32_t)t, 0, (uint32_t)j, 1u);
        if ((int32_t)(dr % 100u) < drop) { if (d) d->dropped++; continue; }
        push_msg(o, 0, j, MSG_JOINREP);
    }
}

gsp_pview_oracle *gsp_pview_oracle_create(const gsp_pview_cfg *cfg) {
    if (!cfg || cfg->n < 2 || cfg->view < 1 || cfg->fanout < 1 || cfg->fanout > 60 ||
        cfg->inbox < 0 || cfg->swim < 0 || cfg->swim > 8 || cfg->pol.intro_list < 0 ||
        cfg->pol.intro_list > 16)
        return NULL;
    gsp_pview_oracle *o = calloc(1, sizeof *o);
    o->c = *cfg;
    const int32_t n = cfg->n, V = cfg->view;
    for (int b = 0; b < 2; ++b) {
        o->tab[b] = calloc((size_t)n * V, sizeof(pv_ent));
        o->len[b] = calloc(n, sizeof(int32_t));
    }
    o->own_hb = calloc(n, sizeof(int32_t));
    o->fail_tick = calloc(n, sizeof(int32_t));
    o->start_tick = calloc(n, sizeof(int32_t));
    o->ping = malloc(sizeof(int32_t) * n);
    for (int32_t r = 0; r < n; ++r) o->ping[r] = -1;
    gsp_sched_start_ticks(&cfg->pol, n, o->start_tick);
    gsp_sched_fail_ticks(&cfg->pol, n, cfg->seed, cfg->fail_mode, cfg->fail_tick, cfg->fail_ppm,
                         o->fail_tick);
    for (int32_t r = 0; r < n; ++r) {
        pv_ent *l = o->tab[0] + (size_t)r * V;
        int32_t m = 0;
        if (o->start_tick[r] != 0) { o->len[0][r] = 0; continue; }   /* a later joiner */
        if (n - 1 <= V) {
            for (int32_t x = 0; x < n; ++x)
                if (x != r && o->start_tick[x] == 0) l[m++] = (pv_ent){x, cfg->h0, 0};
        } else {
            int32_t stride = n / V;
            for (int32_t j = 0; j < V; ++j) {
                int32_t x = (int32_t)(((int64_t)r + 1 + (int64_t)j * stride) % n);
                if (o->start_tick[x] == 0) l[m++] = (pv_ent){x, cfg->h0, 0};
            }
            /* a rotation of an ascending run: sort by id */
            for (int32_t i = 1; i < m; ++i) {
                pv_ent v = l[i];
                int32_t j = i - 1;
                while (j >= 0 && l[j].id > v.id) { l[j + 1] = l[j]; j--; }
                l[j + 1] = v;
            }
        }
        o->len[0][r] = m;
    }
    o->cur = 0;
    o->t = 0;
    pv_send_all(o, 0, 0, NULL);
    return o;
}

void gsp_pview_oracle_destroy(gsp_pview_oracle *o) {
    if (!o) return;
    for (int b = 0; b < 2; ++b) { free(o->tab[b]); free(o->len[b]); }
    free(o->own_hb); free(o->fail_tick); free(o->start_tick); free(o->ping);
    free(o->msrc); free(o->mdst); free(o->mtype);
    free(o->ev_kind); free(o->ev_r); free(o->ev_x);
    free(o);
}

static int cmp_i32(const void *a, const void *b) {
    int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}

/* eviction order (age, -hb, tie key): the tie key is the id, or with evict_order 1 the id
 * rotated by the row's Philox draw (pv_rot) -- no id favoured by every row */
typedef struct { pv_ent e; int32_t age; int32_t tk; } keyed;
static int cmp_keep(const void *a, const void *b) {
    const keyed *x = a, *y = b;
    if (x->age != y->age) return x->age < y->age ? -1 : 1;
    if (x->e.hb != y->e.hb) return x->e.hb > y->e.hb ? -1 : 1;
    return (x->tk > y->tk) - (x->tk < y->tk);
}
static int32_t pv_rot(const gsp_pview_cfg *c, int32_t t, int32_t r) {
    return (int32_t)(gsp_philox_u31(GSP_DOMAIN_EVICT, c->seed, (uint32_t)t, (uint32_t)r, 0, 0) %
                     (uint32_t)c->n);
}
static int cmp_id(const void *a, const void *b) {
    const pv_ent *x = a, *y = b;
    return (x->id > y->id) - (x->id < y->id);
}

/* The reference's per-entry rules for member id x of receiver r at tick t, one message from
 * sender s whose payload holds v for x (NULL: no entry): the fold of pv_row_step and the
 * per-message merge exported below (gsp_pview_oracle_merge_msg) are both made of this. */
static inline void pv_rule(int32_t t, int32_t T, int32_t r, int32_t x, int32_t s, const pv_ent *v,
                           int *present, pv_ent *cur) {
    if (x == s) {                                   /* MP1Node.cpp:237-243 */
        if (*present) { cur->hb += 1; cur->ts = t; }
        else { *present = 1; cur->hb = 1; cur->ts = t; }
        return;
    }
    if (!v) return;
    if (*present) {                                 /* MP1Node.cpp:247-251 */
        if (v->hb > cur->hb) { cur->hb = v->hb; cur->ts = t; }
    } else if (x != r && t - v->ts < T) {           /* MP1Node.cpp:282-301 */
        *present = 1; cur->hb = v->hb; cur->ts = v->ts;
    }
}

/* nodeLoopOps' TREMOVE predicate (MP1Node.cpp:340) */
static inline int pv_expired(int32_t t, int32_t T, int32_t ts) { return t - ts >= T; }

/* One alive receiver's tick t: merge the payloads sv[j] (sorted by id, already cut to what
 * the message carries) of the k senders b[j] (ascending) into its own view, resolve the SWIM
 * probe (probe_x >= 0), TREMOVE scan, eviction to V.  Writes the new view to out (sorted by
 * id) and returns its length; adds the row's counts and event hashes to *d.  Scratch: ids /
 * res / kk of V + K (V + 1) + 1 entries each. */
static int32_t pv_row_step(const gsp_pview_cfg *c, int32_t t, int32_t r, const pv_ent *own,
                           int32_t own_len, int32_t k, const int32_t *b, const pv_ent *const *sv,
                           const int32_t *slen, int32_t probe_x, int probe_ok, pv_ent *out,
                           gsp_pview_digest *d, int32_t *ids, pv_ent *res, keyed *kk,
                           ev_sink *sk) {
    const int32_t V = c->view, T = c->tremove;
    d->delivered += k;
    /* candidate ids: own view, each sender, each payload */
    int32_t nid = 0;
    for (int32_t i = 0; i < own_len; ++i) ids[nid++] = own[i].id;
    for (int32_t j = 0; j < k; ++j) {
        ids[nid++] = b[j];
        for (int32_t i = 0; i < slen[j]; ++i) ids[nid++] = sv[j][i].id;
        d->merges += 1 + slen[j];
    }
    qsort(ids, nid, sizeof(int32_t), cmp_i32);
    int32_t nres = 0;
    for (int32_t i = 0; i < nid; ++i) {
        if (i && ids[i] == ids[i - 1]) continue;
        const int32_t x = ids[i];
        const pv_ent *e0 = find_id(own, own_len, x);
        int present = e0 != NULL;
        pv_ent cur = e0 ? *e0 : (pv_ent){x, 0, 0};
        for (int32_t j = 0; j < k; ++j)
            pv_rule(t, T, r, x, b[j], b[j] == x ? NULL : find_id(sv[j], slen[j], x), &present, &cur);
        if (!present) continue;
        if (x == probe_x) cur.ts = probe_ok ? t : t - T;   /* SWIM: the probe's answer */
        if (!e0) {
            d->joins++; d->event_hash += gsp_pv_event_mix(1, t, r, x);
            push_event(sk, 1, r, x);
        }
        if (pv_expired(t, T, cur.ts)) {                     /* MP1Node.cpp:340 */
            d->removes++; d->event_hash += gsp_pv_event_mix(2, t, r, x);
            push_event(sk, 2, r, x);
            continue;
        }
        res[nres++] = cur;
    }
    if (nres > V) {
        const int32_t m = c->evict_order ? pv_rot(c, t, r) : 0;
        for (int32_t i = 0; i < nres; ++i) {
            kk[i].e = res[i];
            kk[i].age = t - res[i].ts;
            kk[i].tk = c->evict_order ? (res[i].id - m + c->n) % c->n : res[i].id;
        }
        qsort(kk, nres, sizeof(keyed), cmp_keep);
        for (int32_t i = V; i < nres; ++i) {
            d->evicts++;
            d->event_hash += gsp_pv_event_mix(3, t, r, kk[i].e.id);
            push_event(sk, 3, r, kk[i].e.id);
        }
        for (int32_t i = 0; i < V; ++i) res[i] = kk[i].e;
        nres = V;
        qsort(res, nres, sizeof(pv_ent), cmp_id);
    }
    memcpy(out, res, sizeof(pv_ent) * nres);
    return nres;
}

/* The per-row rule above for ONE row, on views handed in by the caller (ids ascending, ts
 * absolute; no TFAIL / SWIM / JOINREP): tests recompute a sampled row of a full-size GPU run
 * from the previous tick's views and the message list.  senders: the ids that sent to r at
 * t - 1 (any order, any count: sorted here, the first K merged, the rest inbox overflow);
 * sv_*: their views, V slots each, in the order of `senders`.  Returns the new length (or -1). */
int32_t gsp_pview_oracle_row_step(const gsp_pview_cfg *c, int32_t t, int32_t r,
                                  const int32_t *own_id, const int32_t *own_hb,
                                  const int32_t *own_ts, int32_t own_len, int32_t nsend,
                                  const int32_t *senders, const int32_t *sv_id,
                                  const int32_t *sv_hb, const int32_t *sv_ts,
                                  const int32_t *sv_len, int32_t *out_id, int32_t *out_hb,
                                  int32_t *out_ts, gsp_pview_digest *d) {
    const int32_t V = c->view, K = c->inbox ? c->inbox : nsend;   /* 0: drain every message */
    if (nsend < 0 || own_len < 0 || own_len > V) return -1;
    int32_t *order = malloc(sizeof(int32_t) * (nsend ? nsend : 1));
    for (int32_t j = 0; j < nsend; ++j) order[j] = j;
    for (int32_t i = 1; i < nsend; ++i) {                  /* ascending sender id */
        int32_t v = order[i], j = i - 1;
        while (j >= 0 && senders[order[j]] > senders[v]) { order[j + 1] = order[j]; j--; }
        order[j + 1] = v;
    }
    const int32_t k = nsend < K ? nsend : K;
    d->overflow += nsend - k;
    pv_ent *own = malloc(sizeof(pv_ent) * (V ? V : 1));
    pv_ent *views = malloc(sizeof(pv_ent) * (size_t)(k ? k : 1) * V);
    const pv_ent **sv = malloc(sizeof(pv_ent *) * (k ? k : 1));
    int32_t *b = malloc(sizeof(int32_t) * (k ? k : 1)), *slen = malloc(sizeof(int32_t) * (k ? k : 1));
    for (int32_t i = 0; i < own_len; ++i) own[i] = (pv_ent){own_id[i], own_hb[i], own_ts[i]};
    for (int32_t j = 0; j < k; ++j) {
        const int32_t q = order[j];
        b[j] = senders[q];
        slen[j] = sv_len[q];
        for (int32_t i = 0; i < sv_len[q]; ++i)
            views[(size_t)j * V + i] = (pv_ent){sv_id[(size_t)q * V + i], sv_hb[(size_t)q * V + i],
                                                 sv_ts[(size_t)q * V + i]};
        sv[j] = views + (size_t)j * V;
    }
    const size_t cap = (size_t)V + (size_t)K * (V + 1) + 1;
    int32_t *ids = malloc(sizeof(int32_t) * cap);
    pv_ent *res = malloc(sizeof(pv_ent) * cap), *out = malloc(sizeof(pv_ent) * (V ? V : 1));
    keyed *kk = malloc(sizeof(keyed) * cap);
    d->node_rounds++;
    const int32_t m = pv_row_step(c, t, r, own, own_len, k, b, sv, slen, -1, 0, out, d, ids, res,
                                  kk, NULL);
    for (int32_t i = 0; i < m; ++i) { out_id[i] = out[i].id; out_hb[i] = out[i].hb; out_ts[i] = out[i].ts; }
    free(order); free(own); free(views); free(sv); free(b); free(slen); free(ids); free(res);
    free(out); free(kk);
    return m;
}

/* ---- the per-entry rules on their own, exported (tests/test_pview_rules_vs_reference.py
 * feeds them the reference's own rows in the reference's own message order) ---- */

/* Receiver r's view (ids ascending; id / hb / ts, len entries, room for cap) merges ONE
 * GOSSIP sent by s whose payload is p (ids ascending, plen entries) at tick t: pv_rule for
 * every id of the view, of the payload and s itself.  New members count into *joins.
 * Returns the new length, or -1 when it would exceed cap (no eviction here). */
int32_t gsp_pview_oracle_merge_msg(int32_t t, int32_t T, int32_t r, int32_t *id, int32_t *hb,
                                   int32_t *ts, int32_t len, int32_t cap, int32_t s,
                                   const int32_t *p_id, const int32_t *p_hb, const int32_t *p_ts,
                                   int32_t plen, int64_t *joins) {
    pv_ent *own = malloc(sizeof(pv_ent) * (size_t)(len + 1));
    pv_ent *pay = malloc(sizeof(pv_ent) * (size_t)(plen + 1));
    pv_ent *res = malloc(sizeof(pv_ent) * (size_t)(len + plen + 1));
    int32_t *ids = malloc(sizeof(int32_t) * (size_t)(len + plen + 1));
    int32_t nid = 0, nres = 0;
    for (int32_t i = 0; i < len; ++i) { own[i] = (pv_ent){id[i], hb[i], ts[i]}; ids[nid++] = id[i]; }
    for (int32_t i = 0; i < plen; ++i) { pay[i] = (pv_ent){p_id[i], p_hb[i], p_ts[i]}; ids[nid++] = p_id[i]; }
    ids[nid++] = s;
    qsort(ids, nid, sizeof(int32_t), cmp_i32);
    for (int32_t i = 0; i < nid; ++i) {
        if (i && ids[i] == ids[i - 1]) continue;
        const int32_t x = ids[i];
        const pv_ent *e0 = find_id(own, len, x);
        int present = e0 != NULL;
        pv_ent cur = e0 ? *e0 : (pv_ent){x, 0, 0};
        pv_rule(t, T, r, x, s, x == s ? NULL : find_id(pay, plen, x), &present, &cur);
        if (!present) continue;
        if (!e0 && joins) (*joins)++;
        res[nres++] = cur;
    }
    if (nres <= cap)
        for (int32_t i = 0; i < nres; ++i) { id[i] = res[i].id; hb[i] = res[i].hb; ts[i] = res[i].ts; }
    free(own); free(pay); free(res); free(ids);
    return nres <= cap ? nres : -1;
}

/* nodeLoopOps' TREMOVE scan of a view at tick t (pv_expired, MP1Node.cpp:339-348): removes
 * in place, keeps id order, counts into *removes; returns the new length. */
int32_t gsp_pview_oracle_remove_scan(int32_t t, int32_t T, int32_t *id, int32_t *hb, int32_t *ts,
                                     int32_t len, int64_t *removes) {
    int32_t m = 0;
    for (int32_t i = 0; i < len; ++i) {
        if (pv_expired(t, T, ts[i])) { if (removes) (*removes)++; continue; }
        id[m] = id[i]; hb[m] = hb[i]; ts[m] = ts[i];
        m++;
    }
    return m;
}

int gsp_pview_oracle_step(gsp_pview_oracle *o, gsp_pview_digest *d) {
    const gsp_pview_cfg *c = &o->c;
    const int32_t n = c->n, V = c->view;
    const int32_t t = o->t + 1;
    const int prev = o->cur, next = 1 - o->cur;
    memset(d, 0, sizeof *d);
    d->tick = t;
    o->nev = 0;
    ev_sink sink = {o};

    int32_t *deg = calloc((size_t)n + 1, sizeof(int32_t));
    for (int64_t m = 0; m < o->nmsg; ++m) deg[o->mdst[m] + 1]++;
    int32_t kmax = 0;                    /* the largest segment: K = 0 merges all of it */
    for (int32_t r = 0; r < n; ++r) kmax = deg[r + 1] > kmax ? deg[r + 1] : kmax;
    for (int32_t r = 0; r < n; ++r) deg[r + 1] += deg[r];
    const int32_t K = c->inbox ? c->inbox : (kmax > 0 ? kmax : 1);
    int32_t *fill = calloc(n, sizeof(int32_t));
    int32_t *bucket = malloc(sizeof(int32_t) * (o->nmsg ? o->nmsg : 1));
    for (int64_t m = 0; m < o->nmsg; ++m) {
        int32_t r = o->mdst[m];
        bucket[deg[r] + fill[r]++] = (int32_t)m;
    }
    int32_t *ids = malloc(sizeof(int32_t) * (size_t)(V + (size_t)K * (V + 1) + 1));
    pv_ent *res = malloc(sizeof(pv_ent) * (size_t)(V + (size_t)K * (V + 1) + 1));
    keyed *kk = malloc(sizeof(keyed) * (size_t)(V + (size_t)K * (V + 1) + 1));
    const pv_ent **sv = malloc(sizeof(pv_ent *) * (size_t)K);
    int32_t *slen = malloc(sizeof(int32_t) * (size_t)K), *b = malloc(sizeof(int32_t) * (size_t)K);
    pv_ent *pay = malloc(sizeof(pv_ent) * (size_t)K * V), *g0 = malloc(sizeof(pv_ent) * V);
    int32_t ranks[16];
    /* node 0's gossipable members of tick t - 1 (the JOINREP payloads draw from them) */
    const int32_t cnt0 = gossip_list(c, o->tab[prev], o->len[prev][0], t - 1, g0);
    const int32_t drop_prev = gsp_sched_drop(&c->pol, c->drop_pct, t - 1);

    for (int32_t r = 0; r < n; ++r) {
        pv_ent *out = o->tab[next] + (size_t)r * V;
        const pv_ent *own = o->tab[prev] + (size_t)r * V;
        const int32_t own_len = o->len[prev][r];
        if (!alive_at(o, r, t)) {
            memcpy(out, own, sizeof(pv_ent) * V);
            o->len[next][r] = own_len;
            continue;
        }
        d->node_rounds++;
        int32_t *mb = bucket + deg[r];
        int32_t k = deg[r + 1] - deg[r];
        for (int32_t i = 1; i < k; ++i) {               /* ascending sender */
            int32_t v = mb[i], j = i - 1;
            while (j >= 0 && o->msrc[mb[j]] > o->msrc[v]) { mb[j + 1] = mb[j]; j--; }
            mb[j + 1] = v;
        }
        if (k > K) { d->overflow += k - K; k = K; }
        for (int32_t j = 0; j < k; ++j) {               /* each message's payload */
            const int32_t m = mb[j], s = o->msrc[m];
            pv_ent *p = pay + (size_t)j * V;
            b[j] = s;
            if (o->mtype[m] == MSG_JOINREP) {
                const int32_t nb = gsp_sched_intro_ranks(&c->pol, c->seed, t - 1, r, cnt0, ranks);
                for (int32_t i = 0; i < nb; ++i) p[i] = g0[ranks[i]];
                slen[j] = nb;
            } else {
                slen[j] = gossip_list(c, o->tab[prev] + (size_t)s * V, o->len[prev][s], t - 1, p);
            }
            sv[j] = p;
        }
        int32_t probe = -1, ok = 0;
        if (c->swim > 0 && o->ping[r] >= 0) {         /* the probe sent at t - 1 */
            probe = o->ping[r];
            for (int32_t i = 0; i < c->swim; ++i)
                ok |= (int32_t)(gsp_philox_u31(GSP_DOMAIN_PING, c->seed, (uint32_t)(t - 1), (uint32_t)r,
                                               (uint32_t)probe, (uint32_t)i) % 100u) >= drop_prev;
            ok = ok && alive_at(o, probe, t);
        }
        const int32_t nres = pv_row_step(c, t, r, own, own_len, k, b, sv, slen, probe, ok, out, d,
                                         ids, res, kk, &sink);
        o->own_hb[r] += 1;
        o->len[next][r] = nres;
    }
    free(deg); free(fill); free(bucket); free(ids); free(res); free(kk); free(sv); free(slen);
    free(b); free(pay); free(g0);
    o->cur = next;
    o->t = t;
    pv_send_all(o, next, t, d);
    return 0;
}

int32_t gsp_pview_oracle_row(const gsp_pview_oracle *o, int32_t r, int32_t *id, int32_t *hb,
                             int32_t *ts) {
    if (r < 0 || r >= o->c.n) return -1;
    const pv_ent *l = o->tab[o->cur] + (size_t)r * o->c.view;
    int32_t m = o->len[o->cur][r];
    for (int32_t i = 0; i < m; ++i) {
        if (id) id[i] = l[i].id;
        if (hb) hb[i] = l[i].hb;
        if (ts) ts[i] = l[i].ts;
    }
    return m;
}

int gsp_pview_oracle_own_hb(const gsp_pview_oracle *o, int32_t r) { return o->own_hb[r]; }
int32_t gsp_pview_oracle_fail_tick(const gsp_pview_oracle *o, int32_t r) { return o->fail_tick[r]; }
int32_t gsp_pview_oracle_start_tick(const gsp_pview_oracle *o, int32_t r) { return o->start_tick[r]; }

int64_t gsp_pview_oracle_messages(const gsp_pview_oracle *o, int32_t *src, int32_t *dst,
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

int64_t gsp_pview_oracle_joinreps(const gsp_pview_oracle *o, int32_t *dst, int64_t cap) {
    int64_t k = 0;
    for (int64_t m = 0; m < o->nmsg; ++m)
        if (o->mtype[m] == MSG_JOINREP) {
            if (dst && k < cap) dst[k] = o->mdst[m];
            k++;
        }
    return k;
}

/* The join (1) / remove (2) / evict (3) events of the last step: rows ascending; within a
 * row joins and removes in id order as the fold meets them, then evictions. */
int64_t gsp_pview_oracle_events(const gsp_pview_oracle *o, int32_t *kind, int32_t *r, int32_t *x,
                                int64_t cap) {
    const int64_t k = o->nev < cap ? o->nev : cap;
    if (kind) memcpy(kind, o->ev_kind, sizeof(int32_t) * (size_t)k);
    if (r) memcpy(r, o->ev_r, sizeof(int32_t) * (size_t)k);
    if (x) memcpy(x, o->ev_x, sizeof(int32_t) * (size_t)k);
    return o->nev;
}
