/*
 * oracle/gsp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's hot path, used only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.  The product
 * (gossip_protocol_amd/, libgossip_amd.so) never links, loads or calls anything here.
 *
 * Two restatements:
 *   gsp_oracle_mp1_run    -- the reference MP1 simulator, byte-exact (dbg.log,
 *                            msgcount.log, end-of-tick state).  Spec: SURVEY.md 3.2;
 *                            pinned against oracle/_ref (the reference compiled from
 *                            /root/reference) and the reference's committed dbg.log.
 *   gsp_scale_oracle_*    -- the build-defined scale protocol (DESIGN.md "Scale mode"),
 *                            full view, int32 hb/ts with absolute timestamps.  The reference
 *                            cannot run at these sizes (EmulNet.h:10 MAX_NODES, MP1Node.cpp:245
 *                            id<10 filter); the restatement follows the same per-entry rules.
 */
#ifndef GSP_ORACLE_H
#define GSP_ORACLE_H
#include <stdint.h>

/* ---- glibc TYPE_3 rand() stream (glibc_rand.c) ---- */
typedef struct {
    uint32_t ring[34];
    uint64_t pos;
} gsp_glibc_rng;
void gsp_glibc_srand(gsp_glibc_rng *g, uint32_t seed);
int gsp_glibc_rand(gsp_glibc_rng *g);
void gsp_glibc_stream(uint32_t seed, int32_t *out, int64_t n);

/* ---- exact MP1 restatement (mp1_oracle.c) ---- */
enum { GSP_RNG_GLIBC = 0, GSP_RNG_PHILOX = 1 };
/* Returns 0 on success, <0 on error.  Any output path may be NULL. */
int gsp_oracle_mp1_run(const char *conf_path, uint64_t seed, int rng_mode, int ticks,
                       const char *dbg_path, const char *msgcount_path, const char *state_path,
                       const char *stdout_path);

/* ---- driver policies shared by both scale restatements (schedule.c) ----
 * The reference hard-codes them in its driver (Application.cpp:143, 177-200; Params.cpp:30);
 * the scale protocols take them as data.  Same layout as gsp_policy in include/gossip/gossip.h. */
#define GSP_ORACLE_MAX_FAIL_EVENTS 8
typedef struct { int32_t tick, mode, ppm; } gsp_oracle_fail_event;
enum { GSP_OFAIL_NONE = 0, GSP_OFAIL_RANDOM = 1, GSP_OFAIL_BLOCK = 2, GSP_OFAIL_SINGLE = 3,
       GSP_OFAIL_HALF = 4 };
typedef struct {
    int32_t drop_from, drop_until;  /* drop_pct applies to sends at ticks t, from <= t < until
                                       (until <= 0: no end); Application.cpp:177, 198      */
    double step_rate;               /* join schedule: node i starts at tick (int)(step_rate i)
                                       (Application.cpp:143, Params.cpp:30); 0: pre-joined  */
    int32_t intro_list;             /* JOINREP payload bound B, 0..16 (MP1Node.cpp:221-230)  */
    int32_t n_fail_events;          /* further failure events (index e + 1 in the draws)    */
    gsp_oracle_fail_event fail_events[GSP_ORACLE_MAX_FAIL_EVENTS];
} gsp_oracle_policy;
/* start ticks / crash ticks of every node, and the drop percentage of sends at tick t */
void gsp_sched_start_ticks(const gsp_oracle_policy *p, int32_t n, int32_t *start);
void gsp_sched_fail_ticks(const gsp_oracle_policy *p, int32_t n, uint64_t seed, int32_t mode0,
                          int32_t tick0, int32_t ppm0, int32_t *fail);
int32_t gsp_sched_drop(const gsp_oracle_policy *p, int32_t drop_pct, int32_t t);
/* the B_eff = min(B, cnt) distinct ranks a JOINREP sent at tick t to joiner j carries, among
 * the introducer's cnt gossipable members (ascending); returns B_eff */
int32_t gsp_sched_intro_ranks(const gsp_oracle_policy *p, uint64_t seed, int32_t t, int32_t j,
                              int32_t cnt, int32_t *ranks);

/* ---- scale protocol restatement (scale_oracle.c) ---- */
typedef struct {
    int32_t n;          /* nodes (full view: V = n)                         */
    int32_t fanout;     /* peers per sender per tick                        */
    int32_t drop_pct;   /* drop iff philox_u31 % 100 < drop_pct             */
    int32_t tremove;    /* removal timeout (reference TREMOVE = 20)         */
    int32_t h0;         /* initial heartbeat of every pre-joined entry      */
    int32_t fail_mode;  /* 0 none, 1 per-node Bernoulli, 2 contiguous block */
    int32_t fail_tick;  /* nodes fail at the end of this tick               */
    int32_t fail_ppm;   /* failure fraction, parts per million              */
    uint64_t seed;
    int32_t tfail;      /* 0: off (the reference: TFAIL unused); else members with
                           t - ts >= tfail are suspected: not gossiped, not chosen as
                           peers, not counted (MP1Node.h:22, spec p.3)         */
    int32_t swim;       /* 0: off; s >= 1: SWIM ping/ack probing with one direct path
                           and s - 1 indirect (ping-req) paths (spec p.3)      */
    gsp_oracle_policy pol; /* drop window, join schedule + JOINREP bound, failure events */
} gsp_scale_cfg;

typedef struct {
    int64_t tick;
    int64_t node_rounds; /* nodes that ran merge+ops this tick             */
    int64_t merges;      /* sum over delivered GOSSIPs of 1 + |payload|    */
    int64_t sent;        /* GOSSIP sends attempted (after peer choice)      */
    int64_t dropped;     /* sends rejected by the drop draw                 */
    int64_t delivered;   /* messages merged by an alive receiver            */
    int64_t joins;       /* join events                                     */
    int64_t removes;     /* remove events                                   */
    uint64_t event_hash; /* sum of mix64(event key), order independent      */
} gsp_tick_digest;

typedef struct gsp_scale_oracle gsp_scale_oracle;
gsp_scale_oracle *gsp_scale_oracle_create(const gsp_scale_cfg *cfg);
void gsp_scale_oracle_destroy(gsp_scale_oracle *o);
/* Advance one tick (t = 1, 2, ...).  Fills *d.  Returns 0 on success. */
int gsp_scale_oracle_step(gsp_scale_oracle *o, gsp_tick_digest *d);
/* Row r as of the last completed tick: present/hb/ts for every column (absent: 0/0/0). */
int gsp_scale_oracle_row(const gsp_scale_oracle *o, int32_t r, uint8_t *present, int32_t *hb,
                         int32_t *ts);
int gsp_scale_oracle_own_hb(const gsp_scale_oracle *o, int32_t r);
int32_t gsp_scale_oracle_fail_tick(const gsp_scale_oracle *o, int32_t r);
/* The GOSSIP messages (src, dst) sent at the last completed tick that survived the drop
 * draw; the JOINREPs (node 0 -> joiner) separately; start / crash tick of a node. */
int64_t gsp_scale_oracle_messages(const gsp_scale_oracle *o, int32_t *src, int32_t *dst,
                                  int64_t cap);
int64_t gsp_scale_oracle_joinreps(const gsp_scale_oracle *o, int32_t *dst, int64_t cap);
int32_t gsp_scale_oracle_start_tick(const gsp_scale_oracle *o, int32_t r);
/* The join (kind 1) / remove (kind 2) events of the last step (row r, member x), rows
 * ascending, a row's joins before its removes, members ascending. */
int64_t gsp_scale_oracle_events(const gsp_scale_oracle *o, int32_t *kind, int32_t *r, int32_t *x,
                                int64_t cap);

/* OpenMP threads of the scale oracle's step and send phase (0: OpenMP's default; 1: the
 * single-threaded restatement).  Results do not depend on it. */
void gsp_oracle_set_threads(int nt);

/* The scale protocol's per-row rules (the reference's, MP1Node.cpp:237-251, 282-301, 339-348),
 * exported so tests can feed them the reference's own rows: one GOSSIP merge, and the
 * TREMOVE scan (returns the gossipable member count). */
void gsp_scale_oracle_merge_msg(int32_t n, int32_t t, int32_t T, int32_t tfail, int32_t r,
                                uint8_t *P, int32_t *H, int32_t *S, int32_t s, const uint8_t *Ps,
                                const int32_t *Hs, const int32_t *Ss, int64_t *joins,
                                uint64_t *hash);
int32_t gsp_scale_oracle_remove_scan(int32_t n, int32_t t, int32_t T, int32_t tfail, int32_t r,
                                     uint8_t *P, int32_t *H, int32_t *S, int64_t *removes,
                                     uint64_t *hash);
/* mp1 restatement: the next gsp_oracle_mp1_run writes every message a node handles, in
 * handling order, to `path` (NULL: off) as "t receiver_id src_id type send_tick" lines. */
void gsp_oracle_mp1_set_queue_trace(const char *path);
/* opt-in bounded introducer list of the exact engine (gsp_params.intro_list); 0 = reference */
void gsp_oracle_mp1_set_intro_list(int b);
int64_t gsp_oracle_mp1_merges(void);

uint64_t gsp_event_mix(int kind, int64_t t, int64_t r, int64_t x);
uint64_t gsp_pv_event_mix(int kind, int64_t t, int64_t r, int64_t x);   /* partial view */

/* ---- partial-view scale protocol restatement (pview_oracle.c) ---- */
typedef struct {
    int32_t n;          /* nodes                                                    */
    int32_t view;       /* V: entries kept per node                                 */
    int32_t fanout;
    int32_t inbox;      /* K: messages merged per node per tick (rest = overflow); 0: all */
    int32_t drop_pct, tremove, h0, fail_mode, fail_tick, fail_ppm;
    uint64_t seed;
    int32_t tfail, swim;   /* as gsp_scale_cfg */
    gsp_oracle_policy pol;
    int32_t evict_order;   /* 0: ties by id; 1: by the rotated id (x - m) mod n, m =
                              Philox(EVICT; t, r) mod n (gsp_pview_params.evict_order) */
} gsp_pview_cfg;

typedef struct {
    int64_t tick, node_rounds, merges, sent, dropped, delivered, overflow;
    int64_t joins, removes, evicts;
    uint64_t event_hash;   /* kinds: 1 join, 2 remove, 3 evict */
} gsp_pview_digest;

typedef struct gsp_pview_oracle gsp_pview_oracle;
gsp_pview_oracle *gsp_pview_oracle_create(const gsp_pview_cfg *cfg);
void gsp_pview_oracle_destroy(gsp_pview_oracle *o);
int gsp_pview_oracle_step(gsp_pview_oracle *o, gsp_pview_digest *d);
/* view of r (ascending id); returns its length */
int32_t gsp_pview_oracle_row(const gsp_pview_oracle *o, int32_t r, int32_t *id, int32_t *hb,
                             int32_t *ts);
int gsp_pview_oracle_own_hb(const gsp_pview_oracle *o, int32_t r);
int32_t gsp_pview_oracle_fail_tick(const gsp_pview_oracle *o, int32_t r);
int64_t gsp_pview_oracle_messages(const gsp_pview_oracle *o, int32_t *src, int32_t *dst,
                                  int64_t cap);
int64_t gsp_pview_oracle_joinreps(const gsp_pview_oracle *o, int32_t *dst, int64_t cap);
int32_t gsp_pview_oracle_start_tick(const gsp_pview_oracle *o, int32_t r);
/* join (1) / remove (2) / evict (3) events of the last step */
int64_t gsp_pview_oracle_events(const gsp_pview_oracle *o, int32_t *kind, int32_t *r, int32_t *x,
                                int64_t cap);
/* The per-row rule of gsp_pview_oracle_step for ONE alive row r at tick t, on views the caller
 * hands in (ids ascending, absolute ts): own view, the ids that sent to r at t - 1 (any order
 * and count: sorted, the first `inbox` merged, the rest counted as overflow) and their views
 * (`view` slots each, in the order of `senders`).  Writes r's view of tick t, returns its
 * length; adds the row's counts / event hashes to *d (node_rounds += 1). */
int32_t gsp_pview_oracle_row_step(const gsp_pview_cfg *c, int32_t t, int32_t r,
                                  const int32_t *own_id, const int32_t *own_hb,
                                  const int32_t *own_ts, int32_t own_len, int32_t nsend,
                                  const int32_t *senders, const int32_t *sv_id,
                                  const int32_t *sv_hb, const int32_t *sv_ts,
                                  const int32_t *sv_len, int32_t *out_id, int32_t *out_hb,
                                  int32_t *out_ts, gsp_pview_digest *d);
/* The partial view's per-entry rules on their own (the ones gsp_pview_oracle_step folds
 * with): one GOSSIP merged into a view (ids ascending; returns the new length, -1 past cap),
 * and the TREMOVE scan (returns the new length). */
int32_t gsp_pview_oracle_merge_msg(int32_t t, int32_t T, int32_t r, int32_t *id, int32_t *hb,
                                   int32_t *ts, int32_t len, int32_t cap, int32_t s,
                                   const int32_t *p_id, const int32_t *p_hb, const int32_t *p_ts,
                                   int32_t plen, int64_t *joins);
int32_t gsp_pview_oracle_remove_scan(int32_t t, int32_t T, int32_t *id, int32_t *hb, int32_t *ts,
                                     int32_t len, int64_t *removes);

#endif
