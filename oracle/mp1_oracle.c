/*
 * oracle/mp1_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Sequential plain-C restatement of the reference MP1 simulator, following the
 * normative tick semantics written down in SURVEY.md 3.2.  Every rule cites the
 * reference line it restates (paths relative to /root/reference).  Output files are
 * byte-compatible with the reference's dbg.log (Log.cpp:44-130), msgcount.log
 * (EmulNet.cpp:184-220) and the end-of-tick state dump written by
 * oracle/ref_hooks.cpp.  Pinned by tests/test_oracle_golden.py against the
 * reference's committed dbg.log and against fixtures produced by oracle/_ref.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gsp_oracle.h"
#include "gsp_philox.h"

#define T_REMOVE 20          /* MP1Node.h:21                      */
#define EN_BUFF_CAP 30000    /* EmulNet.h:12                      */
#define ID_FILTER_LIMIT 10   /* MP1Node.cpp:245: id >= 0 && id < 10 */
#define MAX_TICKS 3600       /* EmulNet.h:11 MAX_TIME             */

enum { M_JOINREQ = 0, M_JOINREP = 1, M_GOSSIP = 3 }; /* MP1Node.h:31-36 */

typedef struct { int id; long hb; long ts; } entry_t;

typedef struct {
    int src, dst, type;
    entry_t *payload; /* GOSSIP: copy of the sender's list at send time (MP1Node.cpp:357) */
    int npayload;
    int dkey;         /* addr_key(dst): the destination address as strcmp() sees it */
    int st;           /* send tick */
} msg_t;

typedef struct {
    int inited, in_group, failed;
    long hb;
    entry_t *list; int nlist;       /* ordered member list (vector order)    */
    msg_t *queue; int nqueue, cap;  /* mp1q, FIFO                             */
} node_t;

typedef struct {
    int n, single_failure, drop_msg;
    double drop_prob;
    int dropmsg;                    /* Params::dropmsg                        */
    int t;
    int rng_mode;
    uint64_t seed;
    gsp_glibc_rng glibc;
    node_t *nodes;
    msg_t *buf; int nbuf;           /* EmulNet global buffer                  */
    int *sent, *recv;               /* [n+1][MAX_TICKS]                       */
    FILE *dbg;
    int log_first;                  /* first LOG call prints no address       */
    int log_magic_done;
    int cur_src, cur_dst, cur_type; /* context of the draw in flight          */
} sim_t;

/* ---------------- logging (Log.cpp) ---------------- */
static void log_line(sim_t *s, int node, const char *msg) {
    if (!s->dbg) return;
    if (!s->log_magic_done) {
        /* "%x\n" of the ASCII sum of "CS425" (Log.cpp:79-88) */
        const char *m = "CS425";
        int sum = 0;
        for (const char *p = m; *p; ++p) sum += *p;
        fprintf(s->dbg, "%x\n", sum);
        s->log_magic_done = 1;
    }
    if (s->log_first) {
        /* the else on Log.cpp:71 binds to the sprintf on :73, so the very first
         * call leaves the static address string empty */
        fprintf(s->dbg, "\n [%d] %s", s->t, msg);
        s->log_first = 0;
        return;
    }
    int id = node + 1;
    signed char b[4];
    memcpy(b, &id, 4);
    fprintf(s->dbg, "\n %d.%d.%d.%d:%d [%d] %s", b[0], b[1], b[2], b[3], 0, s->t, msg);
}

static void log_member(sim_t *s, int node, int subject_id, const char *verb) {
    signed char b[4];
    memcpy(b, &subject_id, 4);
    char line[128];
    snprintf(line, sizeof line, "Node %d.%d.%d.%d:%d %s at time %d", b[0], b[1], b[2], b[3], 0,
             verb, s->t);
    log_line(s, node, line);
}

/* ---------------- RNG ---------------- */
static int draw_send(sim_t *s) {
    if (s->rng_mode == GSP_RNG_PHILOX)
        return (int)gsp_philox_u31(GSP_DOMAIN_SEND, s->seed, (uint32_t)s->t, (uint32_t)s->cur_src,
                                   (uint32_t)s->cur_dst, (uint32_t)s->cur_type);
    return gsp_glibc_rand(&s->glibc);
}
static int draw_fail(sim_t *s) {
    if (s->rng_mode == GSP_RNG_PHILOX)
        return (int)gsp_philox_u31(GSP_DOMAIN_FAIL, s->seed, (uint32_t)s->t, 0, 0, 0);
    return gsp_glibc_rand(&s->glibc);
}

/* strcmp() over the 6-byte addresses (EmulNet.cpp:154) is C-string equality of the
 * little-endian id bytes followed by the port bytes (port 0 here): two addresses compare equal
 * iff their id bytes agree up to the first 0 byte.  addr_key keeps exactly those bytes, so the
 * buffer scan compares one int per message (equal keys <=> strcmp() == 0; e.g. ids 256 and
 * 512 share the key 0). */
static int addr_key(int id) {
    unsigned char x[7] = {0};
    memcpy(x, &id, 4);
    int key = 0;
    for (int i = 0; i < 4 && x[i]; ++i) key |= (int)x[i] << (8 * i);
    return key;
}

/* sends the last gsp_oracle_mp1_run rejected because the 30,000-message buffer was full
 * (EmulNet.cpp:92): lets the fixture tests show that a case reaches that path */
static int64_t g_buffer_full_rejects;
/* optional handling-order trace (gsp_oracle_mp1_set_queue_trace) */
static char g_trace_path[4096];
static FILE *g_trace;
void gsp_oracle_mp1_set_queue_trace(const char *path) {
    g_trace_path[0] = 0;
    if (path) snprintf(g_trace_path, sizeof g_trace_path, "%s", path);
}
int64_t gsp_oracle_mp1_buffer_full_rejects(void) { return g_buffer_full_rejects; }
/* opt-in bounded introducer list (gsp_params.intro_list; 0 = the reference) */
static int g_intro_list;
void gsp_oracle_mp1_set_intro_list(int b) { g_intro_list = b; }
/* member-entry merges of the last run: 1 + |payload| per GOSSIP handled (the exact engine's
 * gsp_exact_stats.merges) */
static int64_t g_merges;
int64_t gsp_oracle_mp1_merges(void) { return g_merges; }

/* ---------------- EmulNet (EmulNet.cpp) ---------------- */
static void en_send(sim_t *s, int src_node, int dst_id, int type, const entry_t *pl, int npl) {
    s->cur_src = src_node + 1; s->cur_dst = dst_id; s->cur_type = type;
    int r = draw_send(s);                                  /* EmulNet.cpp:89, always drawn */
    int thr = (int)(s->drop_prob * 100);                   /* EmulNet.cpp:91               */
    if (s->nbuf >= EN_BUFF_CAP) { g_buffer_full_rejects++; return; }   /* EmulNet.cpp:92 */
    if (s->dropmsg && r % 100 < thr) return;
    msg_t m = {src_node + 1, dst_id, type, NULL, 0, addr_key(dst_id), s->t};
    if (type == M_GOSSIP && npl) {
        m.payload = malloc(sizeof(entry_t) * npl);
        memcpy(m.payload, pl, sizeof(entry_t) * npl);
        m.npayload = npl;
    }
    s->buf[s->nbuf++] = m;
    s->sent[(src_node + 1) * MAX_TICKS + s->t]++;          /* EmulNet.cpp:110 */
}

static void en_recv(sim_t *s, int node) {
    node_t *nd = &s->nodes[node];
    const int key = addr_key(node + 1);
    for (int k = s->nbuf - 1; k >= 0; --k) {               /* EmulNet.cpp:151 top-down scan */
        if (s->buf[k].dkey != key) continue;               /* EmulNet.cpp:154 strcmp() */
        if (nd->nqueue == nd->cap) {
            nd->cap = nd->cap ? nd->cap * 2 : 16;
            nd->queue = realloc(nd->queue, sizeof(msg_t) * nd->cap);
        }
        nd->queue[nd->nqueue++] = s->buf[k];
        s->buf[k] = s->buf[s->nbuf - 1];                   /* swap-with-last removal */
        s->nbuf--;
        s->recv[(node + 1) * MAX_TICKS + s->t]++;          /* EmulNet.cpp:172 */
    }
}

/* ---------------- MP1Node ---------------- */
static entry_t *find(node_t *nd, int id) {               /* check_exist, MP1Node.cpp:308-326 */
    for (int i = 0; i < nd->nlist; ++i)
        if (nd->list[i].id == id) return &nd->list[i];
    return NULL;
}

static void add_from_header(sim_t *s, int node, int src_id) { /* MP1Node.cpp:265-280 */
    node_t *nd = &s->nodes[node];
    if (find(nd, src_id)) return;
    entry_t e = {src_id, 1, s->t};
    nd->list[nd->nlist++] = e;
    log_member(s, node, src_id, "joined");
}

static void add_from_entry(sim_t *s, int node, const entry_t *v) { /* MP1Node.cpp:282-301 */
    node_t *nd = &s->nodes[node];
    if (v->id == node + 1) return;
    if (s->t - v->ts < T_REMOVE) {
        log_member(s, node, v->id, "joined");
        nd->list[nd->nlist++] = *v;
    }
}

static void handle(sim_t *s, int node, msg_t *m) {       /* recvCallBack, MP1Node.cpp:219-260 */
    node_t *nd = &s->nodes[node];
    if (m->type == M_JOINREQ) {
        add_from_header(s, node, m->src);
        en_send(s, node, m->src, M_JOINREP, nd->list, nd->nlist);
    } else if (m->type == M_JOINREP) {
        add_from_header(s, node, m->src);
        nd->in_group = 1;
        if (g_intro_list > 0) {
            /* variant: merge B entries of the introducer's list as of the end of the tick it
             * replied -- its current list, since phase P runs it last (Application.cpp:138) --
             * at sequential distinct Philox ranks, with the GOSSIP payload rules */
            const node_t *in = &s->nodes[m->src - 1];
            const int cnt = in->nlist, b = g_intro_list < cnt ? g_intro_list : cnt;
            int ranks[16], nch = 0;
            for (int i = 0; i < b; ++i) {
                int rk = (int)(gsp_philox_u31(GSP_DOMAIN_JOIN, s->seed, (uint32_t)(s->t - 1), 0,
                                              (uint32_t)node, (uint32_t)i) % (uint32_t)(cnt - i));
                int pos = 0;
                while (pos < nch && rk >= ranks[pos]) { rk++; pos++; }
                memmove(&ranks[pos + 1], &ranks[pos], sizeof(int) * (size_t)(nch - pos));
                ranks[pos] = rk;
                nch++;
            }
            entry_t pick[16];
            for (int i = 0; i < nch; ++i) pick[i] = in->list[ranks[i]];   /* ascending position */
            for (int i = 0; i < nch; ++i) {
                const entry_t *v = &pick[i];
                if (!(v->id >= 0 && v->id < ID_FILTER_LIMIT)) continue;
                entry_t *x = find(nd, v->id);
                if (x) {
                    if (v->hb > x->hb) { x->hb = v->hb; x->ts = s->t; }
                } else {
                    add_from_entry(s, node, v);
                }
            }
        }
    } else if (m->type == M_GOSSIP) {
        g_merges += 1 + m->npayload;
        entry_t *e = find(nd, m->src);
        if (e) { e->hb += 1; e->ts = s->t; }
        else add_from_header(s, node, m->src);
        for (int i = 0; i < m->npayload; ++i) {
            const entry_t *v = &m->payload[i];
            if (!(v->id >= 0 && v->id < ID_FILTER_LIMIT)) continue;
            entry_t *x = find(nd, v->id);
            if (x) {
                if (v->hb > x->hb) { x->hb = v->hb; x->ts = s->t; }
            } else {
                add_from_entry(s, node, v);
            }
        }
    }
    free(m->payload);
    m->payload = NULL;
}

static void node_ops(sim_t *s, int node) {               /* nodeLoopOps, MP1Node.cpp:335-362 */
    node_t *nd = &s->nodes[node];
    nd->hb += 1;
    for (int i = nd->nlist - 1; i >= 0; --i) {
        if (s->t - nd->list[i].ts >= T_REMOVE) {
            log_member(s, node, nd->list[i].id, "removed");
            memmove(&nd->list[i], &nd->list[i + 1], sizeof(entry_t) * (nd->nlist - i - 1));
            nd->nlist--;
        }
    }
    for (int i = 0; i < nd->nlist; ++i)
        en_send(s, node, nd->list[i].id, M_GOSSIP, nd->list, nd->nlist);
}

static void node_start(sim_t *s, int node) {             /* MP1Node.cpp:67-154 */
    node_t *nd = &s->nodes[node];
    nd->failed = 0; nd->inited = 1; nd->in_group = 0; nd->hb = 0; nd->nlist = 0;
    if (node + 1 == 1) {                                   /* introducer id 1, MP1Node.cpp:382 */
        log_line(s, node, "Starting up group...");
        nd->in_group = 1;
    } else {
        log_line(s, node, "Trying to join...");
        en_send(s, node, 1, M_JOINREQ, NULL, 0);
    }
}

static void node_loop(sim_t *s, int node) {              /* MP1Node.cpp:176-212 */
    node_t *nd = &s->nodes[node];
    if (nd->failed) return;
    for (int i = 0; i < nd->nqueue; ++i) {
        if (g_trace)
            fprintf(g_trace, "%d %d %d %d %d\n", s->t, node + 1, nd->queue[i].src,
                    nd->queue[i].type, nd->queue[i].st);
        handle(s, node, &nd->queue[i]);
    }
    nd->nqueue = 0;
    if (!nd->in_group) return;
    node_ops(s, node);
}

/* ---------------- Application ---------------- */
static void app_fail(sim_t *s) {                         /* Application.cpp:173-202 */
    char line[64];
    if (s->drop_msg && s->t == 50) s->dropmsg = 1;
    if (s->single_failure && s->t == 100) {
        int victim = draw_fail(s) % s->n;
        snprintf(line, sizeof line, "Node failed at time=%d", s->t);
        log_line(s, victim, line);
        s->nodes[victim].failed = 1;
    } else if (s->t == 100) {
        int first = draw_fail(s) % s->n / 2;
        for (int i = first; i < first + s->n / 2; ++i) {
            snprintf(line, sizeof line, "Node failed at time = %d", s->t);
            log_line(s, i, line);
            s->nodes[i].failed = 1;
        }
    }
    if (s->drop_msg && s->t == 300) s->dropmsg = 0;
}

static void dump_state(sim_t *s, FILE *f) {
    for (int i = 0; i < s->n; ++i) {
        node_t *nd = &s->nodes[i];
        fprintf(f, "%d %d %d %d %d %ld %d", s->t, i + 1, nd->inited, nd->in_group, nd->failed,
                nd->hb, nd->nlist);
        for (int k = 0; k < nd->nlist; ++k)
            fprintf(f, " %d:%ld:%ld", nd->list[k].id, nd->list[k].hb, nd->list[k].ts);
        fputc('\n', f);
    }
}

static void write_msgcount(sim_t *s, const char *path) { /* EmulNet.cpp:184-220 */
    FILE *f = fopen(path, "w");
    if (!f) return;
    for (int i = 1; i <= s->n; ++i) {
        fprintf(f, "node %3d ", i);
        int st = 0, rt = 0;
        for (int j = 0; j < s->t; ++j) {
            int a = s->sent[i * MAX_TICKS + j], b = s->recv[i * MAX_TICKS + j];
            st += a; rt += b;
            if (i != 67) {
                fprintf(f, " (%4d, %4d)", a, b);
                if (j % 10 == 9) fprintf(f, "\n         ");
            } else {
                fprintf(f, "special %4d %4d %4d\n", j, a, b);
            }
        }
        fprintf(f, "\n");
        fprintf(f, "node %3d sent_total %6u  recv_total %6u\n\n", i, (unsigned)st, (unsigned)rt);
    }
    fclose(f);
}

static int read_conf(sim_t *s, const char *path) {       /* Params.cpp:19-43 */
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    int nnb = 0, single = 0, drop = 0;
    double prob = 0;
    if (fscanf(f, "MAX_NNB: %d", &nnb) != 1) nnb = 0;
    if (fscanf(f, "\nSINGLE_FAILURE: %d", &single) != 1) single = 0;
    if (fscanf(f, "\nDROP_MSG: %d", &drop) != 1) drop = 0;
    if (fscanf(f, "\nMSG_DROP_PROB: %lf", &prob) != 1) prob = 0;
    fclose(f);
    s->n = nnb; s->single_failure = single; s->drop_msg = drop; s->drop_prob = prob;
    return 0;
}

int gsp_oracle_mp1_run(const char *conf_path, uint64_t seed, int rng_mode, int ticks,
                       const char *dbg_path, const char *msgcount_path, const char *state_path,
                       const char *stdout_path) {
    sim_t s;
    memset(&s, 0, sizeof s);
    g_buffer_full_rejects = 0;
    g_merges = 0;
    g_trace = g_trace_path[0] ? fopen(g_trace_path, "w") : NULL;
    if (read_conf(&s, conf_path) != 0) return -1;
    if (s.n <= 0 || s.n > 1000 || ticks <= 0 || ticks > MAX_TICKS) return -2;
    s.rng_mode = rng_mode;
    s.seed = seed;
    gsp_glibc_srand(&s.glibc, (uint32_t)seed);  /* the second srand (Application.cpp:96) rules */
    s.nodes = calloc(s.n, sizeof(node_t));
    for (int i = 0; i < s.n; ++i) s.nodes[i].list = calloc(s.n + 1, sizeof(entry_t));
    s.buf = calloc(EN_BUFF_CAP, sizeof(msg_t));
    s.sent = calloc((size_t)(s.n + 1) * MAX_TICKS, sizeof(int));
    s.recv = calloc((size_t)(s.n + 1) * MAX_TICKS, sizeof(int));
    s.dbg = dbg_path ? fopen(dbg_path, "w") : NULL;
    FILE *st = state_path ? fopen(state_path, "w") : NULL;
    FILE *out = stdout_path ? fopen(stdout_path, "w") : NULL;
    s.log_first = 1;

    for (int i = 0; i < s.n; ++i) log_line(&s, i, "APP");  /* Application.cpp:67 */

    for (s.t = 0; s.t < ticks; ++s.t) {                    /* Application.cpp:99 */
        for (int i = 0; i < s.n; ++i)                      /* phase R, Application.cpp:125-135 */
            if (s.t > (int)(0.25 * i) && !s.nodes[i].failed) en_recv(&s, i);
        for (int i = s.n - 1; i >= 0; --i) {               /* phase P, Application.cpp:138-163 */
            if (s.t == (int)(0.25 * i)) {
                node_start(&s, i);
                if (out) fprintf(out, "%d-th introduced node is assigned with the address: %d:0\n",
                                 i, i + 1);
            } else if (s.t > (int)(0.25 * i) && !s.nodes[i].failed) {
                node_loop(&s, i);
                if (i == 0 && s.t % 500 == 0) {
                    char line[32];
                    snprintf(line, sizeof line, "@@time=%d", s.t);
                    log_line(&s, 0, line);
                }
            }
        }
        app_fail(&s);
        if (st) dump_state(&s, st);
    }
    if (msgcount_path) write_msgcount(&s, msgcount_path);

    if (s.dbg) fclose(s.dbg);
    if (g_trace) { fclose(g_trace); g_trace = NULL; }
    if (st) fclose(st);
    if (out) fclose(out);
    for (int k = 0; k < s.nbuf; ++k) free(s.buf[k].payload);
    for (int i = 0; i < s.n; ++i) {
        for (int k = 0; k < s.nodes[i].nqueue; ++k) free(s.nodes[i].queue[k].payload);
        free(s.nodes[i].list);
        free(s.nodes[i].queue);
    }
    free(s.nodes); free(s.buf); free(s.sent); free(s.recv);
    return 0;
}
