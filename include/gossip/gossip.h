/*
 * include/gossip/gossip.h -- the drop-in boundary of the MI355X gossip-membership engine.
 *
 * Plain C ABI (extern "C", plain pointers and sizes, int status returns, no exceptions
 * and no torch/HIP types) over libgossip_amd.so.  Two engines live behind it:
 *
 *  gsp_engine  -- EXACT mode: the reference MP1 semantics, bit-exact.  The caller drives
 *                 it with the same per-tick call pattern the reference Application uses
 *                 on MP1Node/EmulNet (/root/reference/Application.cpp:121-202); the
 *                 engine batches the calls of one phase and runs them as HIP kernels
 *                 (merge = MP1Node::recvCallBack, ops = MP1Node::nodeLoopOps).  The C++
 *                 facade in <gossip/mp1_facade.hpp> keeps the reference's class and method
 *                 names on top of these entry points.
 *  gsp_scale   -- SCALE mode: the build-defined full-view protocol with the
 *                 membership table resident in HBM as packed 16-bit entries and one fused
 *                 HIP kernel per tick; rows sharded over GPUs.
 *
 * Every entry point returns GSP_OK (0) or a negative gsp_status.  gsp_last_error()
 * returns a human-readable message for the last failure on the calling thread.
 * Threading: an engine is used by one host thread at a time.  Ownership: the engine
 * owns all device and pinned memory; callers own every buffer they pass in.
 */
#ifndef GOSSIP_GOSSIP_H
#define GOSSIP_GOSSIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSP_ABI_VERSION 7

typedef enum {
    GSP_OK = 0,
    GSP_ERR_INVALID = -1,      /* bad argument                                       */
    GSP_ERR_IO = -2,           /* file could not be read / written                   */
    GSP_ERR_HIP = -3,          /* a HIP runtime call failed (no GPU, OOM, fault)      */
    GSP_ERR_ORDER = -4,        /* call order the batched engine cannot reproduce     */
    GSP_ERR_CAPACITY = -5,     /* a device buffer bound was exceeded                  */
    GSP_ERR_RCCL = -6,         /* an RCCL call failed                                  */
    GSP_ERR_RANGE = -7         /* a value would overflow its packed representation   */
} gsp_status;

const char *gsp_last_error(void);
int gsp_abi_version(void);
/* Number of visible HIP devices (0 when none); never fails. */
int gsp_device_count(void);

/* ------------------------------------------------------------------------------------
 * Replay draws.  The counter-based Philox4x32-10 the engine uses in GSP_RNG_PHILOX mode,
 * host-callable so that the reference-side EmulNet replay hook can make
 * the identical draw in place of rand() at EmulNet.cpp:89 and Application.cpp:182/189:
 *   drop draw:  gsp_replay_draw(GSP_DOMAIN_SEND, seed, tick, src_id, dst_id, msgType)
 *   fail draw:  gsp_replay_draw(GSP_DOMAIN_FAIL, seed, tick, 0, 0, 0)
 * The value is in [0, 2^31) like rand().
 * ---------------------------------------------------------------------------------- */
#define GSP_DOMAIN_SEND 0x53454E44u
#define GSP_DOMAIN_FAIL 0x4641494Cu
#define GSP_DOMAIN_PEER 0x50454552u
#define GSP_DOMAIN_PING 0x50494E47u
#define GSP_DOMAIN_JOIN 0x4A4F494Eu
uint32_t gsp_replay_draw(uint32_t domain, uint64_t seed, uint32_t a, uint32_t b, uint32_t c,
                         uint32_t d);
int gsp_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* ------------------------------------------------------------------------------------
 * Params -- /root/reference/Params.{h,cpp}.  gsp_params_from_conf parses the same
 * four-key .conf grammar as Params::setparams (Params.cpp:19-43) and fills the same
 * hard-coded values (STEP_RATE 0.25, MAX_MSG_SIZE 4000, Params.cpp:29-31).
 * ---------------------------------------------------------------------------------- */
typedef struct {
    int32_t max_nnb;            /* MAX_NNB -> EN_GPSZ, the number of peers             */
    int32_t single_failure;     /* SINGLE_FAILURE                                      */
    int32_t drop_msg;           /* DROP_MSG                                            */
    double msg_drop_prob;       /* MSG_DROP_PROB                                       */
    double step_rate;           /* STEP_RATE (join schedule), 0.25                      */
    int32_t max_msg_size;       /* MAX_MSG_SIZE, 4000                                  */
    int32_t en_buff_size;       /* EmulNet buffer bound, ENBUFFSIZE 30000 (EmulNet.h:12) */
    int32_t total_running_time; /* TOTAL_RUNNING_TIME, 700 (Application.h:27)          */
    int32_t tremove;            /* TREMOVE, 20 (MP1Node.h:21)                          */
    int32_t id_filter_limit;    /* payload filter id < limit, 10 (MP1Node.cpp:245)     */
    int32_t intro_list;         /* opt-in protocol variant, 0 = the reference: the JOINREP
                                   carries the introducer's whole list and its receiver ignores
                                   it (MP1Node.cpp:221-233).  B = 1..16: the joiner merges B
                                   entries of the introducer's list, chosen by sequential
                                   distinct Philox ranks over list order (Philox(JOIN; t - 1,
                                   0, joiner index, i), t = the handling tick), with the GOSSIP
                                   payload rules (MP1Node.cpp:244-258, id filter included); the
                                   list is the introducer's as of the end of the tick it
                                   replied (the snapshot its GOSSIPs of that tick carry)      */
} gsp_params;

int gsp_params_default(gsp_params *out);
int gsp_params_from_conf(const char *path, gsp_params *out);

/* ------------------------------------------------------------------------------------
 * EXACT engine
 * ---------------------------------------------------------------------------------- */
typedef struct gsp_engine gsp_engine;

typedef enum {
    GSP_RNG_GLIBC = 0,  /* the reference's srand(seed)/rand() stream, indexed by draw order */
    GSP_RNG_PHILOX = 1  /* counter-based replay: Philox4x32-10(seed; tick, src, dst, type)  */
} gsp_rng_mode;

typedef enum {          /* message types, /root/reference/MP1Node.h:31-36 */
    GSP_MSG_JOINREQ = 0,
    GSP_MSG_JOINREP = 1,
    GSP_MSG_GOSSIP = 3
} gsp_msg_type;

typedef enum {          /* per-node operations of one phase-P batch */
    GSP_OP_START = 0,   /* MP1Node::nodeStart     (MP1Node.cpp:67)                     */
    GSP_OP_LOOP = 1,    /* MP1Node::nodeLoop      (MP1Node.cpp:176): drain + ops if inGroup */
    GSP_OP_CHECK = 2,   /* MP1Node::checkMessages (MP1Node.cpp:200): drain only         */
    GSP_OP_OPS = 3      /* MP1Node::nodeLoopOps   (MP1Node.cpp:335)                      */
} gsp_op;

/* Create an engine for p->max_nnb nodes (<= 1024) on HIP device `device`.
 * dbg_log_path: where the dbg.log event stream is written (NULL: keep in memory only).
 * The engine assigns node i the address id i+1, port 0 (EmulNet::ENinit, EmulNet.cpp:72). */
int gsp_create(const gsp_params *p, int device, gsp_rng_mode rng, uint64_t seed,
               const char *dbg_log_path, gsp_engine **out);
int gsp_destroy(gsp_engine *e);

/* Phase R: EmulNet::ENrecv for each node in `order`, in that order (the reference calls
 * MP1Node::recvLoop for i ascending, Application.cpp:125-135).  Delivery follows the
 * reference buffer permutation (top-down scan, swap-with-last, EmulNet.cpp:151-161). */
int gsp_tick_recv(gsp_engine *e, int32_t tick, const int32_t *order, int32_t n);

/* Phase P: one batch of per-node operations, executed in `order` (the reference calls
 * them for i descending, Application.cpp:138-163).  dropmsg is Params::dropmsg at call
 * time.  A node may appear at most once per batch. */
int gsp_tick_process(gsp_engine *e, int32_t tick, const int32_t *order, const int8_t *ops,
                     int32_t n, int32_t dropmsg);

/* EmulNet::ENsend issued directly by the caller (EmulNet.cpp:87-118): one draw, the drop
 * window and buffer bound, then the message joins the buffer.  A GOSSIP's payload is the
 * sender's current member list.  Returns GSP_OK; *admitted = message size or 0. */
int gsp_send(gsp_engine *e, int32_t tick, int32_t src_node, int32_t dst_id, int32_t type,
             int32_t dropmsg, int32_t *admitted);

/* One rand() draw in the engine's global draw order (the draw Application::fail makes,
 * Application.cpp:182/189).  In Philox mode the draw is Philox(seed; tick, 0, 0, 0). */
int gsp_rand(gsp_engine *e, int32_t tick, int32_t *value);

/* srand(seed) (Application.cpp:50/96): the next draw is the first of seed's stream (glibc
 * mode: the TYPE_3 stream of srand(seed) restarts at that draw; Philox mode: seed becomes
 * the replay key).  Draws already made are not affected. */
int gsp_srand(gsp_engine *e, uint64_t seed);

/* A line from the driver into dbg.log, ordered after all work submitted before it
 * (Log::LOG, Log.cpp:44).  node < 0 prints the empty address of the very first LOG. */
int gsp_log(gsp_engine *e, int32_t node, int32_t tick, const char *text);

/* Member mirror (/root/reference/Member.h:89-122). */
typedef struct {
    int32_t id;
    int16_t port;
    int8_t inited, in_group, failed;
    int64_t heartbeat;
    int32_t n_members;
} gsp_member_view;
typedef struct {
    int32_t id;
    int16_t port;
    int64_t heartbeat;
    int64_t timestamp;
} gsp_entry;
int gsp_set_failed(gsp_engine *e, int32_t node, int32_t failed);
int gsp_get_member(gsp_engine *e, int32_t node, gsp_member_view *out);
/* The member list of `node` in list order (MemberListEntry vector order). */
int gsp_member_list(gsp_engine *e, int32_t node, gsp_entry *buf, int32_t cap, int32_t *n);
/* The member lists of n nodes with one device read: list i (list order) at buf + i * N,
 * N = max_nnb entries each, its length in lens[i]. */
int gsp_member_lists(gsp_engine *e, const int32_t *nodes, int32_t n, gsp_entry *buf,
                     int32_t *lens);

/* MP1Node::addMember on `node`'s committed list at `tick` (MP1Node.cpp:265-301), a list
 * change of its own (the list's send-time version changes as after a batch):
 *  GSP_ADD_SENDER  addMember(MessageHdr *): entry->id absent -> appended as (id, 1, tick)
 *                  with its "joined" dbg.log line; present -> nothing;
 *  GSP_ADD_COPY    addMember(MemberListEntry *): the node itself -> nothing; else, when
 *                  tick - entry->timestamp < TREMOVE, the entry is appended as given with its
 *                  "joined" line.  The reference appends without looking the id up (its
 *                  callers check_exist first); an id already listed is GSP_ERR_INVALID here,
 *                  since a list holds each id once.
 * entry: id 1..N, port 0 (heartbeat / timestamp within int32).  *added = 1 if appended. */
#define GSP_ADD_SENDER 0
#define GSP_ADD_COPY 1
int gsp_add_member(gsp_engine *e, int32_t tick, int32_t node, const gsp_entry *entry,
                   int32_t mode, int32_t *added);

/* gsp_send with the message's own list (MessageHdr::vector_list of a message the driver
 * built, MP1Node.cpp:355-359): `payload` holds n_payload entries (ids 1..N, port 0, each id
 * once), which the receiver merges instead of the sender's committed list.  payload NULL is
 * gsp_send. */
int gsp_send_list(gsp_engine *e, int32_t tick, int32_t src_node, int32_t dst_id, int32_t type,
                  int32_t dropmsg, const gsp_entry *payload, int32_t n_payload, int32_t *admitted);

/* ---- Driver-side receive: EmulNet::ENrecv with the driver's own callback and direct
 * MP1Node::recvCallBack calls (MP1Node.cpp:46, 209, 219).  The reference hands the callback
 * each message as a MessageHdr whose vector_list is the sender's list at send time
 * (MP1Node.cpp:138/227/357); these calls move such messages between the engine and the
 * driver with that list attached, so a driver can observe, drop, reorder, hold back or
 * rewrite messages and process them one at a time.  mp1_facade.hpp builds the reference's
 * ENrecv / recvCallBack / checkMessages on them. */
typedef struct {
    int32_t src_id;       /* the sender's address id (MessageHdr::addr)                    */
    int32_t type;         /* gsp_msg_type (MessageHdr::msgType)                            */
    int64_t send_batch;   /* engine-side payload version (opaque to the driver)            */
    int64_t payload_off;  /* gsp_recv_detach: first entry of the payload in `payload`      */
    int32_t payload_len;  /* payload entries (MessageHdr::vector_list.size())              */
    int32_t pad;
} gsp_queued_msg;

/* Keep each sender's send-time list while messages carry it and the sender commits a newer
 * one (off by default: a driver that runs each phase as one batch never needs it).  Needed
 * once messages can be handled in separate batches (driver callbacks, gsp_recv_callback,
 * gsp_add_member), so mp1_facade.hpp turns it on when its EmulNet is constructed: every
 * message admitted from then on holds its list, whatever receive path the driver takes
 * later. */
int gsp_payload_snapshots(gsp_engine *e, int32_t on);

/* EmulNet::ENrecv for `node` with a driver callback (EmulNet.cpp:151-173): takes the node's
 * messages off the EmulNet buffer in the reference's delivery order, counts them as received
 * at `tick` (msgcount.log), and returns them with their payloads instead of queueing them.
 * msgs == NULL: sizes only (*n messages, *n_payload entries), nothing taken.  A buffer too
 * small for the sizes is GSP_ERR_CAPACITY with nothing taken. */
int gsp_recv_detach(gsp_engine *e, int32_t tick, int32_t node, gsp_queued_msg *msgs, int32_t cap,
                    gsp_entry *payload, int64_t payload_cap, int32_t *n, int64_t *n_payload);

/* Queue::enqueue into `node`'s queue (Queue.h:22-26), processed by the node's next
 * checkMessages / nodeLoop in queue order.  payload: m->payload_len entries, ids 1..N with
 * port 0, each id once (the list the message carries); NULL: the payload is the sender's list
 * of version m->send_batch, which the engine must still hold (GSP_ERR_ORDER otherwise). */
int gsp_queue_push(gsp_engine *e, int32_t node, const gsp_queued_msg *m, const gsp_entry *payload);

/* MP1Node::recvCallBack(env, data, size) called directly (MP1Node.cpp:219-260): `node`
 * processes exactly this message now -- the merge, a JOINREP reply with its draw -- and its
 * queue is left as it was.  payload as for gsp_queue_push. */
int gsp_recv_callback(gsp_engine *e, int32_t tick, int32_t node, const gsp_queued_msg *m,
                      const gsp_entry *payload, int32_t dropmsg);

/* Every node's end-of-tick state appended to `path`, one line per node in id order:
 * "t id inited inGroup bFailed heartbeat |L| id:hb:ts ..." with the list in MemberListEntry
 * order (Member.h:89-122) -- the state format of the parity fixtures.  bFailed is the flag set
 * by gsp_set_failed (Application::fail, Application.cpp:186/194). */
int gsp_state_dump(gsp_engine *e, int32_t tick, const char *path);

/* EmulNet::ENcleanup (EmulNet.cpp:184-220): writes msgcount.log for ticks [0, tick). */
int gsp_write_msgcount(gsp_engine *e, const char *path, int32_t tick);
/* Per-(node, tick) counters: sent[(id) * ticks + t], recv likewise, id in 1..N. */
int gsp_counters(gsp_engine *e, int32_t *sent, int32_t *recv, int32_t ticks);
/* Flush buffered dbg.log bytes to disk (done automatically on destroy). */
int gsp_flush_log(gsp_engine *e);
/* Copy the whole dbg.log byte stream produced so far. *n receives the full size. */
int gsp_log_bytes(gsp_engine *e, char *buf, size_t cap, size_t *n);

typedef struct {
    int64_t batches;            /* phase-P batches executed on the device             */
    int64_t node_rounds;        /* GSP_OP_LOOP operations executed                      */
    int64_t merges;             /* member-entry merges: 1 + |payload| per GOSSIP        */
    int64_t draws;              /* rand() draws consumed                                */
    int64_t sends_admitted;     /* messages appended to the EmulNet buffer             */
    double device_ms;           /* time inside the exact-mode kernels (HIP events)     */
} gsp_exact_stats;
int gsp_exact_stats_get(gsp_engine *e, gsp_exact_stats *out);

/* ------------------------------------------------------------------------------------
 * Driver policies of the scale engines.  The reference hard-codes them in
 * its driver -- node i starts at tick (int)(STEP_RATE * i) (Application.cpp:143,
 * Params.cpp:30), messages are dropped from the end of t = 50 to the end of t = 300, i.e.
 * the sends of ticks [51, 301) (Application.cpp:177, 198: fail() sets and clears the flag
 * after that tick's mp1Run), one random node or N/2 contiguous nodes crash at t = 100 (Application.cpp:180-196);
 * the scale engines take them as data, run on the device.  All zeros = the pre-joined,
 * always-dropping, single-event protocol of ABI 2.
 * ---------------------------------------------------------------------------------- */
#define GSP_MAX_FAIL_EVENTS 8
typedef enum {
    GSP_FAIL_NONE = 0,
    GSP_FAIL_RANDOM = 1,   /* each node with probability ppm / 10^6                        */
    GSP_FAIL_BLOCK = 2,    /* n * ppm / 10^6 contiguous nodes from a Philox start (wrapping) */
    GSP_FAIL_SINGLE = 3,   /* one node: Philox % n (Application.cpp:182)                    */
    GSP_FAIL_HALF = 4      /* n / 2 contiguous nodes from (Philox % n) / 2 (Application.cpp:189) */
} gsp_fail_mode;
typedef struct {
    int32_t tick;          /* the nodes crash at the end of this tick                       */
    int32_t mode;          /* gsp_fail_mode                                                 */
    int32_t ppm;           /* fraction for RANDOM / BLOCK, parts per million                */
} gsp_fail_event;
typedef struct {
    int32_t drop_from, drop_until;  /* drop_pct applies to the sends of ticks t with
                                       drop_from <= t < drop_until (drop_until <= 0: no end) */
    double step_rate;               /* join schedule: node i starts at tick (int)(step_rate * i);
                                       0: every node pre-joined.  Nodes starting at 0 list each
                                       other; a later node starts with an empty list and, one
                                       tick before, node 0 (the introducer, MP1Node.cpp:378-386)
                                       sends it a JOINREP if alive (drop draw Philox(SEND; t, 0,
                                       j, JOINREP)).  The JOINREP merges like a GOSSIP from node
                                       0 whose payload is the bounded introducer list below.   */
    int32_t intro_list;             /* JOINREP payload bound B (0..16): B members of node 0's
                                       gossipable list, Philox-chosen (Philox(JOIN; t, 0, j, i)
                                       sequential distinct ranks) -- MP1Node.cpp:221-230 sends
                                       the whole list and its receiver ignores it (:231-233)   */
    int32_t n_fail_events;          /* further crash events, applied after the one of
                                       (fail_mode, fail_tick, fail_ppm); event e draws with
                                       index e + 1                                           */
    gsp_fail_event fail_events[GSP_MAX_FAIL_EVENTS];
} gsp_policy;

/* The crash tick of every node under a failure schedule -- the first event (mode, tick, ppm of
 * gsp_scale_params / gsp_pview_params) and policy's further events, with the engines' own
 * Philox draws; INT32_MAX = never.  Host only (no device needed): lets a driver know which
 * nodes crashed, e.g. to measure failure detection from the event stream.  pol may be NULL. */
int gsp_fail_schedule(const gsp_policy *pol, int32_t n, uint64_t seed, int32_t mode, int32_t tick,
                      int32_t ppm, int32_t *out);

/* ------------------------------------------------------------------------------------
 * SCALE engine (full view, packed entries, device-resident tick loop)
 * ---------------------------------------------------------------------------------- */
typedef struct gsp_scale gsp_scale;

typedef struct {
    int32_t n;          /* nodes; full view V = n                                     */
    int32_t fanout;     /* peers per sender per tick (distinct), 1..16                 */
    int32_t drop_pct;   /* a send is dropped iff Philox % 100 < drop_pct               */
    int32_t tremove;    /* TREMOVE (20)                                                */
    int32_t h0;         /* initial heartbeat of every pre-joined entry (>= 1)          */
    int32_t fail_mode;  /* 0 none, 1 per-node Bernoulli(fail_ppm), 2 contiguous block  */
    int32_t fail_tick;  /* failed nodes stop after this tick                           */
    int32_t fail_ppm;   /* failure fraction in parts per million                       */
    uint64_t seed;
    int32_t max_ticks;  /* bound for digest storage; hb must stay <= 2047 (h0+ticks)   */
    int32_t tfail;      /* TFAIL suspicion (MP1Node.h:22, unused by the reference): 0 off;
                           1..tremove-1: a member whose heartbeat is tfail or more ticks
                           old is suspected -- listed until TREMOVE but not gossiped, not
                           chosen as a peer and not counted (DESIGN.md "Scale mode")   */
    int32_t swim;       /* SWIM ping/ack probing (spec p.3, not in the reference): 0 off;
                           s = 1..8: each node probes one member per tick over 1 direct +
                           s - 1 indirect paths; answered -> ts refreshed, unanswered ->
                           removed at the next tick (DESIGN.md "Scale mode"); every
                           layout                                                      */
    gsp_policy policy;  /* join schedule + bounded introducer list, drop window, crash
                           events (all zero: off)                                      */
    int32_t events;     /* event stream (Log.cpp:116-130's lines at scale), drained with
                           gsp_scale_drain_events: 0 off, GSP_EVENTS_ALL, or an OR of
                           GSP_EVENTS_JOIN / GSP_EVENTS_REMOVE                          */
    int64_t event_cap;  /* ring capacity in events (0: 2^24; rounded up to a multiple of
                           256, split evenly over 256 stripes)                          */
} gsp_scale_params;

/* params.events: which records the tick kernels keep (bit k = record kind k) */
#define GSP_EVENTS_ALL 1      /* every kind the engine has                              */
#define GSP_EVENTS_JOIN 2     /* kind 1: r added x (MP1Node.cpp:276, 297)               */
#define GSP_EVENTS_REMOVE 4   /* kind 2: r removed x after TREMOVE (MP1Node.cpp:343)    */
#define GSP_EVENTS_EVICT 8    /* kind 3: r's bounded view evicted x (partial view only) */

typedef struct {
    int64_t tick, node_rounds, merges, sent, dropped, delivered, joins, removes;
    uint64_t event_hash;   /* sum over events of mix64(kind, t, r, x), order independent */
} gsp_scale_digest;

typedef struct {
    int64_t ticks;            /* ticks stepped                                        */
    int64_t merge_launches;   /* fused tick-kernel launches timed                     */
    double merge_ms;          /* sum of fused tick-kernel durations (HIP events)      */
    double csr_ms;            /* sum of CSR build kernel durations                    */
    double bytes_per_tick;    /* algorithmic HBM bytes of the fused kernel, last tick  */
    double xgmi_bytes;        /* bytes this engine's shards sent to other shards, summed
                                 over ticks (0 on one GPU)                              */
} gsp_scale_perf;

/* Scale parameters from a .conf: the reference's four keys exactly as Params::setparams reads
 * them (Params.cpp:22-25; every reference testcase parses unchanged) mapped as its driver uses
 * them -- n = MAX_NNB, SINGLE_FAILURE 1: one Philox-chosen node crashes at t = 100, 0: n/2
 * contiguous nodes (Application.cpp:180-196), DROP_MSG: drop_pct = (int)(MSG_DROP_PROB * 100)
 * for the sends of ticks [51, 301) (EmulNet.cpp:91; Application.cpp:177/198 set and clear
 * dropmsg at the end of t = 50 / 300), STEP_RATE 0.25, 700 ticks -- then
 * optional "KEY: value" lines: SCALE_N FANOUT TREMOVE TFAIL SWIM H0 SEED TICKS STEP_RATE
 * INTRO_LIST DROP_PCT DROP_WINDOW(from until) FAIL(tick mode ppm, repeatable) EVENTS EVENT_CAP,
 * and for the partial view VIEW INBOX.  Unknown keys fail with GSP_ERR_INVALID. */
int gsp_scale_params_from_conf(const char *path, gsp_scale_params *out);
/* sizeof of a public struct by name ("gsp_scale_params", ...; 0 if unknown): lets a binding
 * check its layout */
int64_t gsp_struct_size(const char *name);

/* Single-GPU engine on `device` (rows [0, n), full rows, fused tick kernel). */
int gsp_scale_create(const gsp_scale_params *p, int device, gsp_scale **out);

/* Column-sharded job (DESIGN.md "Multi-GPU").  Shard g of G owns columns
 * [g * W, (g + 1) * W) of every row (W = n rounded up to 2048 * G, divided by G); per tick
 * the shards exchange only per-row member counts (all-gather) and the resolved peer
 * choices (all-reduce MAX).
 *   gsp_scale_nccl_id      rank 0 makes the RCCL unique id (NCCL_UNIQUE_ID_BYTES = 128);
 *                          the caller broadcasts it (e.g. torch.distributed) to every rank
 *   gsp_scale_create_rank  one process per GPU: this process holds shard `rank` of `world`
 *   gsp_scale_create_group every shard inside this process on one device, exchanged by
 *                          device copies (the same kernels and protocol, for testing the
 *                          sharded path on a single GPU)
 * Results are identical to gsp_scale_create for any number of shards. */
int gsp_scale_nccl_id(void *out, size_t cap);
int gsp_scale_create_rank(const gsp_scale_params *p, int device, int32_t rank, int32_t world,
                          const void *nccl_id, gsp_scale **out);
int gsp_scale_create_group(const gsp_scale_params *p, int device, int32_t shards,
                           gsp_scale **out);
/* One process per GPU with `tiles` column tiles per rank: the job has world * tiles column
 * shards, rank r holds shards [r * tiles, (r + 1) * tiles) and runs them as one GPU's tiles
 * (shared CSR / counts / picks, DESIGN.md "Column tiles"); the ranks exchange the counts of
 * their tiles (all-gather) and the picks (all-reduce MAX) over RCCL.  Results are identical to
 * gsp_scale_create. */
int gsp_scale_create_rank_tiled(const gsp_scale_params *p, int device, int32_t rank, int32_t world,
                                int32_t tiles, const void *nccl_id, gsp_scale **out);
/* Sharding layout of a multi-shard job.
 *   GSP_SHARD_COLUMNS  shard g owns a column slice of every row (above; O(n) exchange)
 *   GSP_SHARD_ROWS     shard g owns rows [floor(g n / G), floor((g + 1) n / G)); each tick the
 *                      sender rows that messages carry to another shard move there once per
 *                      (sender, shard) by RCCL send/recv, with the message records, and the
 *                      member counts of every row are broadcast (DESIGN.md "Multi-GPU").
 * Results are identical to gsp_scale_create in both layouts.  In the row layout
 * gsp_scale_row / gsp_scale_own_hb fail with GSP_ERR_INVALID for a row another rank holds and
 * gsp_scale_messages returns the slots of the rows held here, in row order. */
typedef enum { GSP_SHARD_COLUMNS = 0, GSP_SHARD_ROWS = 1 } gsp_shard_layout;
int gsp_scale_create_rank_layout(const gsp_scale_params *p, int device, int32_t rank,
                                 int32_t world, const void *nccl_id, int32_t layout, gsp_scale **out);
int gsp_scale_create_group_layout(const gsp_scale_params *p, int device, int32_t shards,
                                  int32_t layout, gsp_scale **out);
/* shards of the job, first shard index held by this engine, columns per shard (row layout:
 * the full row stride) */
int gsp_scale_layout(gsp_scale *s, int32_t *shards, int32_t *rank, int64_t *stride);
int gsp_scale_destroy(gsp_scale *s);
/* Advance `ticks` ticks on the device (no host synchronisation inside). */
int gsp_scale_step(gsp_scale *s, int32_t ticks);
/* Wait for all submitted work. */
int gsp_scale_sync(gsp_scale *s);
/* Current tick (last completed). */
int gsp_scale_tick(gsp_scale *s, int32_t *tick);
/* Digest of tick t (1 <= t <= current tick). */
int gsp_scale_digest_get(gsp_scale *s, int32_t t, gsp_scale_digest *out);
/* Row r of the current table, packed entries (hb << 5 | ts mod 32; 0 = absent). */
int gsp_scale_row(gsp_scale *s, int32_t r, uint16_t *buf, int32_t cap);
int gsp_scale_own_hb(gsp_scale *s, int32_t r, int32_t *hb);
/* Surviving messages sent at the current tick: dst per (src, k) slot, -1 = none/dropped. */
int gsp_scale_messages(gsp_scale *s, int32_t *dst, int64_t cap, int64_t *n);
int gsp_scale_perf_get(gsp_scale *s, gsp_scale_perf *out);
/* Enable/disable per-launch HIP event timing (default on). */
int gsp_scale_set_timing(gsp_scale *s, int32_t on);
/* Cache policy of the row streams of the fused tick kernel: bit 0 = non-temporal loads
 * and stores of the receiver's own row, bit 1 = non-temporal loads of sender rows, bit 2 =
 * software-pipelined chunk loads (with bit 0 and the packed merge; default 5).
 * Results are identical for every policy; only speed differs. */
int gsp_scale_set_cache_policy(gsp_scale *s, int32_t policy);
/* Merge arithmetic: 1 = packed 16-bit (two entries per v_pk_* instruction, default),
 * 0 = one entry at a time.  Identical results. */
int gsp_scale_set_merge(gsp_scale *s, int32_t packed);
/* The hipStream_t (as void*) every launch of this engine is ordered on, so a caller can
 * bracket a timed region with its own HIP events on the same stream. */
int gsp_scale_hip_stream(gsp_scale *s, void **stream);

/* ------------------------------------------------------------------------------------
 * Event stream (params.events != 0): the tick kernels append every join / remove (partial
 * view: and evict) of the selected kinds as one 64-bit record kind << 62 | t << 42 | r << 21
 * | x (kind 1 join, 2 remove, 3 evict; r = the node whose list changed, x = the member) --
 * the scale form of Log::logNodeAdd / logNodeRemove (Log.cpp:116-130).  A row's records are
 * staged in LDS and reserved in the ring at once; the ring is 256 stripes (row % 256), each
 * with its own counter, so reservations do not queue on one address.
 * drain: copies the records of every tick since the last drain (stripe by stripe, device
 * order within a stripe) into buf, at most cap of them, sets *n to the number copied and
 * *lost to the records a full stripe could not hold plus those past cap, and empties the
 * ring; buf = NULL only counts (*n = the records held; the ring is kept).
 * ---------------------------------------------------------------------------------- */
int gsp_scale_drain_events(gsp_scale *s, uint64_t *buf, int64_t cap, int64_t *n, int64_t *lost);
/* Appends event records as the reference's dbg.log lines (Log.cpp:44-130): "\n <r> [t] Node
 * <x> joined at time t" ("removed", "evicted"), addresses printed as Log.cpp:73 does (id =
 * index + 1 in signed bytes, port 0), in a canonical order -- t ascending, r descending (the
 * phase-P order of Application.cpp:138), joins then removes then evictions, x ascending.  A
 * new file starts with the "131" header (Log.cpp:79-88).  ev is sorted in place. */
int gsp_events_write_log(uint64_t *ev, int64_t n, const char *path);

/* ------------------------------------------------------------------------------------
 * PARTIAL-VIEW engine (BASELINE config 5): every node keeps at most `view` member entries
 * (id, hb, ts) sorted by id; a receiver merges at most `inbox` messages per tick (1..7,
 * ascending sender; the rest are counted as overflow) -- or, with inbox = 0, every message it
 * was sent, as the reference's checkMessages drains its queue (MP1Node.cpp:200-212; every
 * protocol option, for n <= 2^21 - 768: the hub kernel's buffers hold any receiver's list);
 * after the TREMOVE scan a view larger than `view` keeps the entries with the smallest
 * (age, -hb, id).  DESIGN.md "Partial view".
 * ---------------------------------------------------------------------------------- */
typedef struct gsp_pview gsp_pview;

typedef struct {
    int32_t n, view, fanout, inbox, drop_pct, tremove, h0, fail_mode, fail_tick, fail_ppm;
    uint64_t seed;
    int32_t max_ticks;
    int32_t tfail, swim;  /* as gsp_scale_params: TFAIL suspicion, SWIM probing (0: off)   */
    gsp_policy policy;    /* as gsp_scale_params                                         */
    int32_t events;       /* as gsp_scale_params, with GSP_EVENTS_EVICT (gsp_pview_drain_events) */
    int64_t event_cap;    /* as gsp_scale_params                                          */
    int32_t evict_order;  /* 0: a view past `view` keeps the smallest (age, -hb, id) -- the
                             default, and the order every headline number is quoted on; 1:
                             ties of (age, hb) broken by the rotated id (id - m) mod n, m =
                             Philox(EVICT; t, r) mod n, so no id is favoured (the id order makes
                             low ids hubs) */
} gsp_pview_params;

typedef struct {
    int64_t tick, node_rounds, merges, sent, dropped, delivered, overflow, joins, removes, evicts;
    uint64_t event_hash;   /* sum of h(kind, t, r, x) = mix64(kind, t, r, 0) + a 3-multiply
                              finaliser of x (oracle: gsp_pv_event_mix); kinds 1 join,
                              2 remove, 3 evict */
} gsp_pview_digest;

/* As gsp_scale_params_from_conf, plus the VIEW / INBOX keys (defaults 256 / 7). */
int gsp_pview_params_from_conf(const char *path, gsp_pview_params *out);
int gsp_pview_create(const gsp_pview_params *p, int device, gsp_pview **out);
/* Row-sharded job (DESIGN.md "Partial view, row shards").  Shard g of G owns the views of
 * nodes [floor(g n / G), floor((g + 1) n / G)); per tick every sender view that a message
 * carries to another shard moves there once per (sender, shard), with the message records,
 * by RCCL send/recv (one process per GPU: gsp_pview_create_rank, RCCL id from
 * gsp_scale_nccl_id) or by device copies (gsp_pview_create_group: every shard inside this
 * process on one device, for testing the sharded path on one GPU).  Results are identical
 * to gsp_pview_create for any number of shards. */
int gsp_pview_create_rank(const gsp_pview_params *p, int device, int32_t rank, int32_t world,
                          const void *nccl_id, gsp_pview **out);
int gsp_pview_create_group(const gsp_pview_params *p, int device, int32_t shards, gsp_pview **out);
/* shards of the job, first shard held here, its first row, rows held by this engine */
int gsp_pview_layout(gsp_pview *s, int32_t *shards, int32_t *rank, int32_t *row0, int32_t *rows);
int gsp_pview_destroy(gsp_pview *s);
int gsp_pview_step(gsp_pview *s, int32_t ticks);
int gsp_pview_sync(gsp_pview *s);
int gsp_pview_digest_get(gsp_pview *s, int32_t t, gsp_pview_digest *out);
/* Row r: `view` packed entries (id << 32 | hb << 5 | ts mod 32, ~0 = empty) and its length. */
int gsp_pview_row(gsp_pview *s, int32_t r, uint64_t *buf, int32_t cap, int32_t *len);
/* gsp_pview_row / gsp_pview_own_hb fail with GSP_ERR_INVALID for a row another rank holds;
 * gsp_pview_messages returns the slots of the rows held here, in row order. */
int gsp_pview_own_hb(gsp_pview *s, int32_t r, int32_t *hb);
int gsp_pview_messages(gsp_pview *s, int32_t *dst, int64_t cap, int64_t *n);
int gsp_pview_perf_get(gsp_pview *s, gsp_scale_perf *out);
/* Drain all (inbox 0): per drain row class since create -- rows run, messages they merged and
 * kernel ms (HIP events around each class's launch; 0 with timing off) -- for `classes`
 * entries (class c < 4: the LDS classes, 4: the hub kernel; entries past them 0).  The
 * counts are read back with the split kernels' bucket sizes (the default launch form). */
int gsp_pview_drain_stats(gsp_pview *s, int32_t classes, int64_t *rows, int64_t *messages, double *ms);
/* As gsp_scale_drain_events (join / remove / evict records). */
int gsp_pview_drain_events(gsp_pview *s, uint64_t *buf, int64_t cap, int64_t *n, int64_t *lost);
/* Test diagnostics: the rows the tick kernels of tick t ran, summed over the shards held here
 * -- every row exactly once in every launch form, so it equals the rows held.  Needs the
 * environment variable GSP_TEST_PV_COUNT_ROWS=1 at create (else GSP_ERR_INVALID). */
int gsp_pview_rows_run(gsp_pview *s, int32_t t, int64_t *rows);

#ifdef __cplusplus
}
#endif
#endif /* GOSSIP_GOSSIP_H */
