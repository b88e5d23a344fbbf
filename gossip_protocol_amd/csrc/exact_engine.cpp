// gossip_protocol_amd/csrc/exact_engine.cpp -- host side of the EXACT engine (C ABI).
//
// What stays on the host is the index-only bookkeeping whose result is defined by a
// sequential order in the reference:
//   * the EmulNet buffer and its delivery permutation (top-down scan with swap-with-last
//     removal, EmulNet.cpp:144-177) -- per message only (src, dst, type, send batch);
//   * the per-node FIFO queues (Queue.h:22-26), uploaded as CSR for each batch;
//   * the dbg.log byte stream (Log.cpp:44-130), ordered from device event records.
// Everything per member-list entry -- the recvCallBack merge, nodeLoopOps, list order,
// the send lists, the draws, drop window and buffer admission -- runs in the HIP kernels
// of exact_kernels.hip.
#include <algorithm>
#include <cstring>
#include <memory>
#include <numeric>
#include <set>
#include <unordered_map>
#include <string>
#include <vector>

#include "common.hpp"
#include "exact_kernels.hpp"
#include "glibc_stream.hpp"
#include "philox.hpp"

namespace {

constexpr int32_t kMaxNodes = 1024;    // one workgroup lane per column
constexpr int32_t kMaxTicks = 3600;    // EmulNet.h:11 MAX_TIME
constexpr int32_t kMsgHdrBytes = 40;   // sizeof(MessageHdr), MP1Node.h:43-47
constexpr int32_t kEnMsgBytes = 16;    // sizeof(en_msg), EmulNet.h:23-30

struct NetMsg {
    int32_t src, dst, type;
    int64_t send_batch;   // the sender's list version the payload is (its commit batch)
    int32_t prow = -1;    // >= 0: the payload is pool[prow], a list handed in by the driver
    int32_t vrow = -1;    // >= 0: the list a driver callback sees is pool[vrow] (a JOINREP's
                          // list as the reply was sent, MP1Node.cpp:227), not the payload
};

// A sender's list kept from send time, while messages that carry it are in flight and the
// sender has committed a newer one (snapshot mode: the driver-side receive paths).
struct Snapshot {
    int64_t refs = 0;               // admitted messages carrying this version, not yet consumed
    bool kept = false;
    std::vector<gsp_entry> list;
};
uint64_t version_key(int32_t src_id, int64_t batch) { return (uint64_t(uint32_t(src_id)) << 40) | uint64_t(batch); }

// strcmp() over the two 6-byte addresses (EmulNet.cpp:154) compares the little-endian id
// bytes as a C string (the port bytes that follow are 0 for every node), so two ids match
// iff their bytes agree up to the first 0 byte: e.g. ids 256 and 512 (first byte 0) match each
// other, and 65537 matches 1.  addr_class(id) keeps exactly those bytes: equal classes <=>
// strcmp() == 0.
int32_t addr_class(int32_t id) {
    const uint32_t u = uint32_t(id);
    uint32_t out = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t b = (u >> (8 * i)) & 0xFFu;
        if (!b) break;
        out |= b << (8 * i);
    }
    return int32_t(out);
}

// EmulNet's global message buffer (EmulNet.h:40, en_msg *buff[ENBUFFSIZE]) with its delivery
// rule (EmulNet.cpp:151-161): ENrecv scans the buffer top-down and takes every message whose
// destination address strcmp-matches the receiver, moving the current last message into the
// hole.  Messages that linger (e.g. to a failed node) keep taking part in that permutation.
// The same permutation in O(matches * log |B|) instead of O(|B|) per receiver: the buffer
// positions of every address class are kept in an ordered set.  Scanning top-down takes the
// class's positions in descending order; when position k is taken, every position above k
// holds a message of another class (the class's larger positions were taken first and only
// other classes' messages are moved down), so the message moved from the end into k belongs
// to another class and the class's remaining positions are unchanged.
class EmulBuffer {
  public:
    size_t size() const { return msgs_.size(); }
    void push(const NetMsg &m) {
        pos_[addr_class(m.dst)].insert(int32_t(msgs_.size()));
        msgs_.push_back(m);
    }
    // the messages deliver(id, ...) would take, in the same order, without taking them
    template <typename F>
    void peek(int32_t id, F &&see) const {
        auto it = pos_.find(addr_class(id));
        if (it == pos_.end()) return;
        for (auto k = it->second.rbegin(); k != it->second.rend(); ++k) see(msgs_[size_t(*k)]);
    }
    template <typename F>
    void deliver(int32_t id, F &&take) {
        auto it = pos_.find(addr_class(id));
        if (it == pos_.end()) return;
        std::set<int32_t> &mine = it->second;
        while (!mine.empty()) {
            const int32_t k = *mine.rbegin();
            mine.erase(std::prev(mine.end()));
            take(msgs_[size_t(k)]);
            const int32_t last = int32_t(msgs_.size()) - 1;
            if (last != k) {
                std::set<int32_t> &other = pos_[addr_class(msgs_[size_t(last)].dst)];
                other.erase(last);
                other.insert(k);
                msgs_[size_t(k)] = msgs_[size_t(last)];
            }
            msgs_.pop_back();
        }
    }

  private:
    std::vector<NetMsg> msgs_;
    std::unordered_map<int32_t, std::set<int32_t>> pos_;
};

}  // namespace

struct gsp_engine {
    gsp_params p{};
    int32_t n = 0;
    int device = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int rng_mode = 0;
    uint64_t seed = 0;
    gsp::GlibcStream glibc;
    int64_t draws = 0;
    int64_t batch_seq = 1;

    EmulBuffer buf;                           // EmulNet::emulnet.buff
    std::vector<std::vector<NetMsg>> queue;   // Member::mp1q per node
    std::vector<int8_t> failed;
    std::vector<int64_t> last_commit;
    std::vector<int32_t> inited, in_group, own_hb, nlist;
    std::vector<int32_t> recv_ctr;            // [(n+1) * kMaxTicks]
    std::vector<int32_t> sent_host;           // sends issued through gsp_send

    // dbg.log
    std::string log;
    FILE *logf = nullptr;
    size_t log_flushed = 0;
    bool log_first = true;

    gsp_exact_stats stats{};

    // driver-side receive (gsp_recv_detach / gsp_queue_push / gsp_recv_callback)
    bool snapshots = false;
    std::unordered_map<uint64_t, Snapshot> versions;   // by version_key(src id, send batch)
    std::vector<std::vector<gsp_entry>> pool;          // payloads of pushed messages
    std::vector<int32_t> pool_free;
    gsp::DevBuf<int64_t> p_key;
    gsp::DevBuf<int32_t> p_hb, p_ts, p_rank, p_nlist, q_prow;
    gsp::DevBuf<int64_t> rep_key;
    gsp::DevBuf<int32_t> rep_hb, rep_ts, rep_off, adm_slot;

    void admitted(int32_t src_id, int64_t batch) {
        if (snapshots) versions[version_key(src_id, batch)].refs++;
    }
    void consumed(const NetMsg &m) {
        if (m.vrow >= 0) {
            pool[size_t(m.vrow)].clear();
            pool_free.push_back(m.vrow);
        }
        if (m.prow >= 0) {
            pool[size_t(m.prow)].clear();
            pool_free.push_back(m.prow);
            return;
        }
        auto it = versions.find(version_key(m.src, m.send_batch));
        if (it != versions.end() && --it->second.refs <= 0) versions.erase(it);
    }
    int32_t pool_put(std::vector<gsp_entry> &&list) {
        int32_t k;
        if (!pool_free.empty()) { k = pool_free.back(); pool_free.pop_back(); }
        else { k = int32_t(pool.size()); pool.emplace_back(); }
        pool[size_t(k)] = std::move(list);
        return k;
    }

    // device
    gsp::DevBuf<int64_t> t_key, o_key, d_ev_raw;
    gsp::DevBuf<int32_t> t_hb, t_ts, t_rank, t_state;
    gsp::DevBuf<int32_t> o_hb, o_ts, o_rank, o_state;
    gsp::DevBuf<int32_t> b_node, b_op, q_off, q_src, q_type, send_off, send_dst, send_type, send_cnt;
    gsp::DevBuf<gsp::ExactEvent> events;
    gsp::DevBuf<int32_t> counters;            // ev_count, adm_count, draws
    gsp::DevBuf<unsigned long long> merges;
    gsp::DevBuf<int32_t> stream, adm_src, adm_dst, adm_type, sent_ctr;

    gsp::ExactTable table() {
        gsp::ExactTable t;
        t.key = t_key.p; t.hb = t_hb.p; t.ts = t_ts.p; t.rank = t_rank.p;
        t.inited = t_state.p; t.in_group = t_state.p + n; t.own_hb = t_state.p + 2 * n;
        t.nlist = t_state.p + 3 * n;
        return t;
    }

    void append_line(int32_t node, int32_t tick, const char *text) {
        if (log.empty()) {
            // magic number: "%x\n" of the ASCII sum of "CS425" (Log.cpp:79-88)
            int sum = 0;
            for (const char *c = "CS425"; *c; ++c) sum += *c;
            char m[16];
            std::snprintf(m, sizeof m, "%x\n", sum);
            log += m;
        }
        char head[64];
        if (log_first || node < 0) {
            // the very first LOG prints an empty address (the else at Log.cpp:71 binds to
            // the sprintf at :73)
            std::snprintf(head, sizeof head, "\n [%d] ", tick);
        } else {
            const int32_t id = node + 1;
            signed char b[4];
            std::memcpy(b, &id, 4);
            std::snprintf(head, sizeof head, "\n %d.%d.%d.%d:%d [%d] ", b[0], b[1], b[2], b[3], 0,
                          tick);
        }
        log_first = false;
        log += head;
        log += text;
    }

    void member_line(int32_t node, int32_t tick, int32_t subject, const char *verb) {
        const int32_t id = subject + 1;
        signed char b[4];
        std::memcpy(b, &id, 4);
        char text[96];
        std::snprintf(text, sizeof text, "Node %d.%d.%d.%d:%d %s at time %d", b[0], b[1], b[2],
                      b[3], 0, verb, tick);
        append_line(node, tick, text);
    }

    int flush_log() {
        if (!logf) return GSP_OK;
        if (log.size() > log_flushed) {
            std::fwrite(log.data() + log_flushed, 1, log.size() - log_flushed, logf);
            log_flushed = log.size();
        }
        std::fflush(logf);
        return GSP_OK;
    }
};

namespace {

int upload_i32(gsp::DevBuf<int32_t> &d, const std::vector<int32_t> &h, hipStream_t st) {
    GSP_HIP(d.alloc(h.size()));
    if (!h.empty())
        GSP_HIP(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
    return GSP_OK;
}

int check_engine(gsp_engine *e) {
    GSP_REQUIRE(e, GSP_ERR_INVALID, "engine is NULL");
    GSP_HIP(hipSetDevice(e->device));
    return GSP_OK;
}

// `node`'s committed member list in list order (one device read).
int read_list(gsp_engine *e, int32_t node, std::vector<gsp_entry> &list) {
    const int32_t N = e->n;
    std::vector<int64_t> key(N);
    std::vector<int32_t> hb(N), ts(N), rank(N);
    const size_t row = size_t(node) * N;
    GSP_HIP(hipMemcpyAsync(key.data(), e->t_key.p + row, N * 8, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(hb.data(), e->t_hb.p + row, N * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(ts.data(), e->t_ts.p + row, N * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(rank.data(), e->t_rank.p + row, N * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipStreamSynchronize(e->st));
    list.assign(size_t(N), gsp_entry{});
    int32_t cnt = 0;
    for (int32_t x = 0; x < N; ++x) {
        if (key[x] < 0) continue;
        GSP_REQUIRE(rank[x] >= 0 && rank[x] < N, GSP_ERR_INVALID, "corrupt rank");
        list[size_t(rank[x])] = gsp_entry{x + 1, 0, hb[x], ts[x]};
        cnt++;
    }
    list.resize(size_t(cnt));
    return GSP_OK;
}

// Whether a message's merge reads its payload: GOSSIP always (MP1Node.cpp:244-256), JOINREP
// only with the opt-in introducer list (the reference ignores it, :231-233), JOINREQ never.
bool carries_payload(const gsp_engine *e, const NetMsg &m) {
    return m.type == GSP_MSG_GOSSIP || (m.type == GSP_MSG_JOINREP && e->p.intro_list > 0);
}

// The payload of a queued message (the sender's list at send time, MP1Node.cpp:138/227/357):
// *out = its pool list or the list kept from send time, or nullptr when it is the sender's
// committed row (the sender has not committed since the send).
int payload_of(gsp_engine *e, const NetMsg &m, const std::vector<gsp_entry> **out) {
    *out = nullptr;
    if (m.prow >= 0) {
        *out = &e->pool[size_t(m.prow)];
        return GSP_OK;
    }
    const int32_t s = m.src - 1;
    GSP_REQUIRE(s >= 0 && s < e->n, GSP_ERR_INVALID, "message from id %d", m.src);
    if (e->last_commit[s] == m.send_batch) return GSP_OK;
    auto it = e->versions.find(version_key(m.src, m.send_batch));
    GSP_REQUIRE(it != e->versions.end() && it->second.kept, GSP_ERR_ORDER,
                "message from id %d to id %d has a stale payload (sender re-processed since the "
                "send; gsp_payload_snapshots keeps send-time lists)", m.src, m.dst);
    *out = &it->second.list;
    return GSP_OK;
}

// A driver-built payload: ids 1..N, port 0, each id once (one table column per id).
int check_payload(const gsp_engine *e, const gsp_entry *p, int32_t n) {
    GSP_REQUIRE(n >= 0 && n <= e->n && (p || n == 0), GSP_ERR_INVALID,
                "payload of %d entries (at most %d)", n, e->n);
    std::vector<int8_t> seen(size_t(e->n), 0);
    for (int32_t i = 0; i < n; ++i) {
        GSP_REQUIRE(p[i].id >= 1 && p[i].id <= e->n && p[i].port == 0, GSP_ERR_INVALID,
                    "payload entry %d: id %d port %d (ids 1..%d, port 0)", i, p[i].id,
                    int(p[i].port), e->n);
        GSP_REQUIRE(!seen[size_t(p[i].id - 1)], GSP_ERR_INVALID, "payload entry %d: id %d twice",
                    i, p[i].id);
        GSP_REQUIRE(p[i].heartbeat >= INT32_MIN && p[i].heartbeat <= INT32_MAX &&
                    p[i].timestamp >= INT32_MIN && p[i].timestamp <= INT32_MAX,
                    GSP_ERR_INVALID, "payload entry %d: heartbeat/timestamp outside int32", i);
        seen[size_t(p[i].id - 1)] = 1;
    }
    return GSP_OK;
}

int make_msg(gsp_engine *e, int32_t node, const gsp_queued_msg *m, const gsp_entry *payload,
             NetMsg *out) {
    GSP_REQUIRE(m && node >= 0 && node < e->n, GSP_ERR_INVALID, "bad message or node %d", node);
    GSP_REQUIRE(m->src_id >= 1 && m->src_id <= e->n, GSP_ERR_INVALID, "message from id %d",
                m->src_id);
    GSP_REQUIRE(m->type == GSP_MSG_JOINREQ || m->type == GSP_MSG_JOINREP ||
                m->type == GSP_MSG_GOSSIP, GSP_ERR_INVALID, "message type %d", m->type);
    *out = NetMsg{m->src_id, node + 1, m->type, m->send_batch};
    if (payload) {
        if (int rc = check_payload(e, payload, m->payload_len)) return rc;
        out->prow = e->pool_put(std::vector<gsp_entry>(payload, payload + m->payload_len));
        return GSP_OK;
    }
    // NULL: the payload is the sender's list of version send_batch.  The engine must still
    // hold it when the message carries one (GOSSIP, or JOINREP with an introducer list), and
    // the message counts as one more carrier of that version until it is consumed -- a
    // detached message already gave its count back (gsp_recv_detach -> consumed), so without
    // this the version's refcount would drop twice and a list other in-flight messages still
    // carry could be erased.
    if (carries_payload(e, *out)) {
        const std::vector<gsp_entry> *pl = nullptr;
        if (int rc = payload_of(e, *out, &pl)) return rc;
    }
    e->admitted(out->src, out->send_batch);
    return GSP_OK;
}

}  // namespace

extern "C" {

int gsp_create(const gsp_params *p, int device, gsp_rng_mode rng, uint64_t seed,
               const char *dbg_log_path, gsp_engine **out) {
    GSP_REQUIRE(p && out, GSP_ERR_INVALID, "gsp_create: NULL argument");
    GSP_REQUIRE(p->max_nnb >= 1 && p->max_nnb <= kMaxNodes, GSP_ERR_INVALID,
                "gsp_create: max_nnb=%d outside [1, %d]", p->max_nnb, kMaxNodes);
    GSP_REQUIRE(rng == GSP_RNG_GLIBC || rng == GSP_RNG_PHILOX, GSP_ERR_INVALID,
                "gsp_create: unknown rng mode %d", int(rng));
    GSP_REQUIRE(p->intro_list >= 0 && p->intro_list <= 16, GSP_ERR_INVALID,
                "gsp_create: intro_list=%d outside [0, 16]", p->intro_list);
    *out = nullptr;
    int ndev = 0;
    GSP_HIP(hipGetDeviceCount(&ndev));
    GSP_REQUIRE(device >= 0 && device < ndev, GSP_ERR_HIP, "gsp_create: device %d of %d", device,
                ndev);
    GSP_HIP(hipSetDevice(device));
    std::unique_ptr<gsp_engine> e(new gsp_engine);
    e->p = *p;
    e->n = p->max_nnb;
    e->device = device;
    e->rng_mode = int(rng);
    e->seed = seed;
    e->glibc.reseed(uint32_t(seed));
    const int32_t n = e->n;
    e->queue.resize(n);
    e->failed.assign(n, 0);
    e->last_commit.assign(n, 0);
    e->inited.assign(n, 0);
    e->in_group.assign(n, 0);
    e->own_hb.assign(n, 0);
    e->nlist.assign(n, 0);
    e->recv_ctr.assign(size_t(n + 1) * kMaxTicks, 0);
    e->sent_host.assign(size_t(n + 1) * kMaxTicks, 0);
    if (dbg_log_path) {
        e->logf = std::fopen(dbg_log_path, "w");
        GSP_REQUIRE(e->logf, GSP_ERR_IO, "gsp_create: cannot write %s", dbg_log_path);
    }
    GSP_HIP(hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking));
    GSP_HIP(hipEventCreate(&e->ev0));
    GSP_HIP(hipEventCreate(&e->ev1));
    const size_t nn = size_t(n) * n;
    GSP_HIP(e->t_key.alloc(nn));
    GSP_HIP(e->t_hb.alloc(nn));
    GSP_HIP(e->t_ts.alloc(nn));
    GSP_HIP(e->t_rank.alloc(nn));
    GSP_HIP(e->t_state.alloc(size_t(4) * n));
    GSP_HIP(e->o_key.alloc(nn));
    GSP_HIP(e->o_hb.alloc(nn));
    GSP_HIP(e->o_ts.alloc(nn));
    GSP_HIP(e->o_rank.alloc(nn));
    GSP_HIP(e->o_state.alloc(size_t(4) * n));
    GSP_HIP(e->counters.alloc(4));
    GSP_HIP(e->merges.alloc(1));
    GSP_HIP(e->sent_ctr.alloc(size_t(n + 1) * kMaxTicks));
    GSP_HIP(hipMemsetAsync(e->t_key.p, 0xFF, nn * sizeof(int64_t), e->st));   // all absent
    GSP_HIP(hipMemsetAsync(e->t_hb.p, 0, nn * sizeof(int32_t), e->st));
    GSP_HIP(hipMemsetAsync(e->t_ts.p, 0, nn * sizeof(int32_t), e->st));
    GSP_HIP(hipMemsetAsync(e->t_rank.p, 0xFF, nn * sizeof(int32_t), e->st));
    GSP_HIP(hipMemsetAsync(e->t_state.p, 0, size_t(4) * n * sizeof(int32_t), e->st));
    GSP_HIP(hipMemsetAsync(e->sent_ctr.p, 0, size_t(n + 1) * kMaxTicks * sizeof(int32_t), e->st));
    GSP_HIP(hipMemsetAsync(e->merges.p, 0, sizeof(unsigned long long), e->st));
    GSP_HIP(hipStreamSynchronize(e->st));
    *out = e.release();
    return GSP_OK;
}

int gsp_destroy(gsp_engine *e) {
    if (!e) return GSP_OK;
    (void)hipSetDevice(e->device);
    e->flush_log();
    if (e->logf) std::fclose(e->logf);
    if (e->st) (void)hipStreamSynchronize(e->st);
    for (auto *b : {&e->t_hb, &e->t_ts, &e->t_rank, &e->t_state, &e->o_hb, &e->o_ts, &e->o_rank,
                    &e->o_state, &e->b_node, &e->b_op, &e->q_off, &e->q_src, &e->q_type,
                    &e->send_off, &e->send_dst, &e->send_type, &e->send_cnt, &e->counters,
                    &e->stream, &e->adm_src, &e->adm_dst, &e->adm_type, &e->sent_ctr, &e->p_hb,
                    &e->p_ts, &e->p_rank, &e->p_nlist, &e->q_prow, &e->rep_hb, &e->rep_ts,
                    &e->rep_off, &e->adm_slot})
        b->release();
    e->t_key.release();
    e->p_key.release();
    e->rep_key.release();
    e->o_key.release();
    e->events.release();
    e->merges.release();
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->st) (void)hipStreamDestroy(e->st);
    delete e;
    return GSP_OK;
}

int gsp_tick_recv(gsp_engine *e, int32_t tick, const int32_t *order, int32_t n) {
    GSP_REQUIRE(e && (order || n == 0) && n >= 0, GSP_ERR_INVALID, "gsp_tick_recv: bad argument");
    GSP_REQUIRE(tick >= 0 && tick < kMaxTicks, GSP_ERR_INVALID, "gsp_tick_recv: tick %d", tick);
    for (int32_t i = 0; i < n; ++i) {
        const int32_t node = order[i];
        GSP_REQUIRE(node >= 0 && node < e->n, GSP_ERR_INVALID, "gsp_tick_recv: node %d", node);
        const int32_t id = node + 1;
        e->buf.deliver(id, [&](const NetMsg &m) {             // EmulNet.cpp:151-173
            e->queue[node].push_back(m);
            e->recv_ctr[size_t(id) * kMaxTicks + tick]++;
        });
    }
    return GSP_OK;
}

int gsp_tick_process(gsp_engine *e, int32_t tick, const int32_t *order, const int8_t *ops,
                     int32_t n, int32_t dropmsg) {
    if (int rc = check_engine(e)) return rc;
    GSP_REQUIRE(n >= 0 && (n == 0 || (order && ops)), GSP_ERR_INVALID,
                "gsp_tick_process: bad argument");
    GSP_REQUIRE(tick >= 0 && tick < kMaxTicks, GSP_ERR_INVALID, "gsp_tick_process: tick %d", tick);
    if (n == 0) return GSP_OK;
    const int32_t N = e->n;
    GSP_REQUIRE(n <= N, GSP_ERR_INVALID, "gsp_tick_process: batch of %d > %d nodes", n, N);
    std::vector<int8_t> seen(N, 0);
    std::vector<int32_t> h_node(n), h_op(n), h_qoff(n + 1, 0), h_soff(n + 1, 0);
    std::vector<int32_t> h_repoff(n + 1, 0);   // JOINREP list rows of each batch position
    std::vector<int32_t> h_qsrc, h_qtype, h_qprow;
    // payload rows of messages whose list is not the sender's committed row
    std::vector<int64_t> hp_key;
    std::vector<int32_t> hp_hb, hp_ts, hp_rank, hp_nlist;
    auto stage = [&](const std::vector<gsp_entry> &list) {
        const size_t base = hp_nlist.size() * size_t(N);
        hp_key.resize(base + N, -1);
        hp_hb.resize(base + N, 0);
        hp_ts.resize(base + N, 0);
        hp_rank.resize(base + N, -1);
        for (size_t i = 0; i < list.size(); ++i) {
            const size_t o = base + size_t(list[i].id - 1);
            hp_key[o] = 0;
            hp_hb[o] = int32_t(list[i].heartbeat);
            hp_ts[o] = int32_t(list[i].timestamp);
            hp_rank[o] = int32_t(i);
        }
        hp_nlist.push_back(int32_t(list.size()));
        return int32_t(hp_nlist.size()) - 1;
    };
    for (int32_t i = 0; i < n; ++i) {
        const int32_t node = order[i];
        const int32_t op = ops[i];
        GSP_REQUIRE(node >= 0 && node < N, GSP_ERR_INVALID, "gsp_tick_process: node %d", node);
        GSP_REQUIRE(op >= GSP_OP_START && op <= GSP_OP_OPS, GSP_ERR_INVALID,
                    "gsp_tick_process: op %d", op);
        GSP_REQUIRE(!seen[node], GSP_ERR_ORDER,
                    "gsp_tick_process: node %d appears twice in one batch", node);
        seen[node] = 1;
        h_node[i] = node;
        h_op[i] = op;
        int32_t njreq = 0;
        if (op == GSP_OP_LOOP || op == GSP_OP_CHECK) {
            GSP_REQUIRE(e->queue[node].size() < (1u << 20), GSP_ERR_CAPACITY,
                        "gsp_tick_process: queue of node %d too long", node);
            for (const NetMsg &m : e->queue[node]) {
                int32_t prow = -1;
                if (carries_payload(e, m)) {
                    // the payload is the sender's list at send time (MP1Node.cpp:357): its
                    // committed row while unchanged, else a kept or driver-handed list
                    const std::vector<gsp_entry> *pl = nullptr;
                    if (int rc = payload_of(e, m, &pl)) return rc;
                    if (pl) prow = stage(*pl);
                }
                njreq += m.type == GSP_MSG_JOINREQ;
                h_qsrc.push_back(m.src);
                h_qtype.push_back(m.type);
                h_qprow.push_back(prow);
            }
            for (const NetMsg &m : e->queue[node]) e->consumed(m);
            e->queue[node].clear();
        }
        h_qoff[i + 1] = int32_t(h_qsrc.size());
        h_soff[i + 1] = h_soff[i] + njreq + 1 + N;
        h_repoff[i + 1] = h_repoff[i] + (op == GSP_OP_START ? 0 : njreq);
    }
    if (e->snapshots) {
        // keep the lists messages still in flight carry before this batch commits newer ones.
        // After this batch's own queues are consumed: the messages it merges read the committed
        // rows before the commit, so only carriers outside the batch (the buffer, other nodes'
        // queues, driver-held messages) need a kept copy -- one device read per such sender.
        for (int32_t i = 0; i < n; ++i) {
            const int32_t node = order[i];
            auto it = e->versions.find(version_key(node + 1, e->last_commit[node]));
            if (it != e->versions.end() && it->second.refs > 0 && !it->second.kept) {
                if (int rc = read_list(e, node, it->second.list)) return rc;
                it->second.kept = true;
            }
        }
    }
    const int32_t send_cap = h_soff[n];
    hipStream_t st = e->st;
    if (upload_i32(e->b_node, h_node, st) || upload_i32(e->b_op, h_op, st) ||
        upload_i32(e->q_off, h_qoff, st) || upload_i32(e->q_src, h_qsrc, st) ||
        upload_i32(e->q_type, h_qtype, st) || upload_i32(e->send_off, h_soff, st))
        return GSP_ERR_HIP;
    const bool staged = !hp_nlist.empty();
    if (staged) {
        GSP_HIP(e->p_key.alloc(hp_key.size()));
        GSP_HIP(hipMemcpyAsync(e->p_key.p, hp_key.data(), hp_key.size() * 8, hipMemcpyHostToDevice, st));
        if (upload_i32(e->p_hb, hp_hb, st) || upload_i32(e->p_ts, hp_ts, st) ||
            upload_i32(e->p_rank, hp_rank, st) || upload_i32(e->p_nlist, hp_nlist, st) ||
            upload_i32(e->q_prow, h_qprow, st))
            return GSP_ERR_HIP;
    }
    // snapshot mode: the list each JOINREP carries as it is sent, for driver callbacks
    const int32_t n_rep = e->snapshots ? h_repoff[n] : 0;
    if (n_rep) {
        GSP_HIP(e->rep_key.alloc(size_t(n_rep) * N));
        GSP_HIP(e->rep_hb.alloc(size_t(n_rep) * N));
        GSP_HIP(e->rep_ts.alloc(size_t(n_rep) * N));
        GSP_HIP(e->adm_slot.alloc(send_cap));
        if (upload_i32(e->rep_off, h_repoff, st)) return GSP_ERR_HIP;
    }
    GSP_HIP(e->send_dst.alloc(send_cap));
    GSP_HIP(e->send_type.alloc(send_cap));
    GSP_HIP(e->send_cnt.alloc(n));
    GSP_HIP(e->adm_src.alloc(send_cap));
    GSP_HIP(e->adm_dst.alloc(send_cap));
    GSP_HIP(e->adm_type.alloc(send_cap));
    const int32_t ev_cap = n * (2 * N + 2);
    GSP_HIP(e->events.alloc(ev_cap));
    GSP_HIP(hipMemsetAsync(e->counters.p, 0, 4 * sizeof(int32_t), st));
    if (e->rng_mode == GSP_RNG_GLIBC) {
        const int32_t *vals = e->glibc.span(e->draws, send_cap);
        GSP_HIP(e->stream.alloc(send_cap));
        GSP_HIP(hipMemcpyAsync(e->stream.p, vals, size_t(send_cap) * sizeof(int32_t),
                               hipMemcpyHostToDevice, st));
    }

    gsp::ExactBatchDev b{};
    b.n_batch = n;
    b.node = e->b_node.p; b.op = e->b_op.p;
    b.q_off = e->q_off.p; b.q_src = e->q_src.p; b.q_type = e->q_type.p;
    b.q_prow = staged ? e->q_prow.p : nullptr;
    b.p_key = e->p_key.p; b.p_hb = e->p_hb.p; b.p_ts = e->p_ts.p; b.p_rank = e->p_rank.p;
    b.p_nlist = e->p_nlist.p;
    b.rep_off = e->rep_off.p;
    b.rep_key = n_rep ? e->rep_key.p : nullptr;
    b.rep_hb = e->rep_hb.p;
    b.rep_ts = e->rep_ts.p;
    b.send_off = e->send_off.p;
    b.o_key = e->o_key.p; b.o_hb = e->o_hb.p; b.o_ts = e->o_ts.p; b.o_rank = e->o_rank.p;
    b.o_state = e->o_state.p;
    b.send_dst = e->send_dst.p; b.send_type = e->send_type.p; b.send_cnt = e->send_cnt.p;
    b.events = e->events.p; b.ev_count = e->counters.p; b.ev_cap = ev_cap;
    b.merges = e->merges.p;
    b.intro_list = e->p.intro_list;
    b.seed = e->seed;

    gsp::ExactSendDev s{};
    s.n_batch = n;
    s.node = e->b_node.p; s.send_off = e->send_off.p; s.send_cnt = e->send_cnt.p;
    s.send_dst = e->send_dst.p; s.send_type = e->send_type.p;
    s.rng_mode = e->rng_mode;
    s.adm_slot = n_rep ? e->adm_slot.p : nullptr;
    s.glibc_stream = e->stream.p;
    s.stream_base = e->draws;
    s.g0 = e->draws;
    s.seed = e->seed;
    s.tick = tick;
    s.dropmsg = dropmsg ? 1 : 0;
    s.drop_thr = int32_t(e->p.msg_drop_prob * 100);          // EmulNet.cpp:91
    s.buff_room = std::max<int32_t>(0, e->p.en_buff_size - int32_t(e->buf.size()));
    s.size_reject = (kMsgHdrBytes + kEnMsgBytes >= e->p.max_msg_size) ? 1 : 0;
    s.adm_src = e->adm_src.p; s.adm_dst = e->adm_dst.p; s.adm_type = e->adm_type.p;
    s.adm_count = e->counters.p + 1;
    s.draws = e->counters.p + 2;
    s.sent_ctr = e->sent_ctr.p;
    s.max_ticks = kMaxTicks;

    gsp::ExactTable tab = e->table();
    GSP_HIP(hipEventRecord(e->ev0, st));
    GSP_HIP(gsp::launch_exact_batch(tab, b, N, tick, e->batch_seq, e->p.tremove,
                                    e->p.id_filter_limit, st));
    GSP_HIP(gsp::launch_exact_sends(s, st));
    GSP_HIP(gsp::launch_exact_commit(tab, b, N, st));
    GSP_HIP(hipEventRecord(e->ev1, st));

    int32_t ctr[4];
    GSP_HIP(hipMemcpyAsync(ctr, e->counters.p, sizeof ctr, hipMemcpyDeviceToHost, st));
    std::vector<int32_t> o_state(size_t(n) * 4);
    GSP_HIP(hipMemcpyAsync(o_state.data(), e->o_state.p, o_state.size() * sizeof(int32_t),
                           hipMemcpyDeviceToHost, st));
    unsigned long long merges = 0;
    GSP_HIP(hipMemcpyAsync(&merges, e->merges.p, sizeof merges, hipMemcpyDeviceToHost, st));
    GSP_HIP(hipStreamSynchronize(st));
    GSP_REQUIRE(ctr[0] <= ev_cap, GSP_ERR_CAPACITY, "gsp_tick_process: event buffer overflow");
    const int32_t n_ev = ctr[0], n_adm = ctr[1], n_draw = ctr[2];
    std::vector<gsp::ExactEvent> ev(n_ev);
    std::vector<int32_t> a_src(n_adm), a_dst(n_adm), a_type(n_adm);
    if (n_ev)
        GSP_HIP(hipMemcpyAsync(ev.data(), e->events.p, size_t(n_ev) * sizeof(gsp::ExactEvent),
                               hipMemcpyDeviceToHost, st));
    if (n_adm) {
        GSP_HIP(hipMemcpyAsync(a_src.data(), e->adm_src.p, size_t(n_adm) * 4, hipMemcpyDeviceToHost, st));
        GSP_HIP(hipMemcpyAsync(a_dst.data(), e->adm_dst.p, size_t(n_adm) * 4, hipMemcpyDeviceToHost, st));
        GSP_HIP(hipMemcpyAsync(a_type.data(), e->adm_type.p, size_t(n_adm) * 4, hipMemcpyDeviceToHost, st));
    }
    std::vector<int64_t> r_key;
    std::vector<int32_t> r_hb, r_ts, a_slot;
    if (n_rep && n_adm) {
        r_key.resize(size_t(n_rep) * N);
        r_hb.resize(r_key.size());
        r_ts.resize(r_key.size());
        a_slot.resize(size_t(n_adm));
        GSP_HIP(hipMemcpyAsync(r_key.data(), e->rep_key.p, r_key.size() * 8, hipMemcpyDeviceToHost, st));
        GSP_HIP(hipMemcpyAsync(r_hb.data(), e->rep_hb.p, r_hb.size() * 4, hipMemcpyDeviceToHost, st));
        GSP_HIP(hipMemcpyAsync(r_ts.data(), e->rep_ts.p, r_ts.size() * 4, hipMemcpyDeviceToHost, st));
        GSP_HIP(hipMemcpyAsync(a_slot.data(), e->adm_slot.p, size_t(n_adm) * 4, hipMemcpyDeviceToHost, st));
    }
    GSP_HIP(hipStreamSynchronize(st));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e->ev0, e->ev1) == hipSuccess) e->stats.device_ms += ms;

    // dbg.log lines in the reference's order: batch position (call order), then within a
    // node the start line, join lines (queue order j, payload order p), remove lines
    // (descending list index)
    auto phase = [](int32_t k) { return k == gsp::kEvJoin ? 1 : (k == gsp::kEvRemove ? 2 : 0); };
    std::sort(ev.begin(), ev.end(), [&](const gsp::ExactEvent &a, const gsp::ExactEvent &c) {
        if (a.pos != c.pos) return a.pos < c.pos;
        if (phase(a.kind) != phase(c.kind)) return phase(a.kind) < phase(c.kind);
        return a.ord < c.ord;
    });
    for (const auto &x : ev) {
        const int32_t node = h_node[x.pos];
        switch (x.kind) {
            case gsp::kEvStartGroup: e->append_line(node, tick, "Starting up group..."); break;
            case gsp::kEvStartJoin: e->append_line(node, tick, "Trying to join..."); break;
            case gsp::kEvJoin: e->member_line(node, tick, x.subject, "joined"); break;
            default: e->member_line(node, tick, x.subject, "removed"); break;
        }
    }
    for (int32_t k = 0; k < n_adm; ++k) {
        NetMsg m{a_src[k], a_dst[k], a_type[k], e->batch_seq};
        if (!a_slot.empty() && a_type[k] == GSP_MSG_JOINREP) {
            // replies lead each node's send list: slot - send_off[pos] is the reply index
            const int32_t pos = int32_t(std::upper_bound(h_soff.begin(), h_soff.end(), a_slot[k]) -
                                        h_soff.begin()) - 1;
            const size_t row = size_t(h_repoff[pos] + a_slot[k] - h_soff[pos]) * N;
            std::vector<std::pair<int64_t, int32_t>> cols;
            for (int32_t x = 0; x < N; ++x)
                if (r_key[row + x] >= 0) cols.emplace_back(r_key[row + x], x);
            std::sort(cols.begin(), cols.end());
            std::vector<gsp_entry> list;
            for (const auto &c : cols)
                list.push_back(gsp_entry{c.second + 1, 0, r_hb[row + c.second], r_ts[row + c.second]});
            m.vrow = e->pool_put(std::move(list));
        }
        e->buf.push(m);
        e->admitted(a_src[k], e->batch_seq);
    }
    for (int32_t i = 0; i < n; ++i) {
        const int32_t node = h_node[i];
        e->inited[node] = o_state[size_t(i) * 4 + 0];
        e->in_group[node] = o_state[size_t(i) * 4 + 1];
        e->own_hb[node] = o_state[size_t(i) * 4 + 2];
        e->nlist[node] = o_state[size_t(i) * 4 + 3];
        e->last_commit[node] = e->batch_seq;
        if (h_op[i] == GSP_OP_START) e->failed[node] = 0;   // initThisNode, MP1Node.cpp:102
        if (h_op[i] == GSP_OP_LOOP) e->stats.node_rounds++;
    }
    e->draws += n_draw;
    e->glibc.trim(e->draws);
    e->stats.draws = e->draws;
    e->stats.batches++;
    e->stats.sends_admitted += n_adm;
    e->stats.merges = int64_t(merges);
    e->batch_seq++;
    return GSP_OK;
}

int gsp_payload_snapshots(gsp_engine *e, int32_t on) {
    GSP_REQUIRE(e, GSP_ERR_INVALID, "gsp_payload_snapshots: NULL engine");
    e->snapshots = on != 0;
    if (!e->snapshots) e->versions.clear();
    return GSP_OK;
}

int gsp_recv_detach(gsp_engine *e, int32_t tick, int32_t node, gsp_queued_msg *msgs, int32_t cap,
                    gsp_entry *payload, int64_t payload_cap, int32_t *n, int64_t *n_payload) {
    if (int rc = check_engine(e)) return rc;
    GSP_REQUIRE(n && n_payload && node >= 0 && node < e->n, GSP_ERR_INVALID,
                "gsp_recv_detach: bad argument");
    GSP_REQUIRE(tick >= 0 && tick < kMaxTicks, GSP_ERR_INVALID, "gsp_recv_detach: tick %d", tick);
    const int32_t id = node + 1;
    int32_t cnt = 0;
    int64_t total = 0;
    int rc = GSP_OK;
    static const std::vector<gsp_entry> kNoList;
    // the list a driver callback sees: a JOINREP's send-time list, a driver-built list, an
    // engine JOINREQ's empty list (nodeStart clears the list before introduceSelfToGroup sends
    // it, MP1Node.cpp:95-150), or the sender's list of the message's version
    auto list_of = [&](const NetMsg &m, const std::vector<gsp_entry> **pl) {
        *pl = m.vrow >= 0 ? &e->pool[size_t(m.vrow)] : nullptr;
        if (!*pl && m.prow < 0 && m.type == GSP_MSG_JOINREQ) *pl = &kNoList;
        return *pl ? GSP_OK : payload_of(e, m, pl);
    };
    e->buf.peek(id, [&](const NetMsg &m) {
        const std::vector<gsp_entry> *pl = nullptr;
        if (rc == GSP_OK) rc = list_of(m, &pl);
        cnt++;
        total += pl ? int64_t(pl->size()) : int64_t(e->nlist[size_t(m.src - 1)]);
    });
    if (rc) return rc;
    *n = cnt;
    *n_payload = total;
    if (!msgs) return GSP_OK;                                 // sizes only, nothing taken
    GSP_REQUIRE(cap >= cnt && payload_cap >= total && (payload || total == 0), GSP_ERR_CAPACITY,
                "gsp_recv_detach: %d messages / %lld payload entries do not fit %d / %lld", cnt,
                (long long)total, cap, (long long)payload_cap);
    std::unordered_map<int32_t, std::vector<gsp_entry>> live;   // committed rows read here
    int32_t k = 0;
    int64_t off = 0;
    e->buf.deliver(id, [&](const NetMsg &m) {                 // EmulNet.cpp:151-173
        e->recv_ctr[size_t(id) * kMaxTicks + tick]++;
        const std::vector<gsp_entry> *pl = nullptr;
        if (rc == GSP_OK) rc = list_of(m, &pl);
        if (rc == GSP_OK && !pl) {
            auto it = live.find(m.src);
            if (it == live.end()) {
                it = live.emplace(m.src, std::vector<gsp_entry>()).first;
                rc = read_list(e, m.src - 1, it->second);
            }
            pl = &it->second;
        }
        gsp_queued_msg &q = msgs[k++];
        q.src_id = m.src;
        q.type = m.type;
        q.send_batch = m.send_batch;
        q.payload_off = off;
        q.payload_len = pl && rc == GSP_OK ? int32_t(pl->size()) : 0;
        if (q.payload_len) std::memcpy(payload + off, pl->data(), pl->size() * sizeof(gsp_entry));
        off += q.payload_len;
        e->consumed(m);
    });
    return rc;
}

int gsp_queue_push(gsp_engine *e, int32_t node, const gsp_queued_msg *m, const gsp_entry *payload) {
    GSP_REQUIRE(e, GSP_ERR_INVALID, "gsp_queue_push: NULL engine");
    NetMsg nm;
    if (int rc = make_msg(e, node, m, payload, &nm)) return rc;
    e->queue[size_t(node)].push_back(nm);
    return GSP_OK;
}

int gsp_recv_callback(gsp_engine *e, int32_t tick, int32_t node, const gsp_queued_msg *m,
                      const gsp_entry *payload, int32_t dropmsg) {
    GSP_REQUIRE(e, GSP_ERR_INVALID, "gsp_recv_callback: NULL engine");
    NetMsg nm;
    if (int rc = make_msg(e, node, m, payload, &nm)) return rc;
    // exactly this message, now: a CHECK batch over a one-message queue; the node's own queue
    // is set aside and comes back unchanged
    std::vector<NetMsg> held;
    held.swap(e->queue[size_t(node)]);
    e->queue[size_t(node)].push_back(nm);
    const int8_t op = GSP_OP_CHECK;
    const int rc = gsp_tick_process(e, tick, &node, &op, 1, dropmsg);
    if (rc && !e->queue[size_t(node)].empty()) e->consumed(e->queue[size_t(node)].front());
    e->queue[size_t(node)].swap(held);
    return rc;
}

int gsp_send(gsp_engine *e, int32_t tick, int32_t src_node, int32_t dst_id, int32_t type,
             int32_t dropmsg, int32_t *admitted) {
    return gsp_send_list(e, tick, src_node, dst_id, type, dropmsg, nullptr, 0, admitted);
}

int gsp_send_list(gsp_engine *e, int32_t tick, int32_t src_node, int32_t dst_id, int32_t type,
                  int32_t dropmsg, const gsp_entry *payload, int32_t n_payload, int32_t *admitted) {
    GSP_REQUIRE(e && admitted, GSP_ERR_INVALID, "gsp_send: NULL argument");
    if (payload)
        if (int rc = check_payload(e, payload, n_payload)) return rc;
    GSP_REQUIRE(src_node >= 0 && src_node < e->n, GSP_ERR_INVALID, "gsp_send: node %d", src_node);
    GSP_REQUIRE(tick >= 0 && tick < kMaxTicks, GSP_ERR_INVALID, "gsp_send: tick %d", tick);
    GSP_REQUIRE(type == GSP_MSG_JOINREQ || type == GSP_MSG_JOINREP || type == GSP_MSG_GOSSIP,
                GSP_ERR_INVALID, "gsp_send: type %d", type);
    const int32_t src_id = src_node + 1;
    int32_t draw;                                            // EmulNet.cpp:89, always drawn
    if (e->rng_mode == GSP_RNG_PHILOX)
        draw = int32_t(gsp::draw_u31(gsp::kDomainSend, e->seed, uint32_t(tick), uint32_t(src_id),
                                     uint32_t(dst_id), uint32_t(type)));
    else
        draw = e->glibc.at(e->draws);
    e->draws++;
    e->glibc.trim(e->draws);
    e->stats.draws = e->draws;
    const int32_t thr = int32_t(e->p.msg_drop_prob * 100);
    *admitted = 0;
    if (int32_t(e->buf.size()) >= e->p.en_buff_size ||
        kMsgHdrBytes + kEnMsgBytes >= e->p.max_msg_size || (dropmsg && draw % 100 < thr))
        return GSP_OK;
    // the payload is the list handed in, or the sender's list as committed now
    NetMsg m{src_id, dst_id, type, e->last_commit[src_node]};
    if (payload) m.prow = e->pool_put(std::vector<gsp_entry>(payload, payload + n_payload));
    else e->admitted(src_id, e->last_commit[src_node]);
    e->buf.push(m);
    e->sent_host[size_t(src_id) * kMaxTicks + tick]++;
    e->stats.sends_admitted++;
    *admitted = kMsgHdrBytes;
    return GSP_OK;
}

int gsp_rand(gsp_engine *e, int32_t tick, int32_t *value) {
    GSP_REQUIRE(e && value, GSP_ERR_INVALID, "gsp_rand: NULL argument");
    if (e->rng_mode == GSP_RNG_PHILOX)
        *value = int32_t(gsp::draw_u31(gsp::kDomainFail, e->seed, uint32_t(tick), 0, 0, 0));
    else
        *value = e->glibc.at(e->draws);
    e->draws++;
    e->glibc.trim(e->draws);
    e->stats.draws = e->draws;
    return GSP_OK;
}

int gsp_srand(gsp_engine *e, uint64_t seed) {
    GSP_REQUIRE(e, GSP_ERR_INVALID, "gsp_srand: NULL engine");
    e->seed = seed;
    e->glibc.reseed_at(uint32_t(seed), e->draws);
    return GSP_OK;
}

int gsp_log(gsp_engine *e, int32_t node, int32_t tick, const char *text) {
    GSP_REQUIRE(e && text, GSP_ERR_INVALID, "gsp_log: NULL argument");
    GSP_REQUIRE(node < e->n, GSP_ERR_INVALID, "gsp_log: node %d", node);
    e->append_line(node, tick, text);
    return GSP_OK;
}

int gsp_set_failed(gsp_engine *e, int32_t node, int32_t failed) {
    GSP_REQUIRE(e && node >= 0 && node < e->n, GSP_ERR_INVALID, "gsp_set_failed: bad node");
    e->failed[node] = failed ? 1 : 0;
    return GSP_OK;
}

int gsp_get_member(gsp_engine *e, int32_t node, gsp_member_view *out) {
    GSP_REQUIRE(e && out && node >= 0 && node < e->n, GSP_ERR_INVALID, "gsp_get_member: bad arg");
    out->id = node + 1;
    out->port = 0;
    out->inited = int8_t(e->inited[node]);
    out->in_group = int8_t(e->in_group[node]);
    out->failed = e->failed[node];
    out->heartbeat = e->own_hb[node];
    out->n_members = e->nlist[node];
    return GSP_OK;
}

int gsp_member_list(gsp_engine *e, int32_t node, gsp_entry *buf, int32_t cap, int32_t *n) {
    if (int rc = check_engine(e)) return rc;
    GSP_REQUIRE(node >= 0 && node < e->n && n && (buf || cap == 0), GSP_ERR_INVALID,
                "gsp_member_list: bad argument");
    std::vector<gsp_entry> list;
    if (int rc = read_list(e, node, list)) return rc;
    *n = int32_t(list.size());
    for (int32_t k = 0; k < *n && k < cap; ++k) buf[k] = list[size_t(k)];
    return GSP_OK;
}

int gsp_member_lists(gsp_engine *e, const int32_t *nodes, int32_t n, gsp_entry *buf,
                     int32_t *lens) {
    if (int rc = check_engine(e)) return rc;
    GSP_REQUIRE(n >= 0 && (n == 0 || (nodes && buf && lens)), GSP_ERR_INVALID,
                "gsp_member_lists: bad argument");
    if (n == 0) return GSP_OK;
    const int32_t N = e->n;
    for (int32_t i = 0; i < n; ++i)
        GSP_REQUIRE(nodes[i] >= 0 && nodes[i] < N, GSP_ERR_INVALID, "gsp_member_lists: node %d",
                    nodes[i]);
    // the whole committed table in one read per array (N <= 1024: at most 20 MB)
    const size_t nn = size_t(N) * N;
    std::vector<int64_t> key(nn);
    std::vector<int32_t> hb(nn), ts(nn), rank(nn);
    GSP_HIP(hipMemcpyAsync(key.data(), e->t_key.p, nn * 8, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(hb.data(), e->t_hb.p, nn * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(ts.data(), e->t_ts.p, nn * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(rank.data(), e->t_rank.p, nn * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipStreamSynchronize(e->st));
    for (int32_t i = 0; i < n; ++i) {
        const size_t row = size_t(nodes[i]) * N;
        gsp_entry *out = buf + size_t(i) * N;
        int32_t cnt = 0;
        for (int32_t x = 0; x < N; ++x) {
            if (key[row + x] < 0) continue;
            GSP_REQUIRE(rank[row + x] >= 0 && rank[row + x] < N, GSP_ERR_INVALID, "corrupt rank");
            out[rank[row + x]] = gsp_entry{x + 1, 0, hb[row + x], ts[row + x]};
            cnt++;
        }
        lens[i] = cnt;
    }
    return GSP_OK;
}

int gsp_add_member(gsp_engine *e, int32_t tick, int32_t node, const gsp_entry *entry,
                   int32_t mode, int32_t *added) {
    if (int rc = check_engine(e)) return rc;
    GSP_REQUIRE(entry && added && node >= 0 && node < e->n, GSP_ERR_INVALID,
                "gsp_add_member: bad argument");
    GSP_REQUIRE(mode == GSP_ADD_SENDER || mode == GSP_ADD_COPY, GSP_ERR_INVALID,
                "gsp_add_member: mode %d", mode);
    GSP_REQUIRE(tick >= 0 && tick < kMaxTicks, GSP_ERR_INVALID, "gsp_add_member: tick %d", tick);
    const int32_t N = e->n, id = entry->id;
    GSP_REQUIRE(id >= 1 && id <= N && entry->port == 0, GSP_ERR_INVALID,
                "gsp_add_member: id %d port %d (ids 1..%d, port 0)", id, int(entry->port), N);
    *added = 0;
    const int32_t x = id - 1;
    const size_t o = size_t(node) * N + size_t(x);
    int64_t key = -1;
    GSP_HIP(hipMemcpyAsync(&key, e->t_key.p + o, 8, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipStreamSynchronize(e->st));
    int32_t hb, ts;
    if (mode == GSP_ADD_SENDER) {                               // MP1Node.cpp:265-280
        if (key >= 0) return GSP_OK;                            // check_exist(id, port)
        hb = 1;
        ts = tick;
    } else {                                                    // MP1Node.cpp:282-301
        if (id == node + 1) return GSP_OK;                      // *addr == memberNode->addr
        if (int64_t(tick) - entry->timestamp >= e->p.tremove) return GSP_OK;
        GSP_REQUIRE(key < 0, GSP_ERR_INVALID,
                    "gsp_add_member: id %d is listed already (the reference would list it twice)", id);
        GSP_REQUIRE(entry->heartbeat >= INT32_MIN && entry->heartbeat <= INT32_MAX &&
                    entry->timestamp >= INT32_MIN && entry->timestamp <= INT32_MAX,
                    GSP_ERR_INVALID, "gsp_add_member: heartbeat/timestamp outside int32");
        hb = int32_t(entry->heartbeat);
        ts = int32_t(entry->timestamp);
    }
    // a new version of the list: keep the old one while messages in flight carry it
    if (e->snapshots) {
        auto it = e->versions.find(version_key(node + 1, e->last_commit[node]));
        if (it != e->versions.end() && it->second.refs > 0 && !it->second.kept) {
            if (int rc = read_list(e, node, it->second.list)) return rc;
            it->second.kept = true;
        }
    }
    // push_back: an insertion key above every key of earlier batches (make_key(batch, 0, 0),
    // exact_kernels.hip), rank = the list length
    const int64_t nkey = e->batch_seq << 40;
    const int32_t rank = e->nlist[node];
    const int32_t nl = rank + 1;
    GSP_HIP(hipMemcpyAsync(e->t_key.p + o, &nkey, 8, hipMemcpyHostToDevice, e->st));
    GSP_HIP(hipMemcpyAsync(e->t_hb.p + o, &hb, 4, hipMemcpyHostToDevice, e->st));
    GSP_HIP(hipMemcpyAsync(e->t_ts.p + o, &ts, 4, hipMemcpyHostToDevice, e->st));
    GSP_HIP(hipMemcpyAsync(e->t_rank.p + o, &rank, 4, hipMemcpyHostToDevice, e->st));
    GSP_HIP(hipMemcpyAsync(e->t_state.p + 3 * size_t(N) + node, &nl, 4, hipMemcpyHostToDevice, e->st));
    GSP_HIP(hipStreamSynchronize(e->st));
    e->nlist[node] = nl;
    e->last_commit[node] = e->batch_seq;
    e->batch_seq++;
    e->member_line(node, tick, x, "joined");                    // Log::logNodeAdd
    *added = 1;
    return GSP_OK;
}

// Every node's state after tick `tick`, appended to `path` as one line per node in id order:
//   t id inited inGroup bFailed heartbeat |L| id:hb:ts ...      (list in MemberListEntry order)
// -- the Member fields the reference keeps (Member.h:89-122), in the end-of-tick dump format
// of the parity fixtures (oracle/ref_hooks.cpp).  One copy of the device tables per call.
int gsp_state_dump(gsp_engine *e, int32_t tick, const char *path) {
    if (int rc = check_engine(e)) return rc;
    GSP_REQUIRE(path, GSP_ERR_INVALID, "gsp_state_dump: NULL path");
    const int32_t N = e->n;
    const size_t nn = size_t(N) * N;
    std::vector<int64_t> key(nn);
    std::vector<int32_t> hb(nn), ts(nn), rank(nn);
    GSP_HIP(hipMemcpyAsync(key.data(), e->t_key.p, nn * 8, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(hb.data(), e->t_hb.p, nn * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(ts.data(), e->t_ts.p, nn * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipMemcpyAsync(rank.data(), e->t_rank.p, nn * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipStreamSynchronize(e->st));
    FILE *f = std::fopen(path, "a");
    GSP_REQUIRE(f, GSP_ERR_IO, "gsp_state_dump: cannot open %s", path);
    std::vector<int32_t> order(static_cast<size_t>(N));
    std::string line;
    char tmp[64];
    for (int32_t node = 0; node < N; ++node) {
        const size_t row = size_t(node) * N;
        int32_t cnt = 0;
        for (int32_t x = 0; x < N; ++x) {
            if (key[row + x] < 0) continue;
            const int32_t rk = rank[row + x];
            if (rk < 0 || rk >= N) { std::fclose(f); GSP_REQUIRE(false, GSP_ERR_INVALID, "corrupt rank"); }
            order[size_t(rk)] = x;
            cnt++;
        }
        std::snprintf(tmp, sizeof tmp, "%d %d %d %d %d %d %d", tick, node + 1, e->inited[node],
                      e->in_group[node], int(e->failed[node]), e->own_hb[node], cnt);
        line = tmp;
        for (int32_t k = 0; k < cnt; ++k) {
            const int32_t x = order[size_t(k)];
            std::snprintf(tmp, sizeof tmp, " %d:%d:%d", x + 1, hb[row + x], ts[row + x]);
            line += tmp;
        }
        line += '\n';
        std::fwrite(line.data(), 1, line.size(), f);
    }
    std::fclose(f);
    return GSP_OK;
}

int gsp_counters(gsp_engine *e, int32_t *sent, int32_t *recv, int32_t ticks) {
    if (int rc = check_engine(e)) return rc;
    GSP_REQUIRE(ticks >= 0 && ticks <= kMaxTicks, GSP_ERR_INVALID, "gsp_counters: ticks %d", ticks);
    const int32_t N = e->n;
    std::vector<int32_t> dev(size_t(N + 1) * kMaxTicks);
    GSP_HIP(hipMemcpyAsync(dev.data(), e->sent_ctr.p, dev.size() * 4, hipMemcpyDeviceToHost, e->st));
    GSP_HIP(hipStreamSynchronize(e->st));
    for (int32_t id = 0; id <= N; ++id)
        for (int32_t t = 0; t < ticks; ++t) {
            if (sent)
                sent[size_t(id) * ticks + t] = dev[size_t(id) * kMaxTicks + t] +
                                               e->sent_host[size_t(id) * kMaxTicks + t];
            if (recv) recv[size_t(id) * ticks + t] = e->recv_ctr[size_t(id) * kMaxTicks + t];
        }
    return GSP_OK;
}

// EmulNet::ENcleanup's msgcount.log (EmulNet.cpp:195-216), including the node-67 layout.
int gsp_write_msgcount(gsp_engine *e, const char *path, int32_t tick) {
    GSP_REQUIRE(e && path, GSP_ERR_INVALID, "gsp_write_msgcount: NULL argument");
    const int32_t N = e->n;
    std::vector<int32_t> sent(size_t(N + 1) * tick), recv(size_t(N + 1) * tick);
    if (int rc = gsp_counters(e, sent.data(), recv.data(), tick)) return rc;
    FILE *f = std::fopen(path, "w");
    GSP_REQUIRE(f, GSP_ERR_IO, "gsp_write_msgcount: cannot write %s", path);
    for (int32_t id = 1; id <= N; ++id) {
        std::fprintf(f, "node %3d ", id);
        uint32_t st = 0, rt = 0;
        for (int32_t j = 0; j < tick; ++j) {
            const int32_t a = sent[size_t(id) * tick + j], c = recv[size_t(id) * tick + j];
            st += uint32_t(a);
            rt += uint32_t(c);
            if (id == 67) {
                std::fprintf(f, "special %4d %4d %4d\n", j, a, c);
            } else {
                std::fprintf(f, " (%4d, %4d)", a, c);
                if (j % 10 == 9) std::fprintf(f, "\n         ");
            }
        }
        std::fprintf(f, "\nnode %3d sent_total %6u  recv_total %6u\n\n", id, st, rt);
    }
    std::fclose(f);
    return GSP_OK;
}

int gsp_flush_log(gsp_engine *e) {
    GSP_REQUIRE(e, GSP_ERR_INVALID, "gsp_flush_log: NULL engine");
    return e->flush_log();
}

int gsp_log_bytes(gsp_engine *e, char *buf, size_t cap, size_t *n) {
    GSP_REQUIRE(e && n, GSP_ERR_INVALID, "gsp_log_bytes: NULL argument");
    *n = e->log.size();
    if (buf && cap) std::memcpy(buf, e->log.data(), std::min(cap, e->log.size()));
    return GSP_OK;
}

int gsp_exact_stats_get(gsp_engine *e, gsp_exact_stats *out) {
    GSP_REQUIRE(e && out, GSP_ERR_INVALID, "gsp_exact_stats_get: NULL argument");
    *out = e->stats;
    return GSP_OK;
}

}  // extern "C"
