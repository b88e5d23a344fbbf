// include/gossip/mp1_facade.hpp -- the reference's MP1 class surface over the C ABI.
//
// A driver written against the reference headers (/root/reference/{Member,Params,Log,
// EmulNet,MP1Node,Queue}.h) compiles against this header instead and runs on the MI355X
// engine: same class names, same public fields, same method names and signatures, same
// return conventions.  The classes are thin: every MP1Node / EmulNet call is RECORDED and
// the calls of one phase are flushed to the engine as one batch (gsp_tick_recv /
// gsp_tick_process), where the HIP kernels run them for all recorded nodes at once.  A
// flush happens whenever the observable order requires it: a Log::LOG line from the
// driver, a change of tick / phase / Params::dropmsg, a node recorded twice in one phase,
// EmulNet::ENsend/ENcleanup, or MP1Node::syncMember().
//
// Member is a host mirror.  bFailed and addr are driver-owned (Application::fail writes
// bFailed directly, Application.cpp:186/194); inited / inGroup / heartbeat / nnb and
// memberList are refreshed after every batch that ran the node (memberList with one device
// read of the table per batch).  MP1Node::getMemberNode() first runs a batch the node is
// recorded in, so a driver reading getMemberNode()->memberList sees what the reference's
// list holds at that point.  The mirror is read-only: writes to memberList do not reach the
// engine (MP1Node::addMember does).
//
// rand() / srand(): the reference's Application draws from libc rand() (fail(),
// Application.cpp:182/189) on the stream its EmulNet draws from (EmulNet.cpp:89).  The
// engine owns that stream, so the forwarding headers in include/gossip/ref/ (MP1Node.h,
// EmulNet.h, ...) map rand() / srand() of the translation unit that includes them onto
// gsp_mp1_rand() / gsp_mp1_srand() (include/gossip/ref/gsp_rand_interpose.h) -- srand(seed) seeds the engine's
// stream (before the EmulNet exists: the seed it is created with), rand() runs the recorded
// work and returns the stream's next draw.  Application.cpp then compiles unchanged.
//
// Receive paths (EmulNet.cpp:144-177, MP1Node.cpp:44-56, 200-260):
//   * recvLoop (ENrecv with MP1Node::enqueueWrapper into the member's mp1q) is the batched
//     path: the messages stay in the engine and checkMessages / nodeLoop drain them there;
//   * ENrecv with any other callback or queue hands the callback each message as a heap
//     MessageHdr (msgType, addr, vector_list = the sender's list at send time), in the
//     reference's delivery order.  Whatever the callback puts into a member's mp1q is fed
//     back to the engine, with the list it then holds, when that member next receives or
//     processes (recvLoop / checkMessages / nodeLoop), and deleted as the reference's
//     recvCallBack deletes each message it handles (MP1Node.cpp:258);
//   * recvCallBack(env, data, size) called by the driver processes that one MessageHdr at
//     once (the engine's gsp_recv_callback) and deletes it.
// A MessageHdr list must name nodes of this emulation (ids 1..N, port 0), each at most once.
#pragma once

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <queue>
#include <string>
#include <unordered_set>
#include <vector>

#include "gossip/gossip.h"

#ifndef SUCCESS
#define SUCCESS 0
#endif
#ifndef FAILURE
#define FAILURE -1
#endif

#define TREMOVE 20
#define TFAIL 5

class q_elt {
public:
    void *elt;
    int size;
    q_elt(void *e, int s) : elt(e), size(s) {}
};

class Address {
public:
    char addr[6];
    Address() { std::memset(addr, 0, sizeof addr); }
    Address(const Address &o) { std::memcpy(addr, o.addr, sizeof addr); }
    explicit Address(const std::string &a) {
        const size_t c = a.find(':');
        const int id = std::stoi(a.substr(0, c));
        const short port = short(std::stoi(a.substr(c + 1)));
        std::memcpy(&addr[0], &id, 4);
        std::memcpy(&addr[4], &port, 2);
    }
    Address &operator=(const Address &o) {
        std::memcpy(addr, o.addr, sizeof addr);
        return *this;
    }
    bool operator==(const Address &o) const { return std::memcmp(addr, o.addr, sizeof addr) == 0; }
    int id() const { int v; std::memcpy(&v, &addr[0], 4); return v; }
    short port() const { short v; std::memcpy(&v, &addr[4], 2); return v; }
    std::string getAddress() { return std::to_string(id()) + ":" + std::to_string(port()); }
    void init() { std::memset(addr, 0, sizeof addr); }
};

class MemberListEntry {
public:
    int id = 0;
    short port = 0;
    long heartbeat = 0;
    long timestamp = 0;
    MemberListEntry() = default;
    MemberListEntry(int i, short p, long h, long t) : id(i), port(p), heartbeat(h), timestamp(t) {}
    MemberListEntry(int i, short p) : id(i), port(p) {}
    int getid() { return id; }
    short getport() { return port; }
    long getheartbeat() { return heartbeat; }
    long gettimestamp() { return timestamp; }
    void setid(int v) { id = v; }
    void setport(short v) { port = v; }
    void setheartbeat(long v) { heartbeat = v; }
    void settimestamp(long v) { timestamp = v; }
};

class Member {
public:
    Address addr;
    bool inited = false;
    bool inGroup = false;
    bool bFailed = false;
    int nnb = 0;
    long heartbeat = 0;
    int pingCounter = 0;
    int timeOutCounter = 0;
    std::vector<MemberListEntry> memberList;
    std::vector<MemberListEntry>::iterator myPos;
    std::queue<q_elt> mp1q;   // kept for source compatibility; queues live in the engine
    virtual ~Member() {}
};

class Params {
public:
    int MAX_NNB = 0;
    int SINGLE_FAILURE = 0;
    double MSG_DROP_PROB = 0;
    double STEP_RATE = 0.25;
    int EN_GPSZ = 0;
    int MAX_MSG_SIZE = 4000;
    int DROP_MSG = 0;
    int dropmsg = 0;
    int globaltime = 0;
    int allNodesJoined = 0;
    short PORTNUM = 8001;
    gsp_params raw{};

    Params() { gsp_params_default(&raw); }
    void setparams(char *config_file) {
        if (gsp_params_from_conf(config_file, &raw) != GSP_OK) {
            std::fprintf(stderr, "%s\n", gsp_last_error());
            std::exit(1);
        }
        MAX_NNB = raw.max_nnb;
        SINGLE_FAILURE = raw.single_failure;
        DROP_MSG = raw.drop_msg;
        MSG_DROP_PROB = raw.msg_drop_prob;
        EN_GPSZ = MAX_NNB;
        STEP_RATE = raw.step_rate;
        MAX_MSG_SIZE = raw.max_msg_size;
        globaltime = 0;
        dropmsg = 0;
        allNodesJoined = 0;
        for (int i = 0; i < EN_GPSZ; ++i) allNodesJoined += i;
    }
    int getcurrtime() { return globaltime; }
};

namespace gsp_facade {

// Process-wide state shared by the facade objects (the reference's classes share state
// through static / global variables as well: Log.cpp:46-54, Application.h nodeCount).
struct Context {
    gsp_engine *engine = nullptr;
    Params *par = nullptr;
    std::vector<Member *> members;          // by node index (id - 1)
    int kind = 0;                           // 0 none, 1 recv batch, 2 process batch
    int tick = -1, dropmsg = 0;
    std::vector<int32_t> order;
    std::vector<int8_t> ops;
    std::vector<char> in_batch;
    std::vector<Address> addrs;             // [i] = id i+1: MessageHdr::addr of handed messages
    std::unordered_set<void *> issued;      // MessageHdrs handed to driver callbacks, unconsumed
    bool snapshots = false;
    bool seeded = false;                    // srand() before the EmulNet: its seed
    uint64_t seed = 0;
    std::vector<gsp_entry> lists;           // gsp_member_lists scratch
    std::vector<int32_t> lens;

    // the engine keeps send-time lists once messages can be handled in separate batches
    void enable_snapshots() {
        if (snapshots) return;
        if (gsp_payload_snapshots(engine, 1) != GSP_OK) die("gsp_payload_snapshots");
        snapshots = true;
    }

    static void die(const char *what) {
        std::fprintf(stderr, "gossip engine: %s failed: %s\n", what, gsp_last_error());
        std::exit(1);
    }
    void require_engine() {
        if (!engine) {
            std::fprintf(stderr, "gossip engine: no EmulNet was constructed\n");
            std::exit(1);
        }
    }

    void flush() {
        if (kind == 1) {
            if (gsp_tick_recv(engine, tick, order.data(), int32_t(order.size())) != GSP_OK)
                die("gsp_tick_recv");
        } else if (kind == 2) {
            if (gsp_tick_process(engine, tick, order.data(), ops.data(), int32_t(order.size()),
                                 dropmsg) != GSP_OK)
                die("gsp_tick_process");
            refresh_nodes(order);
        }
        for (int32_t node : order) in_batch[size_t(node)] = 0;
        order.clear();
        ops.clear();
        kind = 0;
    }

    void refresh(int32_t node) {
        gsp_member_view v;
        if (gsp_get_member(engine, node, &v) != GSP_OK) die("gsp_get_member");
        Member *m = members[size_t(node)];
        if (!m) return;
        m->inited = v.inited != 0;
        m->inGroup = v.in_group != 0;
        m->heartbeat = long(v.heartbeat);
        m->nnb = v.n_members;
    }

    // the scalar fields and the member lists of `nodes` (one device read for all lists)
    void refresh_nodes(const std::vector<int32_t> &nodes) {
        if (nodes.empty()) return;
        const size_t N = members.size();
        lists.resize(nodes.size() * N);
        lens.resize(nodes.size());
        if (gsp_member_lists(engine, nodes.data(), int32_t(nodes.size()), lists.data(),
                             lens.data()) != GSP_OK)
            die("gsp_member_lists");
        for (size_t i = 0; i < nodes.size(); ++i) {
            refresh(nodes[i]);
            Member *m = members[size_t(nodes[i])];
            if (!m) continue;
            m->memberList.clear();
            for (int32_t k = 0; k < lens[i]; ++k) {
                const gsp_entry &e = lists[i * N + size_t(k)];
                m->memberList.emplace_back(e.id, e.port, long(e.heartbeat), long(e.timestamp));
            }
        }
    }
    void refresh_node(int32_t node) { refresh_nodes(std::vector<int32_t>{node}); }

    // a node whose calls are recorded but not yet run: run them (its mirror is then current)
    void settle(int32_t node) {
        if (node >= 0 && size_t(node) < in_batch.size() && in_batch[size_t(node)]) flush();
    }

    void record(int k, int32_t node, int8_t op) {
        require_engine();
        const int t = par->getcurrtime();
        const int dm = par->dropmsg;
        if (kind != 0 && (kind != k || tick != t || (k == 2 && dropmsg != dm) ||
                          in_batch[size_t(node)]))
            flush();
        kind = k;
        tick = t;
        dropmsg = dm;
        order.push_back(node);
        ops.push_back(op);
        in_batch[size_t(node)] = 1;
    }
};

inline Context &ctx() {
    static Context c;
    return c;
}

inline int32_t node_of(const Address *a) { return a ? a->id() - 1 : -1; }

}  // namespace gsp_facade

class Log {
public:
    explicit Log(Params *p) : par(p) {
        // the reference opens dbg.log and an (unused) stats.log on the first LOG call
        // (Log.cpp:56-69); the engine owns dbg.log, stats.log is created empty here
        if (FILE *f = std::fopen("stats.log", "w")) std::fclose(f);
    }
    virtual ~Log() {}
    void LOG(Address *addr, const char *str, ...) {
        char text[30000];
        va_list ap;
        va_start(ap, str);
        std::vsnprintf(text, sizeof text, str, ap);
        va_end(ap);
        auto &c = gsp_facade::ctx();
        c.require_engine();
        c.flush();
        if (gsp_log(c.engine, gsp_facade::node_of(addr), par->getcurrtime(), text) != GSP_OK)
            c.die("gsp_log");
    }
    void logNodeAdd(Address *self, Address *added) { member_line(self, added, "joined"); }
    void logNodeRemove(Address *self, Address *removed) { member_line(self, removed, "removed"); }

private:
    void member_line(Address *self, Address *who, const char *verb) {
        char line[128];
        std::snprintf(line, sizeof line, "Node %d.%d.%d.%d:%d %s at time %d", who->addr[0],
                      who->addr[1], who->addr[2], who->addr[3], int(who->port()), verb,
                      par->getcurrtime());
        LOG(self, "%s", line);
    }
    Params *par;
};

class EmulNet {
public:
    // The engine is created here (the reference's EmulNet owns the network state).  The
    // reference seeds rand() with srand(time(NULL)) (Application.cpp:50/96); the facade uses
    // the same seed -- time(NULL) -- unless GSP_SEED is set; GSP_RNG=philox selects the
    // counter-based replay stream; GSP_DEVICE selects the HIP device.
    explicit EmulNet(Params *p) : par(p) {
        auto &c = gsp_facade::ctx();
        // the seed: srand()'s when the driver seeded before constructing the EmulNet
        // (Application.cpp:50, with the forwarding headers' rand interposition), else
        // GSP_SEED, else time(NULL) as srand(time(NULL))
        const char *s = std::getenv("GSP_SEED");
        const uint64_t seed = c.seeded ? c.seed
                              : s && *s ? std::strtoull(s, nullptr, 10) : uint64_t(std::time(nullptr));
        const char *m = std::getenv("GSP_RNG");
        const gsp_rng_mode rng = (m && std::strcmp(m, "philox") == 0) ? GSP_RNG_PHILOX : GSP_RNG_GLIBC;
        const char *d = std::getenv("GSP_DEVICE");
        const int dev = d && *d ? std::atoi(d) : 0;
        if (gsp_create(&p->raw, dev, rng, seed, "dbg.log", &c.engine) != GSP_OK)
            c.die("gsp_create");
        c.par = p;
        c.members.assign(size_t(p->EN_GPSZ), nullptr);
        c.in_batch.assign(size_t(p->EN_GPSZ), 0);
        c.addrs.assign(size_t(p->EN_GPSZ), Address());
        for (int i = 0; i < p->EN_GPSZ; ++i) {
            const int id = i + 1;
            std::memcpy(&c.addrs[size_t(i)].addr[0], &id, 4);
        }
        // send-time lists are kept from the first message on, so a driver may switch from
        // recvLoop to its own ENrecv callback / recvCallBack / addMember at any tick
        c.snapshots = false;
        c.enable_snapshots();
    }
    virtual ~EmulNet();
    void *ENinit(Address *myaddr, short /*port*/) {   // ids 1, 2, ... (EmulNet.cpp:72-77)
        const int id = nextid++;
        const short port = 0;
        std::memcpy(&myaddr->addr[0], &id, 4);
        std::memcpy(&myaddr->addr[4], &port, 2);
        return myaddr;
    }
    int ENsend(Address *myaddr, Address *toaddr, char *data, int size);
    int ENsend(Address *myaddr, Address *toaddr, std::string data) {
        return ENsend(myaddr, toaddr, const_cast<char *>(data.data()), int(data.size()));
    }
    // The next rand() of the engine's global draw order.  The reference's Application::fail
    // calls libc rand() (Application.cpp:182/189), which shares its stream with the draws of
    // ENsend (EmulNet.cpp:89); with the draws inside the engine, fail() calls this instead.
    int ENrand() {
        auto &c = gsp_facade::ctx();
        c.require_engine();
        c.flush();
        int32_t v = 0;
        if (gsp_rand(c.engine, par->getcurrtime(), &v) != GSP_OK) c.die("gsp_rand");
        return v;
    }
    int ENrecv(Address *myaddr, int (*enq)(void *, char *, int), struct timeval *t, int times,
               void *queue);
    int ENcleanup() {   // writes msgcount.log for ticks [0, globaltime) (EmulNet.cpp:184-220)
        auto &c = gsp_facade::ctx();
        c.require_engine();
        c.flush();
        if (gsp_write_msgcount(c.engine, "msgcount.log", par->getcurrtime()) != GSP_OK)
            c.die("gsp_write_msgcount");
        gsp_flush_log(c.engine);
        return 0;
    }

private:
    Params *par;
    int nextid = 1;
};

enum MsgTypes { JOINREQ, JOINREP, DUMMYLASTMSGTYPE, GOSSIP };

typedef struct MessageHdr {
    enum MsgTypes msgType;
    Address *addr;
    std::vector<MemberListEntry> vector_list;
} MessageHdr;

// A message the driver built (MP1Node.cpp:355-359) carries its own vector_list.
inline int EmulNet::ENsend(Address *myaddr, Address *toaddr, char *data, int /*size*/) {
    auto &c = gsp_facade::ctx();
    c.require_engine();
    c.flush();
    const MessageHdr *h = reinterpret_cast<const MessageHdr *>(data);
    std::vector<gsp_entry> list;
    for (const MemberListEntry &e : h->vector_list)
        list.push_back(gsp_entry{e.id, e.port, int64_t(e.heartbeat), int64_t(e.timestamp)});
    static const gsp_entry none{};
    int32_t admitted = 0;
    if (gsp_send_list(c.engine, par->getcurrtime(), gsp_facade::node_of(myaddr), toaddr->id(),
                      int32_t(h->msgType), par->dropmsg, list.empty() ? &none : list.data(),
                      int32_t(list.size()), &admitted) != GSP_OK)
        c.die("gsp_send_list");
    return admitted;
}

class Queue {
public:
    static bool enqueue(std::queue<q_elt> *q, void *buffer, int size) {
        q->emplace(buffer, size);
        return true;
    }
};

class MP1Node {
public:
    MP1Node(Member *member, Params *params, EmulNet *emul, Log *log, Address *address)
        : memberNode(member), par(params), emulNet(emul), log(log) {
        memberNode->addr = *address;
        auto &c = gsp_facade::ctx();
        const int32_t node = gsp_facade::node_of(address);
        if (node >= 0 && size_t(node) < c.members.size()) c.members[size_t(node)] = member;
    }
    virtual ~MP1Node() {}
    Member *getMemberNode() {
        gsp_facade::ctx().settle(node());
        return memberNode;
    }

    int recvLoop() {
        if (memberNode->bFailed) return false;
        feed();
        return emulNet->ENrecv(&memberNode->addr, enqueueWrapper, nullptr, 1, &memberNode->mp1q);
    }
    static int enqueueWrapper(void *env, char *buff, int size) {
        return Queue::enqueue(static_cast<std::queue<q_elt> *>(env), buff, size);
    }
    void nodeStart(char * /*servaddrstr*/, short /*serverport*/) {
        // initThisNode + introduceSelfToGroup (MP1Node.cpp:95-154); the mirror is reset now,
        // the engine runs the start in the next process batch
        memberNode->bFailed = false;
        memberNode->inited = true;
        memberNode->inGroup = false;
        memberNode->nnb = 0;
        memberNode->heartbeat = 0;
        memberNode->pingCounter = TFAIL;
        memberNode->timeOutCounter = -1;
        memberNode->memberList.clear();
        gsp_facade::ctx().record(2, node(), GSP_OP_START);
    }
    int initThisNode(Address *) { return 0; }
    int introduceSelfToGroup(Address *) { return 1; }
    int finishUpThisNode() {
        gsp_facade::ctx().flush();
        memberNode->inited = false;
        memberNode->inGroup = false;
        memberNode->heartbeat = 0;
        memberNode->memberList.clear();
        return 0;
    }
    void nodeLoop() {
        if (memberNode->bFailed) return;
        feed();
        gsp_facade::ctx().record(2, node(), GSP_OP_LOOP);
    }
    void checkMessages() {
        feed();
        gsp_facade::ctx().record(2, node(), GSP_OP_CHECK);
    }
    bool recvCallBack(void *env, char *data, int size);
    void nodeLoopOps() { gsp_facade::ctx().record(2, node(), GSP_OP_OPS); }
    // MP1Node.h:77-80.  addMember changes the engine's list (gsp_add_member); check_exist
    // returns the entry of the (current) mirror, or nullptr.
    void addMember(MessageHdr *messageHdr);
    void addMember(MemberListEntry *m);
    MemberListEntry *check_exist(int id, short port) {
        gsp_facade::ctx().settle(node());
        for (MemberListEntry &e : memberNode->memberList)
            if (e.id == id && e.port == port) return &e;
        return nullptr;
    }
    MemberListEntry *check_exist(Address *addr) { return check_exist(addr->id(), addr->port()); }
    int isNullAddress(Address *a) {
        static const char zero[6] = {0};
        return std::memcmp(a->addr, zero, 6) == 0 ? 1 : 0;
    }
    Address getJoinAddress() {
        Address a;
        const int id = 1;
        std::memcpy(&a.addr[0], &id, 4);
        return a;
    }
    void initMemberListTable(Member *m) { m->memberList.clear(); }
    void printAddress(Address *a) {
        std::printf("%d.%d.%d.%d:%d \n", a->addr[0], a->addr[1], a->addr[2], a->addr[3],
                    int(a->port()));
    }
    // Run all recorded work and re-read this node's mirror from the device (kept from ABI 5;
    // the mirror is current after every batch now).
    Member *syncMember() {
        auto &c = gsp_facade::ctx();
        c.flush();
        c.refresh_node(node());
        return memberNode;
    }

    // Hand what driver callbacks left in mp1q to the engine's queue of this node, in order.
    void feed();

private:
    int32_t node() const { return gsp_facade::node_of(&memberNode->addr); }
    Member *memberNode;
    Params *par;
    EmulNet *emulNet;
    Log *log;
};

namespace gsp_facade {

// A MessageHdr as the engine's message: sender, type and the list it carries.
inline bool to_msg(const MessageHdr *h, gsp_queued_msg &q, std::vector<gsp_entry> &list) {
    if (h->msgType != JOINREQ && h->msgType != JOINREP && h->msgType != GOSSIP)
        return false;   // no branch of recvCallBack handles it (MP1Node.cpp:221-257)
    if (!h->addr) {
        std::fprintf(stderr, "gossip engine: MessageHdr without addr\n");
        std::exit(1);
    }
    q = gsp_queued_msg{};
    q.src_id = h->addr->id();
    q.type = int32_t(h->msgType);
    q.send_batch = -1;
    q.payload_len = int32_t(h->vector_list.size());
    list.clear();
    for (const MemberListEntry &e : h->vector_list)
        list.push_back(gsp_entry{e.id, e.port, int64_t(e.heartbeat), int64_t(e.timestamp)});
    return true;
}

inline const gsp_entry *list_ptr(const std::vector<gsp_entry> &list) {
    static const gsp_entry none{};
    return list.empty() ? &none : list.data();   // non-NULL: the list is the message's (empty)
}

inline void release(MessageHdr *h) {
    ctx().issued.erase(h);
    delete h;
}

}  // namespace gsp_facade

inline EmulNet::~EmulNet() {
    auto &c = gsp_facade::ctx();
    if (c.engine) {
        c.flush();
        gsp_destroy(c.engine);
        c.engine = nullptr;
    }
    for (void *h : c.issued) delete static_cast<MessageHdr *>(h);   // never handled
    c.issued.clear();
}

inline int EmulNet::ENrecv(Address *myaddr, int (*enq)(void *, char *, int), struct timeval *,
                           int, void *queue) {
    auto &c = gsp_facade::ctx();
    c.require_engine();
    const int32_t node = gsp_facade::node_of(myaddr);
    if (node < 0 || size_t(node) >= c.members.size()) {
        std::fprintf(stderr, "gossip engine: ENrecv for an unknown address\n");
        std::exit(1);
    }
    Member *m = c.members[size_t(node)];
    if (enq == &MP1Node::enqueueWrapper && m && queue == &m->mp1q) {
        c.record(1, node, 0);   // batched: the messages stay in the engine's queue
        return 0;
    }
    c.flush();
    c.enable_snapshots();
    const int t = par->getcurrtime();
    int32_t n = 0;
    int64_t np = 0;
    if (gsp_recv_detach(c.engine, t, node, nullptr, 0, nullptr, 0, &n, &np) != GSP_OK)
        c.die("gsp_recv_detach");
    if (n == 0) return 0;
    std::vector<gsp_queued_msg> msgs(static_cast<size_t>(n));
    std::vector<gsp_entry> lists(size_t(np) + 1);
    if (gsp_recv_detach(c.engine, t, node, msgs.data(), n, lists.data(), np, &n, &np) != GSP_OK)
        c.die("gsp_recv_detach");
    for (const gsp_queued_msg &q : msgs) {   // EmulNet.cpp:151-162: (*enq)(queue, tmp, sz)
        MessageHdr *h = new MessageHdr();
        h->msgType = MsgTypes(q.type);
        h->addr = &c.addrs[size_t(q.src_id - 1)];
        h->vector_list.reserve(size_t(q.payload_len));
        for (int32_t i = 0; i < q.payload_len; ++i) {
            const gsp_entry &e = lists[size_t(q.payload_off + i)];
            h->vector_list.emplace_back(e.id, e.port, long(e.heartbeat), long(e.timestamp));
        }
        c.issued.insert(h);
        enq(queue, reinterpret_cast<char *>(h), int(sizeof(MessageHdr)));
    }
    return 0;
}

inline void MP1Node::feed() {
    auto &c = gsp_facade::ctx();
    if (memberNode->mp1q.empty()) return;
    // a batch already recorded for this node runs before these messages arrive
    if (c.in_batch[size_t(node())]) c.flush();
    gsp_queued_msg q;
    std::vector<gsp_entry> list;
    while (!memberNode->mp1q.empty()) {
        MessageHdr *h = static_cast<MessageHdr *>(memberNode->mp1q.front().elt);
        memberNode->mp1q.pop();
        if (gsp_facade::to_msg(h, q, list) &&
            gsp_queue_push(c.engine, node(), &q, gsp_facade::list_ptr(list)) != GSP_OK)
            c.die("gsp_queue_push");
        gsp_facade::release(h);
    }
}

inline bool MP1Node::recvCallBack(void *, char *data, int) {
    auto &c = gsp_facade::ctx();
    c.require_engine();
    MessageHdr *h = reinterpret_cast<MessageHdr *>(data);
    gsp_queued_msg q;
    std::vector<gsp_entry> list;
    if (gsp_facade::to_msg(h, q, list)) {
        c.flush();
        c.enable_snapshots();
        if (gsp_recv_callback(c.engine, par->getcurrtime(), node(), &q, gsp_facade::list_ptr(list),
                              par->dropmsg) != GSP_OK)
            c.die("gsp_recv_callback");
        c.refresh_node(node());
    }
    gsp_facade::release(h);
    return true;
}

inline void MP1Node::addMember(MessageHdr *messageHdr) {   // MP1Node.cpp:265-280
    auto &c = gsp_facade::ctx();
    c.require_engine();
    c.flush();
    const gsp_entry e{messageHdr->addr->id(), messageHdr->addr->port(), 1, par->getcurrtime()};
    int32_t added = 0;
    if (gsp_add_member(c.engine, par->getcurrtime(), node(), &e, GSP_ADD_SENDER, &added) != GSP_OK)
        c.die("gsp_add_member");
    if (added) c.refresh_node(node());
}

inline void MP1Node::addMember(MemberListEntry *m) {        // MP1Node.cpp:282-301
    auto &c = gsp_facade::ctx();
    c.require_engine();
    c.flush();
    const gsp_entry e{m->id, m->port, int64_t(m->heartbeat), int64_t(m->timestamp)};
    int32_t added = 0;
    if (gsp_add_member(c.engine, par->getcurrtime(), node(), &e, GSP_ADD_COPY, &added) != GSP_OK)
        c.die("gsp_add_member");
    if (added) c.refresh_node(node());
}

// rand() / srand() of a driver that shares its stream with EmulNet (header comment).
inline void gsp_mp1_srand(unsigned int seed) {
    auto &c = gsp_facade::ctx();
    if (!c.engine) {                  // before the EmulNet: the seed it is created with
        c.seeded = true;
        c.seed = seed;
        return;
    }
    c.flush();                        // recorded sends draw from the stream they were made on
    if (gsp_srand(c.engine, seed) != GSP_OK) c.die("gsp_srand");
}

inline int gsp_mp1_rand() {
    auto &c = gsp_facade::ctx();
    c.require_engine();
    c.flush();
    int32_t v = 0;
    if (gsp_rand(c.engine, c.par->getcurrtime(), &v) != GSP_OK) c.die("gsp_rand");
    return v;
}
