/*
 * oracle/ref_hooks.cpp -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Link-time hooks for the *unmodified* reference objects (built from
 * /root/reference by oracle/Makefile), attached with GNU ld --wrap so that no
 * reference source line is edited or copied:
 *
 *  1. Philox replay hook (north_star "EmulNet replay hook"): with GSP_RNG=philox every
 *     rand() draw is replaced by a counter-based Philox4x32-10 draw.
 *       - draw inside EmulNet::ENsend (/root/reference/EmulNet.cpp:89) -> counter
 *         (tick, src id, dst id, msgType), domain SEND;
 *       - draw inside Application::fail (/root/reference/Application.cpp:182/189) ->
 *         counter (tick, 0, 0, 0), domain FAIL.
 *     The ENsend context is captured by wrapping EmulNet::ENsend itself (its caller,
 *     MP1Node.o, references it as an undefined symbol).
 *  2. End-of-tick state dump (GSP_STATE_DUMP=<path>): Params::getcurrtime is wrapped;
 *     the first call that observes a new globaltime dumps the state of every node as
 *     it stood after Application::fail() of the previous tick
 *     (/root/reference/Application.cpp:99-104).  The Member* of each node is captured
 *     by wrapping the MP1Node constructor (/root/reference/MP1Node.cpp:19).
 *     Line format:  t id inited inGroup bFailed heartbeat |L| id:hb:ts ...
 *  3. Draw trace (GSP_DRAW_TRACE=<path>): one line per rand() draw:
 *     g tick kind src dst type value      (kind: S = ENsend, F = fail)
 */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <vector>

#include "MP1Node.h"   /* reference header, read in place via -I/root/reference */

extern "C" {
#include "gsp_philox.h"
}

namespace {
std::vector<Member *> g_members;
int g_last_tick = -1;
int g_tick = 0;
bool g_in_send = false;
uint32_t g_src = 0, g_dst = 0, g_type = 0;
uint64_t g_draws = 0;
FILE *g_dump = nullptr;
FILE *g_trace = nullptr;
int g_mode = -1; /* 0 glibc, 1 philox */

int rng_mode() {
    if (g_mode < 0) {
        const char *m = getenv("GSP_RNG");
        g_mode = (m && strcmp(m, "philox") == 0) ? 1 : 0;
        const char *d = getenv("GSP_STATE_DUMP");
        if (d && *d) g_dump = fopen(d, "w");
        const char *tr = getenv("GSP_DRAW_TRACE");
        if (tr && *tr) g_trace = fopen(tr, "w");
    }
    return g_mode;
}

uint64_t seed_from_env() {
    const char *s = getenv("GSP_SEED");
    return s ? (uint64_t)strtoull(s, nullptr, 10) : 0;
}

int addr_id(const Address *a) {
    int id;
    memcpy(&id, &a->addr[0], sizeof(int));
    return id;
}

void dump_tick(int t) {
    if (!g_dump) return;
    for (Member *m : g_members) {
        fprintf(g_dump, "%d %d %d %d %d %ld %zu", t, addr_id(&m->addr), (int)m->inited,
                (int)m->inGroup, (int)m->bFailed, m->heartbeat, m->memberList.size());
        for (const MemberListEntry &e : m->memberList)
            fprintf(g_dump, " %d:%ld:%ld", e.id, e.heartbeat, e.timestamp);
        fputc('\n', g_dump);
    }
    fflush(g_dump);
}
} // namespace

extern "C" {
int __real__ZN6Params11getcurrtimeEv(Params *self);
int __wrap__ZN6Params11getcurrtimeEv(Params *self) {
    rng_mode();
    int t = self->globaltime;
    if (t != g_last_tick) {
        if (g_last_tick >= 0) dump_tick(g_last_tick);
        g_last_tick = t;
    }
    g_tick = t;
    return __real__ZN6Params11getcurrtimeEv(self);
}

void __real__ZN7MP1NodeC1EP6MemberP6ParamsP7EmulNetP3LogP7Address(MP1Node *, Member *, Params *,
                                                                  EmulNet *, Log *, Address *);
void __wrap__ZN7MP1NodeC1EP6MemberP6ParamsP7EmulNetP3LogP7Address(MP1Node *self, Member *m,
                                                                  Params *p, EmulNet *en,
                                                                  Log *lg, Address *a) {
    g_members.push_back(m);
    __real__ZN7MP1NodeC1EP6MemberP6ParamsP7EmulNetP3LogP7Address(self, m, p, en, lg, a);
}

int __real__ZN7EmulNet6ENsendEP7AddressS1_Pci(EmulNet *, Address *, Address *, char *, int);
int __wrap__ZN7EmulNet6ENsendEP7AddressS1_Pci(EmulNet *self, Address *from, Address *to,
                                              char *data, int size) {
    g_in_send = true;
    g_src = (uint32_t)addr_id(from);
    g_dst = (uint32_t)addr_id(to);
    g_type = (uint32_t)((MessageHdr *)data)->msgType;
    int r = __real__ZN7EmulNet6ENsendEP7AddressS1_Pci(self, from, to, data, size);
    g_in_send = false;
    return r;
}

int __real_rand(void);
int __wrap_rand(void) {
    int v;
    const bool philox = rng_mode() == 1;
    if (philox) {
        uint64_t seed = seed_from_env();
        if (g_in_send)
            v = (int)gsp_philox_u31(GSP_DOMAIN_SEND, seed, (uint32_t)g_tick, g_src, g_dst, g_type);
        else
            v = (int)gsp_philox_u31(GSP_DOMAIN_FAIL, seed, (uint32_t)g_tick, 0, 0, 0);
    } else {
        v = __real_rand();
    }
    if (g_trace) {
        if (g_in_send)
            fprintf(g_trace, "%llu %d S %u %u %u %d\n", (unsigned long long)g_draws, g_tick, g_src,
                    g_dst, g_type, v);
        else
            fprintf(g_trace, "%llu %d F 0 0 0 %d\n", (unsigned long long)g_draws, g_tick, v);
    }
    ++g_draws;
    return v;
}
} // extern "C"
