// gossip_protocol_amd/csrc/events.cpp -- event records -> dbg.log lines (gsp_events_write_log).
//
// The tick kernels emit join / remove / evict records (scale_kernels.hpp event_record); the
// reference writes each as a Log line (Log::logNodeAdd / logNodeRemove, Log.cpp:116-130):
//   "\n " + addr(r) + " [" + t + "] " + "Node " + addr(x) + " joined at time " + t
// with addr = "%d.%d.%d.%d:%d" over the signed bytes of the little-endian id and the port
// (Log.cpp:73), id = index + 1 (EmulNet.cpp:72-77), port 0.
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "common.hpp"

namespace {

void addr(char *out, size_t cap, uint32_t index) {
    const int32_t id = int32_t(index) + 1;
    signed char b[4];
    std::memcpy(b, &id, 4);
    std::snprintf(out, cap, "%d.%d.%d.%d:%d", b[0], b[1], b[2], b[3], 0);
}

}  // namespace

extern "C" int gsp_events_write_log(uint64_t *ev, int64_t n, const char *path) {
    GSP_REQUIRE(path && n >= 0 && (ev || n == 0), GSP_ERR_INVALID, "gsp_events_write_log: bad argument");
    auto kind = [](uint64_t e) { return uint32_t(e >> 62); };
    auto tick = [](uint64_t e) { return uint32_t(e >> 42) & 0xFFFFFu; };
    auto row = [](uint64_t e) { return uint32_t(e >> 21) & 0x1FFFFFu; };
    auto mem = [](uint64_t e) { return uint32_t(e) & 0x1FFFFFu; };
    std::sort(ev, ev + n, [&](uint64_t a, uint64_t b) {
        if (tick(a) != tick(b)) return tick(a) < tick(b);
        if (row(a) != row(b)) return row(a) > row(b);          // phase P: descending node
        if (kind(a) != kind(b)) return kind(a) < kind(b);      // joins, removes, evictions
        return mem(a) < mem(b);
    });
    FILE *f = std::fopen(path, "a");
    GSP_REQUIRE(f, GSP_ERR_IO, "gsp_events_write_log: cannot open %s", path);
    if (std::ftell(f) == 0) {
        int sum = 0;                                           // Log.cpp:79-88: "%x\n" of
        for (const char *c = "CS425"; *c; ++c) sum += *c;      // the sum of "CS425"
        std::fprintf(f, "%x\n", sum);
    }
    static const char *verb[4] = {"?", "joined", "removed", "evicted"};
    char ra[40], xa[40];
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t e = ev[i];
        addr(ra, sizeof ra, row(e));
        addr(xa, sizeof xa, mem(e));
        std::fprintf(f, "\n %s [%u] Node %s %s at time %u", ra, tick(e), xa, verb[kind(e) & 3u], tick(e));
    }
    std::fclose(f);
    return GSP_OK;
}
