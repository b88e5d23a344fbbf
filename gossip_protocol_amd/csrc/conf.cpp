// gossip_protocol_amd/csrc/conf.cpp -- .conf files for the scale engines.
//
// A reference testcase (/root/reference/testcases/*.conf) is four fscanf literal prefixes
// (Params.cpp:22-25): MAX_NNB, SINGLE_FAILURE, DROP_MSG, MSG_DROP_PROB.  The scale parsers read
// those four exactly as Params::setparams does -- so every reference .conf parses unchanged --
// and map them onto the scale protocol the way the reference's driver uses them:
//   MAX_NNB          n
//   SINGLE_FAILURE   1: one Philox-chosen node crashes at t = 100 (Application.cpp:180-187),
//                    0: n/2 contiguous nodes from (Philox % n)/2 at t = 100 (:188-196)
//   DROP_MSG         1: drop_pct = (int)(MSG_DROP_PROB * 100) (EmulNet.cpp:91) for the sends of
//                    ticks [51, 301): fail() sets dropmsg at the END of t = 50, after that
//                    tick's mp1Run, and clears it at the end of t = 300 (Application.cpp:99-104,
//                    177, 198) -- the same end-of-tick rule as the crash events; 0: no drops
//   (fixed)          STEP_RATE 0.25 (Params.cpp:30), 700 ticks (Application.h:27), TREMOVE 20
// Any further lines are optional "KEY: value..." pairs that the reference's fscanf never
// reaches (they follow the fourth key):
//   SCALE_N n | FANOUT f | VIEW V | INBOX K | TREMOVE t | TFAIL t | SWIM s | H0 h | SEED u64 |
//   TICKS t | STEP_RATE x | INTRO_LIST B | DROP_PCT p | DROP_WINDOW from until |
//   FAIL tick mode ppm (repeatable; mode RANDOM|BLOCK|SINGLE|HALF|0-4; the first FAIL line
//   replaces the SINGLE_FAILURE event) | EVENTS 0|1 | EVENT_CAP n | EVICT_ORDER 0|1
// Full view: VIEW / INBOX / EVICT_ORDER are refused.  Partial view: every key applies.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "common.hpp"
#include "pview_kernels.hpp"

namespace {

struct ConfAll {
    int32_t n = 0, fanout = 3, view = 256, inbox = 7, tremove = 20, tfail = 0, swim = 0, h0 = 1;
    int32_t drop_pct = 0, ticks = 700, events = 0, evict_order = 0;
    int64_t event_cap = 0;
    uint64_t seed = 0x5EED;
    gsp_fail_event first{100, GSP_FAIL_SINGLE, 0};
    gsp_policy pol{};
    bool have_view = false;
};

int parse_mode(const char *s, int32_t *mode) {
    static const char *names[] = {"NONE", "RANDOM", "BLOCK", "SINGLE", "HALF"};
    for (int32_t i = 0; i < 5; ++i)
        if (std::strcmp(s, names[i]) == 0) { *mode = i; return 1; }
    char *end = nullptr;
    const long v = std::strtol(s, &end, 10);
    if (end && *end == 0 && v >= 0 && v <= 4) { *mode = int32_t(v); return 1; }
    return 0;
}

int read_conf(const char *path, ConfAll &c) {
    GSP_REQUIRE(path, GSP_ERR_INVALID, "params_from_conf: NULL path");
    FILE *f = std::fopen(path, "r");
    GSP_REQUIRE(f, GSP_ERR_IO, "params_from_conf: cannot open %s", path);
    int nnb = 0, single = 0, drop = 0;
    double prob = 0.0;
    int ok = 1;                                        // Params.cpp:22-25, verbatim grammar
    ok &= std::fscanf(f, "MAX_NNB: %d", &nnb) == 1;
    ok &= std::fscanf(f, "\nSINGLE_FAILURE: %d", &single) == 1;
    ok &= std::fscanf(f, "\nDROP_MSG: %d", &drop) == 1;
    ok &= std::fscanf(f, "\nMSG_DROP_PROB: %lf", &prob) == 1;
    if (!ok) {
        std::fclose(f);
        GSP_REQUIRE(false, GSP_ERR_IO, "params_from_conf: %s does not start with the MAX_NNB / "
                    "SINGLE_FAILURE / DROP_MSG / MSG_DROP_PROB keys (Params.cpp:22-25)", path);
    }
    c.n = nnb;
    c.first = gsp_fail_event{100, single ? GSP_FAIL_SINGLE : GSP_FAIL_HALF, 0};
    if (drop) {
        c.drop_pct = int32_t(prob * 100);             // EmulNet.cpp:91
        c.pol.drop_from = 51;                          // set at the end of t = 50
        c.pol.drop_until = 301;                        // cleared at the end of t = 300
    }
    c.pol.step_rate = 0.25;                            // Params.cpp:30
    bool first_fail = true;
    char line[512];
    int lineno = 4;
    while (std::fgets(line, sizeof line, f)) {
        ++lineno;
        char key[64] = {0};
        int used = 0;
        if (std::sscanf(line, " %63[A-Z_0-9]:%n", key, &used) < 1 || !used) {
            bool blank = true;
            for (const char *p = line; *p; ++p) blank = blank && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r');
            if (blank) continue;
            std::fclose(f);
            GSP_REQUIRE(false, GSP_ERR_INVALID, "%s:%d: expected KEY: value", path, lineno);
        }
        const char *v = line + used;
        long long a = 0, b = 0;
        double x = 0;
        char mode[32] = {0};
        bool good = true;
        const std::string k(key);
        auto one = [&](int32_t *dst) { good = std::sscanf(v, "%lld", &a) == 1; if (good) *dst = int32_t(a); };
        if (k == "SCALE_N") one(&c.n);
        else if (k == "FANOUT") one(&c.fanout);
        else if (k == "VIEW") { one(&c.view); c.have_view = true; }
        else if (k == "INBOX") { one(&c.inbox); c.have_view = true; }
        else if (k == "EVICT_ORDER") { one(&c.evict_order); c.have_view = true; }
        else if (k == "TREMOVE") one(&c.tremove);
        else if (k == "TFAIL") one(&c.tfail);
        else if (k == "SWIM") one(&c.swim);
        else if (k == "H0") one(&c.h0);
        else if (k == "TICKS") one(&c.ticks);
        else if (k == "EVENTS") one(&c.events);
        else if (k == "INTRO_LIST") one(&c.pol.intro_list);
        else if (k == "DROP_PCT") one(&c.drop_pct);
        else if (k == "EVENT_CAP") { good = std::sscanf(v, "%lld", &a) == 1; c.event_cap = a; }
        else if (k == "SEED") { good = std::sscanf(v, "%lld", &a) == 1; c.seed = uint64_t(a); }
        else if (k == "STEP_RATE") { good = std::sscanf(v, "%lf", &x) == 1; c.pol.step_rate = x; }
        else if (k == "DROP_WINDOW") {
            good = std::sscanf(v, "%lld %lld", &a, &b) == 2;
            c.pol.drop_from = int32_t(a);
            c.pol.drop_until = int32_t(b);
        } else if (k == "FAIL") {
            int32_t m = 0;
            good = std::sscanf(v, "%lld %31s %lld", &a, mode, &b) == 3 && parse_mode(mode, &m);
            const gsp_fail_event e{int32_t(a), m, int32_t(b)};
            if (good && first_fail) { c.first = e; first_fail = false; }
            else if (good) {
                good = c.pol.n_fail_events < GSP_MAX_FAIL_EVENTS;
                if (good) c.pol.fail_events[c.pol.n_fail_events++] = e;
            }
        } else {
            std::fclose(f);
            GSP_REQUIRE(false, GSP_ERR_INVALID, "%s:%d: unknown key %s", path, lineno, key);
        }
        if (!good) {
            std::fclose(f);
            GSP_REQUIRE(false, GSP_ERR_INVALID, "%s:%d: bad value for %s", path, lineno, key);
        }
    }
    std::fclose(f);
    return GSP_OK;
}

}  // namespace

extern "C" {

int gsp_scale_params_from_conf(const char *path, gsp_scale_params *out) {
    GSP_REQUIRE(out, GSP_ERR_INVALID, "gsp_scale_params_from_conf: out is NULL");
    ConfAll c;
    if (int rc = read_conf(path, c)) return rc;
    GSP_REQUIRE(!c.have_view, GSP_ERR_INVALID, "%s: VIEW / INBOX / EVICT_ORDER are partial-view keys", path);
    std::memset(out, 0, sizeof *out);
    out->n = c.n;
    out->fanout = c.fanout;
    out->drop_pct = c.drop_pct;
    out->tremove = c.tremove;
    out->h0 = c.h0;
    out->fail_mode = c.first.mode;
    out->fail_tick = c.first.tick;
    out->fail_ppm = c.first.ppm;
    out->seed = c.seed;
    out->max_ticks = c.ticks;
    out->tfail = c.tfail;
    out->swim = c.swim;
    out->policy = c.pol;
    out->events = c.events;
    out->event_cap = c.event_cap;
    return GSP_OK;
}

int gsp_pview_params_from_conf(const char *path, gsp_pview_params *out) {
    GSP_REQUIRE(out, GSP_ERR_INVALID, "gsp_pview_params_from_conf: out is NULL");
    ConfAll c;
    if (int rc = read_conf(path, c)) return rc;
    std::memset(out, 0, sizeof *out);
    out->n = c.n;
    out->view = c.view;
    out->fanout = c.fanout;
    out->inbox = c.inbox;
    out->drop_pct = c.drop_pct;
    out->tremove = c.tremove;
    out->h0 = c.h0;
    out->fail_mode = c.first.mode;
    out->fail_tick = c.first.tick;
    out->fail_ppm = c.first.ppm;
    out->seed = c.seed;
    out->max_ticks = c.ticks;
    out->tfail = c.tfail;
    out->swim = c.swim;
    out->policy = c.pol;
    out->events = c.events;
    out->event_cap = c.event_cap;
    out->evict_order = c.evict_order;
    return GSP_OK;
}

// sizeof of the public structs, for bindings to check their layout against (0: unknown name)
int64_t gsp_struct_size(const char *name) {
    if (!name) return 0;
    const std::string s(name);
    if (s == "gsp_params") return int64_t(sizeof(gsp_params));
    if (s == "gsp_member_view") return int64_t(sizeof(gsp_member_view));
    if (s == "gsp_entry") return int64_t(sizeof(gsp_entry));
    if (s == "gsp_queued_msg") return int64_t(sizeof(gsp_queued_msg));
    if (s == "gsp_exact_stats") return int64_t(sizeof(gsp_exact_stats));
    if (s == "gsp_fail_event") return int64_t(sizeof(gsp_fail_event));
    if (s == "gsp_policy") return int64_t(sizeof(gsp_policy));
    if (s == "gsp_scale_params") return int64_t(sizeof(gsp_scale_params));
    if (s == "gsp_scale_digest") return int64_t(sizeof(gsp_scale_digest));
    if (s == "gsp_scale_perf") return int64_t(sizeof(gsp_scale_perf));
    if (s == "gsp_pview_params") return int64_t(sizeof(gsp_pview_params));
    if (s == "gsp_pview_digest") return int64_t(sizeof(gsp_pview_digest));
    return 0;
}

}  // extern "C"
