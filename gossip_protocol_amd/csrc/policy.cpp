// gossip_protocol_amd/csrc/policy.cpp -- driver policies of the scale engines (policy.hpp).
#include "policy.hpp"

#include <algorithm>
#include <climits>

#include "common.hpp"
#include "philox.hpp"

namespace gsp {

int validate_policy(const gsp_policy &p, int32_t n) {
    GSP_REQUIRE(p.step_rate >= 0.0 && p.step_rate < 1e6, GSP_ERR_INVALID, "step_rate=%g", p.step_rate);
    GSP_REQUIRE(p.intro_list >= 0 && p.intro_list <= 16, GSP_ERR_INVALID,
                "intro_list=%d outside [0, 16]", p.intro_list);
    GSP_REQUIRE(p.n_fail_events >= 0 && p.n_fail_events <= GSP_MAX_FAIL_EVENTS, GSP_ERR_INVALID,
                "n_fail_events=%d outside [0, %d]", p.n_fail_events, GSP_MAX_FAIL_EVENTS);
    for (int32_t e = 0; e < p.n_fail_events; ++e) {
        const gsp_fail_event &f = p.fail_events[e];
        GSP_REQUIRE(f.mode >= GSP_FAIL_NONE && f.mode <= GSP_FAIL_HALF && f.tick >= 0 &&
                        f.ppm >= 0 && f.ppm <= 1000000,
                    GSP_ERR_INVALID, "fail event %d: tick %d mode %d ppm %d", e, f.tick, f.mode, f.ppm);
    }
    GSP_REQUIRE(p.drop_from >= 0, GSP_ERR_INVALID, "drop_from=%d", p.drop_from);
    (void)n;
    return GSP_OK;
}

std::vector<int32_t> start_ticks(const gsp_policy &p, int32_t n) {
    std::vector<int32_t> s(size_t(n), 0);
    if (p.step_rate > 0)
        for (int32_t i = 0; i < n; ++i) s[size_t(i)] = int32_t(p.step_rate * i);   // Application.cpp:143
    return s;
}

namespace {
void apply_event(int32_t n, uint64_t seed, uint32_t d, int32_t mode, int32_t tick, int32_t ppm,
                 std::vector<int32_t> &f) {
    const uint32_t T = uint32_t(tick);
    auto crash = [&](int64_t r) { f[size_t(r)] = std::min(f[size_t(r)], tick); };
    switch (mode) {
        case GSP_FAIL_RANDOM:
            for (int32_t r = 0; r < n; ++r)
                if (draw_u31(kDomainFail, seed, T, uint32_t(r), 0, d) % 1000000u < uint32_t(ppm)) crash(r);
            break;
        case GSP_FAIL_BLOCK: {
            const int64_t m = int64_t(n) * ppm / 1000000;
            const uint32_t s0 = draw_u31(kDomainFail, seed, T, 0xFFFFFFFFu, 0, d) % uint32_t(n);
            for (int64_t i = 0; i < m; ++i) crash((s0 + i) % uint32_t(n));
            break;
        }
        case GSP_FAIL_SINGLE:      // rand() % N (Application.cpp:182)
            crash(draw_u31(kDomainFail, seed, T, 0xFFFFFFFEu, 0, d) % uint32_t(n));
            break;
        case GSP_FAIL_HALF: {      // (rand() % N) / 2 .. + N/2 - 1 (Application.cpp:189-195)
            const int32_t first = int32_t(draw_u31(kDomainFail, seed, T, 0xFFFFFFFDu, 0, d) % uint32_t(n)) / 2;
            for (int32_t r = first; r < first + n / 2; ++r) crash(r);
            break;
        }
        default: break;
    }
}
}  // namespace

std::vector<int32_t> fail_ticks(const gsp_policy &p, int32_t n, uint64_t seed, int32_t mode0,
                                int32_t tick0, int32_t ppm0) {
    std::vector<int32_t> f(size_t(n), INT32_MAX);
    apply_event(n, seed, 0, mode0, tick0, ppm0, f);
    for (int32_t e = 0; e < p.n_fail_events; ++e)
        apply_event(n, seed, uint32_t(e + 1), p.fail_events[e].mode, p.fail_events[e].tick,
                    p.fail_events[e].ppm, f);
    return f;
}

int32_t drop_at(const gsp_policy &p, int32_t drop_pct, int32_t t) {
    if (t < p.drop_from) return 0;
    if (p.drop_until > 0 && t >= p.drop_until) return 0;
    return drop_pct;
}

JoinPlan join_plan(const std::vector<int32_t> &start, int32_t max_tick) {
    JoinPlan jp;
    jp.ofs.assign(size_t(max_tick) + 2, 0);
    for (int32_t s : start)
        if (s > 0 && s <= max_tick) jp.ofs[size_t(s) + 1]++;
    for (size_t t = 1; t < jp.ofs.size(); ++t) jp.ofs[t] += jp.ofs[t - 1];
    jp.joiners.resize(size_t(jp.ofs.back()));
    std::vector<int64_t> fill(jp.ofs.begin(), jp.ofs.end());
    for (size_t i = 0; i < start.size(); ++i)
        if (start[i] > 0 && start[i] <= max_tick) jp.joiners[size_t(fill[size_t(start[i])]++)] = int32_t(i);
    return jp;
}

}  // namespace gsp

extern "C" int gsp_fail_schedule(const gsp_policy *pol, int32_t n, uint64_t seed, int32_t mode,
                                 int32_t tick, int32_t ppm, int32_t *out) {
    GSP_REQUIRE(out && n >= 1 && mode >= 0 && mode <= 4, GSP_ERR_INVALID,
                "gsp_fail_schedule: n=%d mode=%d", n, mode);
    gsp_policy none{};
    const gsp_policy &p = pol ? *pol : none;
    if (int rc = gsp::validate_policy(p, n)) return rc;
    const std::vector<int32_t> f = gsp::fail_ticks(p, n, seed, mode, tick, ppm);
    std::copy(f.begin(), f.end(), out);
    return GSP_OK;
}
