// gossip_protocol_amd/csrc/policy.hpp -- driver policies of the scale engines (host side).
//
// The reference's driver hard-codes them (Application.cpp:143 join schedule, :177/:198 drop
// window, :180-196 crash injection); gsp_policy (include/gossip/gossip.h) makes them data:
// a start tick and a crash tick per node (alive at t iff start <= t <= crash), the drop
// percentage of the sends of each tick, and the JOINREPs the introducer (node 0) sends at
// t - 1 to the nodes that start at t.
#pragma once
#include <cstdint>
#include <vector>

#include "gossip/gossip.h"

namespace gsp {

int validate_policy(const gsp_policy &p, int32_t n);
std::vector<int32_t> start_ticks(const gsp_policy &p, int32_t n);
// crash tick of every node (INT32_MAX: never): the event (mode0, tick0, ppm0) with draw
// index 0, then p.fail_events[e] with index e + 1; a node crashes at its earliest event
std::vector<int32_t> fail_ticks(const gsp_policy &p, int32_t n, uint64_t seed, int32_t mode0,
                                int32_t tick0, int32_t ppm0);
int32_t drop_at(const gsp_policy &p, int32_t drop_pct, int32_t t);

// The joiners of every start tick (nodes with start > 0), ascending within a tick:
// at(t) = [joiners.data() + ofs[t], joiners.data() + ofs[t + 1]) for 1 <= t <= max_tick.
struct JoinPlan {
    std::vector<int32_t> joiners;
    std::vector<int64_t> ofs;
    int64_t count(int32_t t) const {
        return t >= 0 && size_t(t) + 1 < ofs.size() ? ofs[size_t(t) + 1] - ofs[size_t(t)] : 0;
    }
    int64_t first(int32_t t) const { return t >= 0 && size_t(t) < ofs.size() ? ofs[size_t(t)] : 0; }
};
JoinPlan join_plan(const std::vector<int32_t> &start, int32_t max_tick);

}  // namespace gsp
