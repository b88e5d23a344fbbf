// gossip_protocol_amd/csrc/join_kernels.hpp -- JOINREP messages of the join schedule (both
// scale engines).
//
// At the end of tick t the introducer (node 0, MP1Node.cpp:378-386) sends a JOINREP to every
// node that starts at t + 1 (policy.hpp), if it is alive at t; the message takes the drop draw
// Philox(SEND; t, 0, j, JOINREP) like any send (EmulNet.cpp:89).  A surviving JOINREP joins
// the receiver's CSR segment of tick t + 1 with sender id -1 (it sorts first; node 0 sends a
// joiner nothing else), and the tick kernel merges it like a GOSSIP from node 0 whose payload
// is the bounded introducer list (gossip.h gsp_policy.intro_list).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsp {

constexpr int32_t kJoinRepSrc = -1;   // csr_src of a JOINREP
constexpr int32_t kMaxIntro = 16;     // bound of gsp_policy.intro_list

struct JoinSendArgs {
    const int32_t *joiners;          // the nodes that start at tick + 1
    int32_t count;
    int32_t tick;                    // the send tick
    int32_t drop_pct;                // drop percentage of the sends of `tick`
    uint64_t seed;
    const int32_t *fail_tick;        // [n]: node 0 sends only while alive
    int32_t lo, hi;                  // handled here: joiners in [lo, hi) (a row shard's rows)
    int32_t *ok;                     // [count] 1: the JOINREP is delivered at tick + 1
    int32_t *deg;                    // [n] messages per destination (global ids)
    unsigned long long *sent, *dropped;   // digest counters of `tick` (null: not counted here)
};
hipError_t launch_join_send(const JoinSendArgs &a, hipStream_t st);

// csr_src[off[j - row0] + fill[j - row0]++] = kJoinRepSrc for every delivered JOINREP of a
// joiner in [row0, row0 + rows); csr_slot (row layout) gets 0 there (unused for a JOINREP)
hipError_t launch_join_scatter(const int32_t *joiners, const int32_t *ok, int32_t count,
                               int32_t row0, int32_t rows, const int32_t *off, int32_t *fill,
                               int32_t *csr_src, int32_t *csr_slot, hipStream_t st);

}  // namespace gsp
