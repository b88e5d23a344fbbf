// gossip_protocol_amd/csrc/exact_kernels.hip -- EXACT-mode HIP kernels for gfx950.
//
// exact_batch_kernel: one workgroup per node of a phase-P batch, one lane per member-table
// column.  It runs, for its node, what the reference runs per call:
//   GSP_OP_START  MP1Node::nodeStart/initThisNode/introduceSelfToGroup (MP1Node.cpp:67-154)
//   GSP_OP_LOOP   MP1Node::nodeLoop (MP1Node.cpp:176-193) = checkMessages + nodeLoopOps
//   GSP_OP_CHECK  MP1Node::checkMessages -> recvCallBack per queued message (:200-260)
//   GSP_OP_OPS    MP1Node::nodeLoopOps (:335-362)
// The merge is lane-parallel: every rule of recvCallBack touches only the entry whose id
// it looks up (check_exist, MP1Node.cpp:308-326), so column x evolves independently given
// the ordered queue; list order is restored from insertion keys by an LDS bitonic sort.
#include "exact_kernels.hpp"
#include "philox.hpp"

namespace gsp {

namespace {

constexpr int kMaxBlock = 1024;
constexpr int64_t kAbsentKey = INT64_MAX;

__device__ inline int64_t make_key(int64_t batch_seq, int32_t j, int32_t p1) {
    return (batch_seq << 40) | (int64_t(j) << 20) | int64_t(p1);
}

__device__ inline void push_event(const ExactBatchDev &b, int32_t pos, int32_t kind,
                                  int32_t subject, int64_t ord) {
    const int32_t slot = atomicAdd(b.ev_count, 1);
    if (slot < b.ev_cap) {
        ExactEvent ev;
        ev.pos = pos; ev.kind = kind; ev.subject = subject; ev.pad = 0; ev.ord = ord;
        b.events[slot] = ev;
    }
}

// Where a queued message's payload list lives: the sender's committed row, or a row of the
// payload arrays (a list the driver handed in, or the sender's list kept from send time).
struct Payload {
    const int64_t *key;
    const int32_t *hb, *ts, *rank;
    size_t row;
    int32_t nlist;
};
__device__ inline Payload payload_of(const ExactTable &tab, const ExactBatchDev &b, int32_t q,
                                     int32_t sc, int32_t n) {
    const int32_t pr = b.q_prow ? b.q_prow[q] : -1;
    if (pr >= 0) return Payload{b.p_key, b.p_hb, b.p_ts, b.p_rank, size_t(pr) * n, b.p_nlist[pr]};
    return Payload{tab.key, tab.hb, tab.ts, tab.rank, size_t(sc) * n, tab.nlist[sc]};
}

__global__ void __launch_bounds__(kMaxBlock)
exact_batch_kernel(ExactTable tab, ExactBatchDev b, int32_t n, int32_t tick, int64_t batch_seq,
                   int32_t tremove, int32_t id_filter_limit) {
    __shared__ int64_t s_key[kMaxBlock];
    __shared__ int32_t s_idx[kMaxBlock];
    __shared__ int32_t s_flag[4];  // in_group, do_ops, n_replies, nlist

    const int32_t pos = blockIdx.x;
    const int32_t r = b.node[pos];
    const int32_t op = b.op[pos];
    const int32_t x = threadIdx.x;
    const bool valid = x < n;
    const int32_t id = r + 1;
    const size_t row = size_t(r) * n;

    int64_t key = -1;
    int32_t hb = 0, ts = 0;
    if (valid) {
        key = tab.key[row + x];
        hb = tab.hb[row + x];
        ts = tab.ts[row + x];
    }
    bool present = key >= 0;
    int32_t inited = tab.inited[r], in_group = tab.in_group[r], own_hb = tab.own_hb[r];
    bool do_ops = false;
    int32_t n_replies = 0;
    const int32_t sbase = b.send_off[pos];

    if (op == 0) {  // START
        present = false;
        inited = 1;
        in_group = (id == 1);   // the introducer is id 1 (MP1Node.cpp:378-386)
        own_hb = 0;
        if (x == 0) {
            push_event(b, pos, id == 1 ? kEvStartGroup : kEvStartJoin, r, 0);
            if (id != 1) {      // JOINREQ to the introducer (MP1Node.cpp:133-150)
                b.send_dst[sbase] = 1;
                b.send_type[sbase] = 0;
                n_replies = 1;
            }
        }
    } else if (op == 1 || op == 2) {  // LOOP / CHECK: drain the queue in FIFO order
        const int32_t q0 = b.q_off[pos], q1 = b.q_off[pos + 1];
        unsigned long long merges = 0;
        for (int32_t q = q0; q < q1; ++q) {
            const int32_t j = q - q0;
            const int32_t sid = b.q_src[q];
            const int32_t type = b.q_type[q];
            const int32_t sc = sid - 1;
            if (type == 0 || type == 1) {          // JOINREQ / JOINREP: addMember(hdr)
                if (x == sc && !present) {
                    present = true; hb = 1; ts = tick;
                    key = make_key(batch_seq, j, 0);
                    push_event(b, pos, kEvJoin, x, (int64_t(j) << 20));
                }
                if (type == 0) {                   // reply JOINREP in queue order
                    if (b.rep_key && valid) {
                        const size_t o = size_t(b.rep_off[pos] + n_replies) * n + x;
                        b.rep_key[o] = present ? key : -1;
                        b.rep_hb[o] = hb;
                        b.rep_ts[o] = ts;
                    }
                    if (x == 0) {
                        b.send_dst[sbase + n_replies] = sid;
                        b.send_type[sbase + n_replies] = 1;
                    }
                    n_replies++;
                } else {
                    in_group = 1;
                    if (b.intro_list > 0 && valid && x != sc) {   // opt-in bounded introducer list
                        const Payload pl = payload_of(tab, b, q, sc, n);
                        const size_t srow = pl.row;
                        const int32_t cnt = pl.nlist;
                        const int32_t B = b.intro_list < cnt ? b.intro_list : cnt;
                        int32_t ranks[16];
                        int32_t nch = 0;
                        for (int32_t i = 0; i < B; ++i)
                            next_distinct_rank(draw_u31(kDomainJoin, b.seed, uint32_t(tick - 1), 0u,
                                                        uint32_t(r), uint32_t(i)), cnt, i, ranks, nch);
                        const int64_t kv = pl.key[srow + x];
                        bool chosen = false;
                        if (kv >= 0)
                            for (int32_t i = 0; i < nch; ++i) chosen = chosen || ranks[i] == pl.rank[srow + x];
                        // the GOSSIP payload rules (MP1Node.cpp:244-258), filter included
                        if (chosen && x + 1 < id_filter_limit) {
                            const int32_t hv = pl.hb[srow + x];
                            const int32_t tv = pl.ts[srow + x];
                            if (present) {
                                if (hv > hb) { hb = hv; ts = tick; }
                            } else if (x != r && tick - tv < tremove) {
                                const int32_t p1 = pl.rank[srow + x] + 1;
                                present = true; hb = hv; ts = tv;
                                key = make_key(batch_seq, j, p1);
                                push_event(b, pos, kEvJoin, x, (int64_t(j) << 20) | p1);
                            }
                        }
                    }
                }
            } else if (type == 3) {                // GOSSIP
                const Payload pl = payload_of(tab, b, q, sc, n);
                merges += 1ull + uint64_t(pl.nlist);
                if (x == sc) {
                    if (present) { hb += 1; ts = tick; }
                    else {
                        present = true; hb = 1; ts = tick;
                        key = make_key(batch_seq, j, 0);
                        push_event(b, pos, kEvJoin, x, (int64_t(j) << 20));
                    }
                    // the sender's own entry in its payload (never in a committed row: a list
                    // does not hold its owner; a driver-built list may), MP1Node.cpp:246-251
                    if (valid && pl.key[pl.row + x] >= 0 && x + 1 < id_filter_limit &&
                        pl.hb[pl.row + x] > hb) {
                        hb = pl.hb[pl.row + x];
                        ts = tick;
                    }
                } else if (valid) {
                    const size_t srow = pl.row;
                    const int64_t kv = pl.key[srow + x];
                    // payload filter 0 <= id < 10 (MP1Node.cpp:245); id = x + 1
                    if (kv >= 0 && x + 1 >= 0 && x + 1 < id_filter_limit) {
                        const int32_t hv = pl.hb[srow + x];
                        const int32_t tv = pl.ts[srow + x];
                        if (present) {
                            if (hv > hb) { hb = hv; ts = tick; }
                        } else if (x != r && tick - tv < tremove) {
                            const int32_t p1 = pl.rank[srow + x] + 1;
                            present = true; hb = hv; ts = tv;
                            key = make_key(batch_seq, j, p1);
                            push_event(b, pos, kEvJoin, x, (int64_t(j) << 20) | p1);
                        }
                    }
                }
            }
        }
        if (x == 0 && merges) atomicAdd(b.merges, merges);
        do_ops = (op == 1) && in_group;
    } else if (op == 3) {
        do_ops = true;
    }

    if (do_ops) {               // nodeLoopOps: hb bump + TREMOVE scan (MP1Node.cpp:337-348)
        own_hb += 1;
        if (present && tick - ts >= tremove) {
            push_event(b, pos, kEvRemove, x, -key);  // log order: descending list index
            present = false;
        }
    }
    if (!present) { key = -1; hb = 0; ts = 0; }

    // list order = ascending insertion key: bitonic sort (key, column) in LDS
    const int32_t P = blockDim.x;
    s_key[x] = present ? key : kAbsentKey;
    s_idx[x] = x;
    __syncthreads();
    for (int32_t k = 2; k <= P; k <<= 1) {
        for (int32_t jj = k >> 1; jj > 0; jj >>= 1) {
            const int32_t o = x ^ jj;
            if (o > x) {
                const bool asc = (x & k) == 0;
                const int64_t a = s_key[x], c = s_key[o];
                if ((a > c) == asc) {
                    s_key[x] = c; s_key[o] = a;
                    const int32_t t = s_idx[x]; s_idx[x] = s_idx[o]; s_idx[o] = t;
                }
            }
            __syncthreads();
        }
    }
    // rank of each column, member count
    if (s_key[x] != kAbsentKey) b.o_rank[size_t(pos) * n + s_idx[x]] = x;
    const bool last_present = s_key[x] != kAbsentKey && (x + 1 == P || s_key[x + 1] == kAbsentKey);
    if (x == 0) s_flag[3] = 0;
    __syncthreads();
    if (last_present) s_flag[3] = x + 1;
    __syncthreads();
    const int32_t nlist = s_flag[3];

    if (valid) {
        const size_t o = size_t(pos) * n + x;
        b.o_key[o] = key;
        b.o_hb[o] = hb;
        b.o_ts[o] = ts;
        if (!present) b.o_rank[o] = -1;
    }
    // gossip to every member in list order after the removals (MP1Node.cpp:350-361)
    if (do_ops && x < nlist) {
        b.send_dst[sbase + n_replies + x] = s_idx[x] + 1;
        b.send_type[sbase + n_replies + x] = 3;
    }
    if (x == 0) {
        b.o_state[pos * 4 + 0] = inited;
        b.o_state[pos * 4 + 1] = in_group;
        b.o_state[pos * 4 + 2] = own_hb;
        b.o_state[pos * 4 + 3] = nlist;
        b.send_cnt[pos] = n_replies + (do_ops ? nlist : 0);
    }
}

__global__ void exact_commit_kernel(ExactTable tab, ExactBatchDev b, int32_t n) {
    const int32_t pos = blockIdx.x;
    const int32_t r = b.node[pos];
    const size_t o = size_t(pos) * n, row = size_t(r) * n;
    for (int32_t x = threadIdx.x; x < n; x += blockDim.x) {
        tab.key[row + x] = b.o_key[o + x];
        tab.hb[row + x] = b.o_hb[o + x];
        tab.ts[row + x] = b.o_ts[o + x];
        tab.rank[row + x] = b.o_rank[o + x];
    }
    if (threadIdx.x == 0) {
        tab.inited[r] = b.o_state[pos * 4 + 0];
        tab.in_group[r] = b.o_state[pos * 4 + 1];
        tab.own_hb[r] = b.o_state[pos * 4 + 2];
        tab.nlist[r] = b.o_state[pos * 4 + 3];
    }
}

// inclusive block scan of one int per thread (blockDim.x == 1024, 16 waves of 64)
__device__ inline int32_t block_inclusive_scan(int32_t v, int32_t *s_wave) {
    const int32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int32_t d = 1; d < 64; d <<= 1) {
        const int32_t u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    if (lane == 63) s_wave[wave] = v;
    __syncthreads();
    if (wave == 0) {
        int32_t w = lane < int32_t(blockDim.x >> 6) ? s_wave[lane] : 0;
#pragma unroll
        for (int32_t d = 1; d < 64; d <<= 1) {
            const int32_t u = __shfl_up(w, d, 64);
            if (lane >= d) w += u;
        }
        if (lane < int32_t(blockDim.x >> 6)) s_wave[lane] = w;
    }
    __syncthreads();
    const int32_t add = wave ? s_wave[wave - 1] : 0;
    __syncthreads();
    return v + add;
}

__global__ void __launch_bounds__(kMaxBlock) exact_send_kernel(ExactSendDev s) {
    __shared__ int32_t s_base[kMaxBlock + 1];
    __shared__ int32_t s_wave[16];
    __shared__ int32_t s_carry;
    const int32_t tid = threadIdx.x;

    // 1. exclusive scan of per-node send counts, in batch (call) order
    const int32_t c = tid < s.n_batch ? s.send_cnt[tid] : 0;
    const int32_t inc = block_inclusive_scan(c, s_wave);
    s_base[tid + 1] = inc;
    if (tid == 0) { s_base[0] = 0; s_carry = 0; }
    __syncthreads();
    const int32_t total = s_base[s.n_batch];

    // 2. per send: draw, drop, admission (first buff_room survivors), compaction
    for (int32_t c0 = 0; c0 < total; c0 += blockDim.x) {
        const int32_t i = c0 + tid;
        int32_t src = 0, dst = 0, type = 0, keep = 0, slot = 0;
        if (i < total) {
            int32_t lo = 0, hi = s.n_batch - 1;   // batch node owning send i
            while (lo < hi) {
                const int32_t mid = (lo + hi + 1) >> 1;
                if (s_base[mid] <= i) lo = mid; else hi = mid - 1;
            }
            const int32_t k = i - s_base[lo];
            src = s.node[lo] + 1;
            slot = s.send_off[lo] + k;
            dst = s.send_dst[slot];
            type = s.send_type[slot];
            const int64_t g = s.g0 + i;
            int32_t draw;
            if (s.rng_mode == 1)
                draw = int32_t(draw_u31(kDomainSend, s.seed, uint32_t(s.tick), uint32_t(src),
                                              uint32_t(dst), uint32_t(type)));
            else
                draw = s.glibc_stream[g - s.stream_base];
            const bool dropped = s.size_reject || (s.dropmsg && (draw % 100) < s.drop_thr);
            keep = dropped ? 0 : 1;
        }
        const int32_t incl = block_inclusive_scan(keep, s_wave);
        const int32_t before = s_carry + incl - keep;
        if (keep && before < s.buff_room) {
            s.adm_src[before] = src;
            s.adm_dst[before] = dst;
            s.adm_type[before] = type;
            if (s.adm_slot) s.adm_slot[before] = slot;
            atomicAdd(&s.sent_ctr[size_t(src) * s.max_ticks + s.tick], 1);
        }
        __syncthreads();
        if (tid == blockDim.x - 1) s_carry += incl;
        __syncthreads();
    }
    if (tid == 0) {
        *s.adm_count = s_carry < s.buff_room ? s_carry : s.buff_room;
        *s.draws = total;
    }
}

}  // namespace

hipError_t launch_exact_batch(const ExactTable &tab, const ExactBatchDev &b, int32_t n,
                              int32_t tick, int64_t batch_seq, int32_t tremove,
                              int32_t id_filter_limit, hipStream_t st) {
    int32_t P = 64;
    while (P < n) P <<= 1;
    if (P > kMaxBlock || b.n_batch <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(exact_batch_kernel, dim3(b.n_batch), dim3(P), 0, st, tab, b, n, tick,
                       batch_seq, tremove, id_filter_limit);
    return hipGetLastError();
}

hipError_t launch_exact_commit(const ExactTable &tab, const ExactBatchDev &b, int32_t n,
                               hipStream_t st) {
    if (b.n_batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(exact_commit_kernel, dim3(b.n_batch), dim3(256), 0, st, tab, b, n);
    return hipGetLastError();
}

hipError_t launch_exact_sends(const ExactSendDev &s, hipStream_t st) {
    if (s.n_batch <= 0 || s.n_batch > kMaxBlock) return hipErrorInvalidValue;
    hipLaunchKernelGGL(exact_send_kernel, dim3(1), dim3(kMaxBlock), 0, st, s);
    return hipGetLastError();
}

}  // namespace gsp
