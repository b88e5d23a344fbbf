// gossip_protocol_amd/csrc/rowx_host.cpp -- the row-shard exchange, host side (rowx_host.hpp).
//
//   pack + gather    per local shard: pairs (sender, destination shard) and message records;
//                    partial-view rows packed for the wire (rowx_kernels.hpp)
//   counts           all-gather of every shard's 2G counts + capacity flag (device), copied to
//                    pinned memory behind an event
//   check            the counts against the capacities and the sizes posted; in-band receive
//                    counts for every later kernel
//   rows + records   one ncclGroupStart/End of ncclSend/ncclRecv per peer, sized from earlier
//                    exchanges (one process per GPU), or device copies between the shards of an
//                    in-process group, sized by the device counts
//   unpack + csr     packed rows decoded; received records -> deg, scan, local + remote scatter
#include "rowx_host.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "scale_kernels.hpp"

namespace gsp {

namespace {
constexpr size_t kPiece = size_t(1) << 27;      // 8-byte words per ncclSend / ncclRecv (1 GiB)
}

hipError_t RowxBufs::alloc(int32_t shards, int64_t pair_cap, int64_t msg_cap, int32_t row_words,
                           bool packed, bool rccl, int64_t csr_cap, hipStream_t st) {
    const size_t G = size_t(shards), R = size_t(shards > 1 ? shards - 1 : 1);   // regions
    const size_t wire = size_t(packed ? rowx_packed_words(row_words) : row_words);
    hipError_t e;
    const size_t S = size_t(rowx_cnt_stride(shards));
    if ((e = cnt.alloc(S)) != hipSuccess) return e;
    if ((e = cnt_all.alloc(S * G)) != hipSuccess) return e;
    if ((e = recv_msgs.alloc(G)) != hipSuccess) return e;
    if ((e = recv_pairs.alloc(G)) != hipSuccess) return e;
    if ((e = bounds.alloc(size_t(RowxState::kRing) * 2 * G * G)) != hipSuccess) return e;
    if ((e = pair_row.alloc(R * size_t(pair_cap))) != hipSuccess) return e;
    if ((e = csr_slot.alloc(size_t(csr_cap))) != hipSuccess) return e;
    if ((e = send_rows.alloc(R * size_t(pair_cap) * wire)) != hipSuccess) return e;
    if ((e = recv_rows.alloc(R * size_t(pair_cap) * size_t(row_words))) != hipSuccess) return e;
    // RCCL receives into a wire-format region when rows are packed (raw rows land in place)
    if (rccl && packed && (e = recv_wire.alloc(R * size_t(pair_cap) * wire)) != hipSuccess) return e;
    if ((e = send_rec.alloc(R * size_t(msg_cap))) != hipSuccess) return e;
    if ((e = recv_rec.alloc(R * size_t(msg_cap))) != hipSuccess) return e;
    if ((e = hipMemsetAsync(recv_msgs.p, 0, G * 4, st)) != hipSuccess) return e;
    return hipMemsetAsync(recv_pairs.p, 0, G * 4, st);
}

void RowxBufs::release() {
    for (auto *b : {&cnt, &cnt_all, &recv_msgs, &recv_pairs, &pair_row, &csr_slot, &bounds}) b->release();
    send_rows.release();
    recv_rows.release();
    recv_wire.release();
    send_rec.release();
    recv_rec.release();
}

hipError_t RowxState::init(int32_t g, bool with_rccl) {
    shards = g;
    rccl = with_rccl;
    const size_t S = size_t(rowx_cnt_stride(g));
    hipError_t e;
    if ((e = hipHostMalloc(reinterpret_cast<void **>(&h_cnt), size_t(kRing) * S * g * 4)) != hipSuccess) return e;
    if ((e = hipHostMalloc(reinterpret_cast<void **>(&h_bounds), size_t(kRing) * 2 * g * g * 4)) != hipSuccess)
        return e;
    for (auto &v : ev)
        if ((e = hipEventCreateWithFlags(&v, hipEventDisableTiming)) != hipSuccess) return e;
    max_pairs.assign(size_t(g) * g, -1);
    max_msgs.assign(size_t(g) * g, -1);
    if (const char *tt = std::getenv("GSP_TEST_ROWX_TIGHT")) tight = std::atoi(tt) != 0;
    if (const char *tp = std::getenv("GSP_TEST_ROWX_POSTED")) posted = std::atoi(tp) != 0;
    return hipSuccess;
}

void RowxState::release() {
    if (h_cnt) (void)hipHostFree(h_cnt);
    if (h_bounds) (void)hipHostFree(h_bounds);
    for (auto &v : ev)
        if (v) (void)hipEventDestroy(v);
    h_cnt = h_bounds = nullptr;
    for (auto &v : ev) v = nullptr;
}

namespace {

// The host reads the counts of exchange k (its event has fired or is waited for here): the
// largest counts seen grow, and an in-process group's bytes are accounted from them.
int rowx_see(RowxState &s, int64_t k, double *bytes) {
    const int32_t G = s.shards, S = rowx_cnt_stride(G);
    GSP_HIP(hipEventSynchronize(s.ev[k % RowxState::kRing]));
    const int32_t *c = s.h_cnt + size_t(k % RowxState::kRing) * S * G;
    for (int32_t g = 0; g < G; ++g)
        for (int32_t h = 0; h < G; ++h) {
            if (g == h) continue;
            const int64_t p = c[size_t(g) * S + h], m = c[size_t(g) * S + G + h];
            int64_t &mp = s.max_pairs[size_t(g) * G + h], &mm = s.max_msgs[size_t(g) * G + h];
            mp = std::max(mp, p);
            mm = std::max(mm, m);
            if (!s.rccl) *bytes += double(p) * s.wire_bytes_per_row + double(m) * s.rec_bytes;
        }
    s.seen = k + 1;
    return GSP_OK;
}

}  // namespace

int rowx_collect(RowxState &s, double *bytes) {
    while (s.seen < s.seq)
        if (int rc = rowx_see(s, s.seen, bytes)) return rc;
    return GSP_OK;
}

int rowx_exchange(const RowxJob &job, std::vector<RowxShard> &local, double *bytes) {
    const int32_t G = job.shards, W = job.row_words, F = job.fanout, S = rowx_cnt_stride(G);
    const int32_t PW = job.packed ? rowx_packed_words(W) : W;      // words per row on the wire
    RowxState &st8 = *job.state;
    hipStream_t st = job.st;
    st8.wire_bytes_per_row = double(PW) * 8.0;
    for (RowxShard &sh : local) {
        GSP_HIP(hipMemsetAsync(sh.x->cnt.p, 0, size_t(2 * G) * 4, st));
        GSP_HIP(hipMemcpyAsync(sh.x->cnt.p + 2 * G, sh.err, 4, hipMemcpyDeviceToDevice, st));
        RowxArgs a{};
        a.n = job.n;
        a.shards = G;
        a.shard = sh.g;
        a.fanout = F;
        a.row0 = sh.row0;
        a.rows = sh.rows;
        a.pair_cap = job.pair_cap;
        a.msg_cap = job.msg_cap;
        a.row_words = W;
        a.packed = job.packed ? 1 : 0;
        a.out_dst = sh.out_dst;
        a.table = sh.table;
        a.pair_cnt = sh.x->cnt.p;
        a.msg_cnt = sh.x->cnt.p + G;
        a.pair_row = sh.x->pair_row.p;
        a.send_rows = sh.x->send_rows.p;
        a.send_rec = sh.x->send_rec.p;
        GSP_HIP(launch_rowx_pack(a, st));
        GSP_HIP(launch_rowx_gather(a, st));
    }
    // counts of every shard -> cnt_all[G][2G + 1] of the first local shard (every local shard
    // reads that one), then to pinned memory for the sizes of later exchanges
    RowxBufs &x0 = *local[0].x;
    if (job.comm) {
        GSP_NCCL(ncclAllGather(x0.cnt.p, x0.cnt_all.p, size_t(S), ncclInt32, job.comm, st));
    } else {
        for (RowxShard &src : local)
            GSP_HIP(hipMemcpyAsync(x0.cnt_all.p + size_t(src.g) * S, src.x->cnt.p, size_t(S) * 4,
                                   hipMemcpyDeviceToDevice, st));
    }
    const int64_t k = st8.seq++;
    const int slot = int(k % RowxState::kRing);
    GSP_HIP(hipMemcpyAsync(st8.h_cnt + size_t(slot) * S * G, x0.cnt_all.p, size_t(S) * G * 4,
                           hipMemcpyDeviceToHost, st));
    GSP_HIP(hipEventRecord(st8.ev[slot], st));
    // the host reads the previous exchange's counts (its only wait: one tick behind)
    if (k >= 1)
        while (st8.seen < k)
            if (int rc = rowx_see(st8, st8.seen, bytes)) return rc;
    const int32_t *d_bounds = nullptr;
    const size_t GG = size_t(G) * G;
    if (job.comm || st8.tight || st8.posted) {
        // sizes posted to RCCL, the same on every rank: derived from the all-gathered counts
        // of exchanges 0 .. k - 1 (the capacity for the first exchange), with margins for the
        // drop draws' spread (1/16 + 256 pairs / 1024 records) and for the growth the host knows
        // of: every new sender may add a pair and F records to every shard pair,
        // and a drop percentage that falls scales what gets through by (100 - now) / (100 - before)
        int32_t *hb = st8.h_bounds + size_t(slot) * 2 * GG;
        const bool tight = st8.tight;
        const int64_t mpa = tight ? 0 : 256 + job.new_senders, mma = tight ? 0 : 1024 + job.new_senders * F;
        const int64_t div = tight ? int64_t(1) << 40 : 16;
        const bool rise = !tight && job.drop_now < job.drop_before;   // more of the sends get through
        const int64_t num = 100 - job.drop_now, den = 100 - job.drop_before;
        auto grow = [&](int64_t c, int64_t cap) {
            if (rise) c = den > 0 ? (c * num + den - 1) / den : cap;
            return std::min<int64_t>(cap, c);
        };
        for (size_t i = 0; i < GG; ++i) {
            const int64_t mp = st8.max_pairs[i], mm = st8.max_msgs[i];
            hb[i] = int32_t(mp < 0 ? job.pair_cap : std::min<int64_t>(job.pair_cap, grow(mp, job.pair_cap) + mp / div + mpa));
            hb[GG + i] = int32_t(mm < 0 ? job.msg_cap : std::min<int64_t>(job.msg_cap, grow(mm, job.msg_cap) + mm / div + mma));
        }
        int32_t *db = x0.bounds.p + size_t(slot) * 2 * GG;
        GSP_HIP(hipMemcpyAsync(db, hb, 2 * GG * 4, hipMemcpyHostToDevice, st));
        d_bounds = db;
    }
    for (RowxShard &sh : local)
        GSP_HIP(launch_rowx_check(x0.cnt_all.p, d_bounds, G, sh.g, job.pair_cap, job.msg_cap, job.tick,
                                  sh.err, sh.x->recv_pairs.p, sh.x->recv_msgs.p, st));
    if (job.comm) {
        const int32_t *hb = st8.h_bounds + size_t(slot) * 2 * GG;
        RowxShard &sh = local[0];
        const int32_t me = sh.g;
        double sent = 0;
        GSP_NCCL(ncclGroupStart());
        for (int32_t h = 0; h < G; ++h) {
            if (h == me) continue;
            const size_t reg = size_t(rowx_region(h, me));      // same index for h's region here
            const size_t so = reg * size_t(job.pair_cap), mo = reg * size_t(job.msg_cap);
            const size_t bs_p = size_t(hb[size_t(me) * G + h]), bs_m = size_t(hb[GG + size_t(me) * G + h]);
            const size_t br_p = size_t(hb[size_t(h) * G + me]), br_m = size_t(hb[GG + size_t(h) * G + me]);
            uint64_t *rbase = job.packed ? sh.x->recv_wire.p : sh.x->recv_rows.p;
            // rows move in pieces of at most kPiece words (a full-view region can pass 2^31
            // elements), matched in order on both sides
            const size_t ns = bs_p * PW, nr = br_p * PW;
            for (size_t o = 0; o < ns; o += kPiece)
                GSP_NCCL(ncclSend(sh.x->send_rows.p + so * PW + o, std::min(kPiece, ns - o), ncclUint64,
                                  h, job.comm, st));
            if (bs_m)
                GSP_NCCL(ncclSend(sh.x->send_rec.p + mo, bs_m * 3, ncclInt32, h, job.comm, st));
            for (size_t o = 0; o < nr; o += kPiece)
                GSP_NCCL(ncclRecv(rbase + so * PW + o, std::min(kPiece, nr - o), ncclUint64, h, job.comm, st));
            if (br_m)
                GSP_NCCL(ncclRecv(sh.x->recv_rec.p + mo, br_m * 3, ncclInt32, h, job.comm, st));
            sent += double(bs_p) * double(PW) * 8.0 + double(bs_m) * 12.0;
        }
        GSP_NCCL(ncclGroupEnd());
        *bytes += sent;
        if (job.packed)
            GSP_HIP(launch_rowx_unpack(sh.x->recv_wire.p, sh.x->recv_rows.p, sh.x->recv_pairs.p, G, me,
                                       job.pair_cap, W, 1, st));
    } else {
        for (RowxShard &src : local)
            for (RowxShard &dst : local)
                if (src.g != dst.g)
                    GSP_HIP(launch_rowx_local_copy(src.x->send_rows.p, src.x->send_rec.p, dst.x->recv_rows.p,
                                                   dst.x->recv_rec.p, x0.cnt_all.p, G, src.g, dst.g,
                                                   job.pair_cap, job.msg_cap, W, job.packed ? 1 : 0, st));
    }
    for (RowxShard &sh : local) {
        GSP_HIP(launch_rowx_recv_deg(sh.x->recv_rec.p, sh.x->recv_msgs.p, G, sh.g, job.msg_cap,
                                     sh.row0, sh.deg, st));
        GSP_HIP(launch_exclusive_scan(sh.deg + sh.row0, sh.off, sh.rows, sh.tile_sum, st));
        GSP_HIP(hipMemsetAsync(sh.fill, 0, size_t(sh.rows) * 4, st));
        GSP_HIP(launch_rowx_scatter_local(sh.out_dst, sh.rows, F, sh.row0, sh.off, sh.fill, sh.csr_src,
                                          sh.x->csr_slot.p, st));
        GSP_HIP(launch_rowx_scatter_remote(sh.x->recv_rec.p, sh.x->recv_msgs.p, G, sh.g,
                                           job.msg_cap, job.pair_cap, sh.off, sh.fill, sh.csr_src,
                                           sh.x->csr_slot.p, st));
        GSP_HIP(hipMemsetAsync(sh.deg, 0, size_t(job.n) * 4, st));
    }
    return GSP_OK;
}

}  // namespace gsp
