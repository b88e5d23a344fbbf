// gossip_protocol_amd/csrc/rowx_host.cpp -- the row-shard exchange, host side (rowx_host.hpp).
//
//   pack + gather    per local shard: pairs (sender, destination shard) and message records
//   counts           all-gather of every shard's 2G counts; the host reads them (the one sync
//                    per tick: RCCL needs element counts)
//   rows + records   one ncclGroupStart/End of ncclSend/ncclRecv per peer (one process per
//                    GPU), or device copies between the shards of an in-process group
//   csr              received records -> deg, scan, local + remote scatter
#include "rowx_host.hpp"

#include <algorithm>

#include "scale_kernels.hpp"

namespace gsp {

namespace {
constexpr size_t kPiece = size_t(1) << 27;      // 8-byte words per ncclSend / ncclRecv (1 GiB)
}

hipError_t RowxBufs::alloc(int32_t shards, int64_t pair_cap, int64_t msg_cap, int32_t row_words,
                           int64_t csr_cap, hipStream_t st) {
    const size_t G = size_t(shards), R = size_t(shards > 1 ? shards - 1 : 1);   // regions
    hipError_t e;
    const size_t S = size_t(rowx_cnt_stride(shards));
    if ((e = cnt.alloc(S)) != hipSuccess) return e;
    if ((e = cnt_all.alloc(S * G)) != hipSuccess) return e;
    if ((e = recv_msgs.alloc(G)) != hipSuccess) return e;
    if ((e = pair_row.alloc(R * size_t(pair_cap))) != hipSuccess) return e;
    if ((e = csr_slot.alloc(size_t(csr_cap))) != hipSuccess) return e;
    if ((e = send_rows.alloc(R * size_t(pair_cap) * size_t(row_words))) != hipSuccess) return e;
    if ((e = recv_rows.alloc(R * size_t(pair_cap) * size_t(row_words))) != hipSuccess) return e;
    if ((e = send_rec.alloc(R * size_t(msg_cap))) != hipSuccess) return e;
    if ((e = recv_rec.alloc(R * size_t(msg_cap))) != hipSuccess) return e;
    return hipMemsetAsync(recv_msgs.p, 0, G * 4, st);
}

void RowxBufs::release() {
    for (auto *b : {&cnt, &cnt_all, &recv_msgs, &pair_row, &csr_slot}) b->release();
    send_rows.release();
    recv_rows.release();
    send_rec.release();
    recv_rec.release();
}

int rowx_exchange(const RowxJob &job, std::vector<RowxShard> &local, double *bytes) {
    const int32_t G = job.shards, W = job.row_words, F = job.fanout, S = rowx_cnt_stride(G);
    hipStream_t st = job.st;
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
    // counts of every shard -> cnt_all[G][2G + 1] of the first local shard, read by the host
    RowxBufs &x0 = *local[0].x;
    if (job.comm) {
        GSP_NCCL(ncclAllGather(x0.cnt.p, x0.cnt_all.p, size_t(S), ncclInt32, job.comm, st));
    } else {
        for (RowxShard &src : local)
            GSP_HIP(hipMemcpyAsync(x0.cnt_all.p + size_t(src.g) * S, src.x->cnt.p, size_t(S) * 4,
                                   hipMemcpyDeviceToDevice, st));
    }
    GSP_HIP(hipMemcpyAsync(job.h_cnt, x0.cnt_all.p, size_t(S) * G * 4, hipMemcpyDeviceToHost, st));
    GSP_HIP(hipStreamSynchronize(st));
    auto pairs = [&](int32_t g, int32_t h) { return int64_t(job.h_cnt[size_t(g) * S + h]); };
    auto msgs = [&](int32_t g, int32_t h) { return int64_t(job.h_cnt[size_t(g) * S + G + h]); };
    for (int32_t g = 0; g < G; ++g)       // the same all-gathered flags on every rank
        GSP_REQUIRE(job.h_cnt[size_t(g) * S + 2 * G] == 0, GSP_ERR_CAPACITY,
                    "a receiver of shard %d got more messages than the kernel's segment bound at "
                    "tick %d; ticks after it did not run", g, job.h_cnt[size_t(g) * S + 2 * G]);
    for (int32_t g = 0; g < G; ++g)
        for (int32_t h = 0; h < G; ++h)
            GSP_REQUIRE(pairs(g, h) <= job.pair_cap && msgs(g, h) <= job.msg_cap, GSP_ERR_CAPACITY,
                        "row exchange: shard %d sends %lld rows / %lld records to shard %d "
                        "(capacity %lld / %lld)", g, (long long)pairs(g, h), (long long)msgs(g, h),
                        h, (long long)job.pair_cap, (long long)job.msg_cap);
    const size_t row_bytes = size_t(W) * 8, rec_bytes = sizeof(RowxRec);
    double sent = 0;
    if (job.comm) {
        RowxShard &sh = local[0];
        const int32_t me = sh.g;
        GSP_NCCL(ncclGroupStart());
        for (int32_t h = 0; h < G; ++h) {
            if (h == me) continue;
            const size_t reg = size_t(rowx_region(h, me));      // same index for h's region here
            const size_t so = reg * size_t(job.pair_cap), mo = reg * size_t(job.msg_cap);
            // full-view rows are 512 KB at 262,144 nodes: a region can pass 2^31 elements, so
            // rows move in pieces of at most kPiece words (matched in order on both sides)
            const size_t ns = size_t(pairs(me, h)) * W, nr = size_t(pairs(h, me)) * W;
            for (size_t o = 0; o < ns; o += kPiece)
                GSP_NCCL(ncclSend(sh.x->send_rows.p + so * W + o, std::min(kPiece, ns - o), ncclUint64,
                                  h, job.comm, st));
            if (msgs(me, h))
                GSP_NCCL(ncclSend(sh.x->send_rec.p + mo, size_t(msgs(me, h)) * 3, ncclInt32, h,
                                  job.comm, st));
            for (size_t o = 0; o < nr; o += kPiece)
                GSP_NCCL(ncclRecv(sh.x->recv_rows.p + so * W + o, std::min(kPiece, nr - o), ncclUint64,
                                  h, job.comm, st));
            if (msgs(h, me))
                GSP_NCCL(ncclRecv(sh.x->recv_rec.p + mo, size_t(msgs(h, me)) * 3, ncclInt32, h,
                                  job.comm, st));
            sent += double(pairs(me, h)) * row_bytes + double(msgs(me, h)) * rec_bytes;
        }
        GSP_NCCL(ncclGroupEnd());
    } else {
        for (RowxShard &src : local)
            for (RowxShard &dst : local) {
                const int32_t g = src.g, h = dst.g;
                if (g == h) continue;
                // src's region for h (send side), dst's region for g (receive side)
                const size_t sr = size_t(rowx_region(h, g)), rr = size_t(rowx_region(g, h));
                const size_t so = sr * size_t(job.pair_cap), mo = sr * size_t(job.msg_cap);
                const size_t ro = rr * size_t(job.pair_cap), qo = rr * size_t(job.msg_cap);
                if (pairs(g, h))
                    GSP_HIP(hipMemcpyAsync(dst.x->recv_rows.p + ro * W, src.x->send_rows.p + so * W,
                                           size_t(pairs(g, h)) * row_bytes, hipMemcpyDeviceToDevice, st));
                if (msgs(g, h))
                    GSP_HIP(hipMemcpyAsync(dst.x->recv_rec.p + qo, src.x->send_rec.p + mo,
                                           size_t(msgs(g, h)) * rec_bytes, hipMemcpyDeviceToDevice, st));
                sent += double(pairs(g, h)) * row_bytes + double(msgs(g, h)) * rec_bytes;
            }
    }
    *bytes += sent;
    for (size_t i = 0; i < local.size(); ++i) {
        RowxShard &sh = local[i];
        int32_t *hr = job.h_recv + i * size_t(G);
        for (int32_t h = 0; h < G; ++h) hr[h] = h == sh.g ? 0 : int32_t(msgs(h, sh.g));
        GSP_HIP(hipMemcpyAsync(sh.x->recv_msgs.p, hr, size_t(G) * 4, hipMemcpyHostToDevice, st));
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
