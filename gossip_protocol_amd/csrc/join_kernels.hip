// gossip_protocol_amd/csrc/join_kernels.hip -- JOINREP send and CSR scatter (join_kernels.hpp).
#include "join_kernels.hpp"
#include "philox.hpp"
#include "wave_ops.hpp"

namespace gsp {
namespace {

__global__ void __launch_bounds__(256) join_send_kernel(JoinSendArgs a) {
    const int32_t i = int32_t(blockIdx.x) * 256 + int32_t(threadIdx.x);
    uint32_t sent = 0, dropped = 0;
    if (i < a.count) {
        const int32_t j = a.joiners[i];
        int32_t ok = 0;
        if (j >= a.lo && j < a.hi && a.tick <= a.fail_tick[0]) {   // node 0 alive at tick
            sent = 1;
            const uint32_t dr = draw_u31(kDomainSend, a.seed, uint32_t(a.tick), 0u, uint32_t(j), 1u);
            if (int32_t(dr % 100u) < a.drop_pct) dropped = 1;
            else { ok = 1; atomicAdd(&a.deg[j], 1); }
        }
        a.ok[i] = ok;
    }
    sent = wave_sum32(sent);
    dropped = wave_sum32(dropped);
    if ((threadIdx.x & 63) == 0 && a.sent) {
        if (sent) atomicAdd(a.sent, (unsigned long long)sent);
        if (dropped) atomicAdd(a.dropped, (unsigned long long)dropped);
    }
}

__global__ void join_scatter_kernel(const int32_t *joiners, const int32_t *ok, int32_t count,
                                    int32_t row0, int32_t rows, const int32_t *off, int32_t *fill,
                                    int32_t *csr_src, int32_t *csr_slot) {
    const int32_t i = int32_t(blockIdx.x) * blockDim.x + int32_t(threadIdx.x);
    if (i >= count || !ok[i]) return;
    const int32_t lr = joiners[i] - row0;
    if (lr < 0 || lr >= rows) return;
    const int32_t p = off[lr] + atomicAdd(&fill[lr], 1);
    csr_src[p] = kJoinRepSrc;
    if (csr_slot) csr_slot[p] = 0;
}

}  // namespace

hipError_t launch_join_send(const JoinSendArgs &a, hipStream_t st) {
    if (a.count <= 0) return hipSuccess;
    hipLaunchKernelGGL(join_send_kernel, dim3(unsigned((a.count + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_join_scatter(const int32_t *joiners, const int32_t *ok, int32_t count,
                               int32_t row0, int32_t rows, const int32_t *off, int32_t *fill,
                               int32_t *csr_src, int32_t *csr_slot, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(join_scatter_kernel, dim3(unsigned((count + 255) / 256)), dim3(256), 0, st,
                       joiners, ok, count, row0, rows, off, fill, csr_src, csr_slot);
    return hipGetLastError();
}

}  // namespace gsp
