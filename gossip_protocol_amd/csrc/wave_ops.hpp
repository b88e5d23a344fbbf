// gossip_protocol_amd/csrc/wave_ops.hpp -- wave64 cross-lane primitives on the gfx950 DPP
// network.  A __shfl_up / __shfl_xor step lowers to a ds_bpermute round trip through the LDS
// crossbar plus index and select VALU work; a DPP step is one v_add_u32_dpp.  Callers run them
// with the whole wave active.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gsp {

// x of the lane the DPP control names, 0 where the shift or the row mask leaves a lane out
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint32_t dpp_take(uint32_t x) {
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), kCtrl, kRowMask, 0xF, false));
}

// Inclusive scan: four row_shr steps scan each 16-lane row, then row_bcast:15 (into rows 1, 3)
// and row_bcast:31 (into rows 2, 3) carry the row totals -- six v_add_u32_dpp.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += dpp_take<0x111>(x);            // row_shr:1
    x += dpp_take<0x112>(x);            // row_shr:2
    x += dpp_take<0x114>(x);            // row_shr:4
    x += dpp_take<0x118>(x);            // row_shr:8
    x += dpp_take<0x142, 0xA>(x);       // row_bcast:15
    x += dpp_take<0x143, 0xC>(x);       // row_bcast:31
    return x;
}

// value of lane l (wave-uniform l, e.g. from a ballot): one v_readlane
__device__ __forceinline__ uint32_t lane_of(uint32_t x, int32_t l) {
    return uint32_t(__builtin_amdgcn_readlane(int(x), l));
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) { return lane_of(wave_incl_scan(v), 63); }

// 64-bit wave sum (mod 2^64) from three 32-bit scans: the low word in two 16-bit halves (each
// sum < 2^22, no carry lost) and the high word mod 2^32
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
    const uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
    const uint64_t a = wave_sum32(lo & 0xFFFFu), b = wave_sum32(lo >> 16), c = wave_sum32(hi);
    return a + (b << 16) + (c << 32);
}

}  // namespace gsp
