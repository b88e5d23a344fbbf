// gossip_protocol_amd/csrc/common.hpp -- error plumbing shared by the C-ABI implementation.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <string>

#include "gossip/gossip.h"

namespace gsp {

void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
const char *get_error();

// Returns from the enclosing C-ABI function with GSP_ERR_HIP on failure.
#define GSP_HIP(call)                                                                   \
    do {                                                                                \
        hipError_t gsp_e_ = (call);                                                     \
        if (gsp_e_ != hipSuccess) {                                                     \
            ::gsp::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #call,         \
                             hipGetErrorString(gsp_e_));                                \
            return GSP_ERR_HIP;                                                         \
        }                                                                               \
    } while (0)

#define GSP_REQUIRE(cond, status, ...)                                                  \
    do {                                                                                \
        if (!(cond)) {                                                                  \
            ::gsp::set_error(__VA_ARGS__);                                              \
            return (status);                                                            \
        }                                                                               \
    } while (0)

// Returns from the enclosing C-ABI function with GSP_ERR_RCCL on failure (needs <rccl/rccl.h>).
#define GSP_NCCL(call)                                                                  \
    do {                                                                                \
        ncclResult_t gsp_r_ = (call);                                                   \
        if (gsp_r_ != ncclSuccess) {                                                    \
            ::gsp::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #call,         \
                             ncclGetErrorString(gsp_r_));                               \
            return GSP_ERR_RCCL;                                                        \
        }                                                                               \
    } while (0)

// Device buffer owned by an engine.
template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void **>(&p), (count ? count : 1) * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    // physically contiguous device memory (hipDeviceMallocContiguous): the page-table fragments
    // may then span the whole allocation; falls back to hipMalloc when the driver refuses
    hipError_t alloc_contiguous(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void **>(&p), (count ? count : 1) * sizeof(T),
                                             hipDeviceMallocContiguous);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            return alloc(count);
        }
        n = count;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace gsp
