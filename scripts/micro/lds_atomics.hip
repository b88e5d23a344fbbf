// Microbenchmark (diagnostic, not product): cycles per wave-instruction of LDS atomics on random
// slots, 4 workgroups of 256 lanes per CU (the drain hash classes' shape), vs. plain reads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int CAP = 4096, ITERS = 256;
template <int MODE>
__global__ void __launch_bounds__(256) k(unsigned long long *out, uint32_t seed) {
    __shared__ uint64_t tab[CAP];
    for (int i = threadIdx.x; i < CAP; i += 256) tab[i] = ~0ull;
    __syncthreads();
    uint32_t x = seed ^ (threadIdx.x * 0x9E3779B1u) ^ (blockIdx.x * 0x85EBCA77u);
    uint64_t acc = 0;
    const uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; ++it) {
        x = x * 1664525u + 1013904223u;
        const int h = int((uint64_t(x) * CAP) >> 32);
        if (MODE == 0) acc += tab[h];                                                       // ds_read_b64
        if (MODE == 1) acc += atomicCAS((unsigned long long *)&tab[h], ~0ull, (unsigned long long)x);  // cmpst b64 rtn
        if (MODE == 2) acc += atomicCAS((unsigned int *)&tab[h], 0xFFFFFFFFu, x);           // cmpst b32 rtn
        if (MODE == 3) atomicMax((unsigned int *)&tab[h], x);                              // ds_max_u32 (no rtn)
        if (MODE == 4) { const ulonglong2 a = *(const ulonglong2 *)&tab[h & ~1]; acc += a.x + a.y; }  // ds_read_b128
    }
    const uint64_t t1 = clock64();
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)(t1 - t0));
    if (acc == 12345) out[1] = acc;
}
int main() {
    unsigned long long *d;
    hipMalloc(&d, 16);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char *names[] = {"ds_read_b64", "ds_cmpst_rtn_b64", "ds_cmpst_rtn_b32", "ds_max_u32", "ds_read_b128"};
    for (int mode = 0; mode < 5; ++mode) {
        for (int per : {1, 4}) {
            hipMemset(d, 0, 16);
            const int blocks = cus * per;
            switch (mode) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, 7u); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, 7u); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, d, 7u); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, d, 7u); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, d, 7u); break;
            }
            unsigned long long h[2];
            hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
            const double waves = blocks * 4.0;
            printf("%-18s %d wg/CU: %.1f cycles per wave-instruction (wave view), %.2f CU-cycles per wave-instr\n",
                   names[mode], per, double(h[0]) / waves / ITERS, double(h[0]) / waves / ITERS / (per * 4));
        }
    }
    return 0;
}
