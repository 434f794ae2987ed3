// LDS atomic throughput for the k=7 pair-counting design (DESIGN.md "K1p"):
// one 1024-thread workgroup per CU, random addresses, comparing
//   plain     : 16 ds_add_u32 per lane per iteration into a 64 KiB table (today's K1, 1 WG/CU)
//   plain2    : the same with 2 WGs/CU (today's K1 shape)
//   rtn-u16   : 8 ds_add_rtn_u32 per lane into a 128 KiB table of u16 halves
//               (delta 1 or 1<<16), the returns OR-folded and tested once per iteration
//   plain-u16 : the same 8 adds without return (lower bound of the pair design)
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_pair tools/lds_pair_rate.hip && /tmp/lds_pair
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
typedef __attribute__((address_space(3))) uint32_t lds_u32;
template <int MODE>
__global__ void __launch_bounds__(1024) k_lds(uint32_t* out, int iters, uint32_t words) {
    extern __shared__ uint32_t h[];
    for (uint32_t i = threadIdx.x; i < words; i += 1024) h[i] = 0;
    __syncthreads();
    uint32_t s = mix(threadIdx.x * 2654435761u + blockIdx.x);
    uint32_t acc = 0;
    const uint32_t wm = words - 1;
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {
            uint32_t a[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) { s = s * 1664525u + 1013904223u; a[j] = ((s >> 8) & wm) << 2; }
#pragma unroll
            for (int j = 0; j < 16; ++j)
                __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            uint32_t a[8], dl[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                s = s * 1664525u + 1013904223u;
                a[j] = ((s >> 8) & wm) << 2;
                dl[j] = 1u << ((s >> 3) & 16u);
            }
            if (MODE == 1) {
                uint32_t o = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    o |= __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a[j], dl[j], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_WORKGROUP);
                if (__builtin_amdgcn_ballot_w64((o & 0x80008000u) != 0)) acc += 1;   // rare path stand-in
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a[j], dl[j], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = h[5] + acc;
}
int main() {
    uint32_t* d;
    (void)hipMalloc(&d, 1 << 20);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 2000;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    struct Case { const char* name; void (*fn)(uint32_t*, int, uint32_t); int per_cu; uint32_t words; int adds; };
    Case cs[] = {
        {"plain 16x, 64K table, 1 WG/CU", k_lds<0>, 1, 16384, 16},
        {"plain 16x, 64K table, 2 WG/CU", k_lds<0>, 2, 16384, 16},
        {"rtn 8x u16, 128K table, 1 WG/CU", k_lds<1>, 1, 32768, 8},
        {"plain 8x u16, 128K table, 1 WG/CU", k_lds<2>, 1, 32768, 8},
    };
    for (auto& c : cs) {
        const size_t lds = c.words * 4;
        (void)hipFuncSetAttribute((const void*)c.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        const int blocks = cus * c.per_cu;
        hipLaunchKernelGGL(c.fn, dim3(blocks), dim3(1024), lds, 0, d, 10, c.words);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(c.fn, dim3(blocks), dim3(1024), lds, 0, d, iters, c.words);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        if (hipGetLastError() != hipSuccess) { printf("%s: launch failed\n", c.name); continue; }
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        // per lane-iteration: 16 windows counted in every case (8 pairs = 16 windows)
        const double iters_per_cu = (double)blocks / cus * 16 * iters;   // wave-iterations per CU
        printf("%-36s %8.3f ms  %6.2f ns per wave-iteration (16 windows) per CU  = %6.1f cyc @2.3GHz, "
               "%.2f cyc per ds op\n", c.name, ms, ms * 1e6 / iters_per_cu, ms * 1e6 / iters_per_cu * 2.3,
               ms * 1e6 / iters_per_cu * 2.3 / c.adds);
    }
    // 160 KiB dynamic LDS: does one workgroup get it?
    (void)hipFuncSetAttribute((const void*)k_lds<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    hipLaunchKernelGGL(k_lds<2>, dim3(cus), dim3(1024), 163840, 0, d, 10, 32768);
    printf("160 KiB launch: %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
