// LDS instruction cost on gfx950 for the access patterns of the K3 bucket kernel
// (DESIGN.md section 4): 1024-thread workgroups, one per CU, 16 independent
// operations per lane per iteration.  Prints cycles per wave-instruction per CU
// (2.4 GHz) for
//   read_seq   ds_read_b32, lane-consecutive words (conflict-free baseline)
//   read_rnd   ds_read_b32, random words of a T-word table (phase-1 offset table: T = 128)
//   bperm_rnd  ds_bpermute_b32 from random source lanes (a register-resident table)
//   add_rnd    ds_add_u32 (no return), random words of 32,768 (phase-2 histogram)
//   addr_rnd   ds_add_rtn_u32, random words of T (phase-1 rank counters)
//   w16_rnd    ds_write_b16, random halves of 16,384 words (phase-1 staging)
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_ops tools/lds_ops_rate.hip && /tmp/lds_ops
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;

template <int OP>
__global__ void __launch_bounds__(1024) k_ops(uint32_t* out, int iters, uint32_t tmask) {
    extern __shared__ uint32_t h[];
    for (uint32_t i = threadIdx.x; i < 32768; i += 1024) h[i] = i;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t s = threadIdx.x * 2654435761u + blockIdx.x * 40503u + 1u, acc = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t a[16], r[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            s = s * 1664525u + 1013904223u;
            a[j] = (s >> 9) & tmask;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if constexpr (OP == 0) r[j] = *(volatile lds_u32*)(uintptr_t)(4 * ((lane + 64 * j + it) & 32767));
            if constexpr (OP == 1) r[j] = *(volatile lds_u32*)(uintptr_t)(4 * a[j]);
            if constexpr (OP == 2) r[j] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * (a[j] & 63)), (int)(s + j));
            if constexpr (OP == 3) {
                __hip_atomic_fetch_add((lds_u32*)(uintptr_t)(4 * a[j]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                r[j] = 0;
            }
            if constexpr (OP == 4)
                r[j] = __hip_atomic_fetch_add((lds_u32*)(uintptr_t)(4 * a[j]), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
            if constexpr (OP == 5) {
                *(volatile lds_u16*)(uintptr_t)(2 * a[j]) = (uint16_t)s;
                r[j] = 0;
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += r[j];
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = h[5] + acc;
    else if (acc == 0xFFFFFFFFu) out[1] = acc;
}

template <int OP>
float run(uint32_t* d, int iters, uint32_t tmask) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_ops<OP>, dim3(256), dim3(1024), 131072, 0, d, 10, tmask);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_ops<OP>, dim3(256), dim3(1024), 131072, 0, d, iters, tmask);
    (void)hipEventRecord(b);
    if (hipEventSynchronize(b) != hipSuccess) return -1.f;
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t* d;
    (void)hipMalloc(&d, 1 << 20);
    const int iters = 2000;
    for (auto f : {k_ops<0>, k_ops<1>, k_ops<2>, k_ops<3>, k_ops<4>, k_ops<5>})
        (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    const double instr = 16.0 * iters * 16;   // wave-instructions per CU (16 waves x 16 per iteration)
    auto show = [&](const char* n, uint32_t t, float ms) {
        printf("%-10s T=%-6u %9.3f ms %8.2f cyc/wave-instr/CU\n", n, t, ms, ms * 1e6 / instr * 2.4);
    };
    show("read_seq", 32768, run<0>(d, iters, 32767));
    for (uint32_t t : {128u, 512u, 32768u}) show("read_rnd", t, run<1>(d, iters, t - 1));
    show("bperm_rnd", 64, run<2>(d, iters, 63));
    show("add_rnd", 32768, run<3>(d, iters, 32767));
    for (uint32_t t : {128u, 512u, 32768u}) show("addr_rnd", t, run<4>(d, iters, t - 1));
    show("w16_rnd", 32768, run<5>(d, iters, 32767));
    return 0;
}
