// LDS ds_add_rtn_u32 rank throughput (the K3 phase-1 rank step):
// 1024-thread workgroups, one per CU, 16 returning adds per lane per iteration into
// NBK bucket counters, each counter split into R lane replicas (word b*R + lane%R),
// optionally private per wave.  Prints wave-instruction cost per CU.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_rank tools/lds_rank_rate.hip && /tmp/lds_rank
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t mix(uint32_t x){x^=x>>16;x*=0x7feb352dU;x^=x>>15;x*=0x846ca68bU;x^=x>>16;return x;}

__global__ void __launch_bounds__(1024) k_rank(uint32_t* out, int iters, uint32_t nbk, uint32_t rlog, uint32_t per_wave,
                                               uint32_t words) {
  extern __shared__ uint32_t h[];
  for (uint32_t i = threadIdx.x; i < words; i += 1024) h[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t base = per_wave ? wave * (nbk << rlog) : 0u;
  const uint32_t rep = lane & ((1u << rlog) - 1u);
  uint32_t s = mix(threadIdx.x * 2654435761u + blockIdx.x), acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t a[16], r[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      s = s * 1664525u + 1013904223u;
      const uint32_t b = (s >> 8) & (nbk - 1u);
      a[j] = (base + (b << rlog) + rep) << 2;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      r[j] = __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += r[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = h[5] + acc;
  else if (acc == 0xFFFFFFFFu) out[1] = acc;
}

int main() {
  uint32_t* d; (void)hipMalloc(&d, 1 << 20);
  const int blocks = 256, iters = 2000;
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  printf("%-6s %-4s %-9s %10s %14s\n", "nbk", "R", "per-wave", "ms", "cyc/wave-instr/CU");
  for (uint32_t nbk : {8u, 32u, 128u, 512u}) {
    for (uint32_t rlog : {0u, 2u, 3u, 4u, 5u, 6u}) {
      for (uint32_t pw : {0u, 1u}) {
        const uint32_t words = (nbk << rlog) * (pw ? 16u : 1u);
        if (words * 4 > 160 * 1024) continue;
        hipLaunchKernelGGL(k_rank, dim3(blocks), dim3(1024), words * 4, 0, d, 10, nbk, rlog, pw, words);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_rank, dim3(blocks), dim3(1024), words * 4, 0, d, iters, nbk, rlog, pw, words);
        (void)hipEventRecord(b);
        if (hipEventSynchronize(b) != hipSuccess) { printf("kernel failed\n"); return 1; }
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        const double instr_per_cu = (double)blocks / 256 * 16 * iters * 16;   // wave-instructions per CU
        printf("%-6u %-4u %-9u %10.3f %14.2f\n", nbk, 1u << rlog, pw, ms, ms * 1e6 / instr_per_cu * 2.4);
      }
    }
  }
  return 0;
}
