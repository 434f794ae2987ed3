// LDS ds_add_u32 throughput by address pattern (MI355X measurement behind
// DESIGN.md "LDS atomics"): conflict-free lane-consecutive, random, and
// random within lane-parity halves.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_rate tools/lds_atomic_rate.hip && /tmp/lds_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__device__ __forceinline__ uint32_t mix(uint32_t x){x^=x>>16;x*=0x7feb352dU;x^=x>>15;x*=0x846ca68bU;x^=x>>16;return x;}
typedef __attribute__((address_space(3))) uint32_t lds_u32;
template <int MODE>
__global__ void __launch_bounds__(1024) k_lds(uint32_t* out, int iters) {
  extern __shared__ uint32_t h[];
  for (int i = threadIdx.x; i < 16384; i += 1024) h[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t s = mix(threadIdx.x * 2654435761u + blockIdx.x);
  for (int it = 0; it < iters; ++it) {
    uint32_t a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      s = s * 1664525u + 1013904223u;
      uint32_t code;
      if (MODE == 0) code = (lane + 64 * j + 1024 * (it & 7)) & 16383;           // conflict-free
      else if (MODE == 1) code = (s >> 8) & 16383;                                 // random
      else if (MODE == 2) code = (((s >> 8) & 8191) << 1) | (lane & 1);            // random, lane-parity halves
      else code = (s >> 8) & 31;                                                   // 32 hot bins
      a[j] = code << 2;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = h[5];
}
int main() {
  uint32_t* d; (void)hipMalloc(&d, 1 << 20);
  const int blocks = 256 * 2, iters = 2000;
  const char* names[] = {"conflict-free", "random", "random lane-parity halves", "32 hot bins"};
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int m = 0; m < 4; ++m) {
    void (*fn)(uint32_t*, int) = m == 0 ? k_lds<0> : m == 1 ? k_lds<1> : m == 2 ? k_lds<2> : k_lds<3>;
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(1024), 65536, 0, d, 10);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(1024), 65536, 0, d, iters);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    const double instr_per_cu = (double)blocks / 256 * 16 * iters * 16;   // wave-instructions per CU
    printf("%-28s %8.3f ms  %6.2f ns per wave-instr per CU (%.2f cyc @2.4GHz)\n", names[m], ms,
           ms * 1e6 / instr_per_cu, ms * 1e6 / instr_per_cu * 2.4);
  }
  return 0;
}
