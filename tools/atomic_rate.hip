// Random u32 global atomicAdd throughput vs footprint (MI355X measurement behind
// ~25-27 G atomics/s whatever the footprint).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/atomic_rate tools/atomic_rate.hip && /tmp/atomic_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__device__ __forceinline__ uint32_t mix(uint32_t x){x^=x>>16;x*=0x7feb352dU;x^=x>>15;x*=0x846ca68bU;x^=x>>16;return x;}
// each thread does N atomics to random addresses in [0, span) of region (g = blockIdx-derived region)
__global__ void k_atom(uint32_t* base, uint64_t region_words, uint32_t span_words, int n_regions, int per_thread) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  int reg = (blockIdx.x / 8) % n_regions;
  uint32_t* r = base + (uint64_t)reg * region_words;
  uint32_t s = mix(t * 2654435761u + 1);
  for (int i = 0; i < per_thread; ++i) {
    s = mix(s + i);
    __hip_atomic_fetch_add(r + (s % span_words), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
int main() {
  size_t total = 9ull << 30;
  uint32_t* d; if (hipMalloc(&d, total) != hipSuccess) { printf("alloc fail\n"); return 1; }
  hipMemset(d, 0, total);
  int blocks = 256 * 8, threads = 256, per = 256;
  double n = (double)blocks * threads * per;
  struct C { const char* name; uint64_t region_words; uint32_t span; int nreg; } cs[] = {
    {"L2 1MB x1", 1<<18, 1<<18, 1},
    {"2MB x1", 1<<19, 1<<19, 1},
    {"8.4MB x1 (1 genome k11)", 2097152, 2097152, 1},
    {"8.4MB x16 regions", 2097152, 2097152, 16},
    {"8.4MB x64 regions", 2097152, 2097152, 64},
    {"8.4MB x256 regions (2GB)", 2097152, 2097152, 256},
    {"8.4MB x1000 regions (8.4GB)", 2097152, 2097152, 1000},
  };
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (auto& c : cs) {
    k_atom<<<blocks, threads>>>(d, c.region_words, c.span, c.nreg, 16);
    hipEventRecord(a);
    k_atom<<<blocks, threads>>>(d, c.region_words, c.span, c.nreg, per);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-32s %8.3f ms  %8.1f G atomics/s\n", c.name, ms, n / ms / 1e6);
  }
  return 0;
}
