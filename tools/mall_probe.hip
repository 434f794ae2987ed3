// Can k=11's record round trip live in the 256 MiB Infinity Cache (MALL)?
// Each workgroup writes its slice of a record buffer R (S bytes in all), then
// reads the slice back (the phase-1 -> phase-2 round trip of one piece), while
// streaming an input buffer (non-temporal loads) and a row buffer (non-temporal
// stores) in the k=11 mix: per 2 B of record, 1 B of input and 1.7 B of row.
// Timed over many cycles for several S; the R traffic is counted twice (write +
// read).  One wave per SIMD-slot pattern as the bucket kernel: 256 workgroups of
// 1024 threads.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mall_probe tools/mall_probe.hip && /tmp/mall_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

// slice: R bytes of this workgroup; in/out: stream slices; mix = 0 -> R only
__global__ void __launch_bounds__(1024) cycle_kernel(v4u* R, size_t rslice, const v4u* in, size_t islice, v4u* out,
                                                     size_t oslice, unsigned salt, unsigned* sink) {
    const size_t nR = rslice / 16, nI = islice / 16, nO = oslice / 16;
    v4u* r = R + blockIdx.x * nR;
    const v4u* a = in + blockIdx.x * nI;
    v4u* o = out + blockIdx.x * nO;
    v4u acc = {0u, 0u, 0u, 0u};
    // phase 1: write the records (and read input)
    for (size_t i = threadIdx.x; i < nR; i += blockDim.x) {
        r[i] = v4u{(unsigned)i ^ salt, salt, (unsigned)i, 1u};
        if (i < nI) acc += __builtin_nontemporal_load(a + i);
    }
    for (size_t i = nR + threadIdx.x; i < nI; i += blockDim.x) acc += __builtin_nontemporal_load(a + i);
    __syncthreads();
    // phase 2: read the records back (and write rows)
    for (size_t i = threadIdx.x; i < nR; i += blockDim.x) {
        acc += r[i];
        if (i < nO) __builtin_nontemporal_store(acc, o + i);
    }
    for (size_t i = nR + threadIdx.x; i < nO; i += blockDim.x) __builtin_nontemporal_store(acc, o + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) atomicAdd(sink, 1u);
}

int main(int argc, char** argv) {
    const int grid = 256;
    const size_t in_total = (size_t)5 << 30, out_total = (size_t)8400 << 20;
    const size_t sizes_mb[] = {32, 64, 128, 192, 256, 384, 512, 1024, 2560};
    const int cycles_per_run = argc > 1 ? atoi(argv[1]) : 8;
    v4u *R, *in, *out;
    unsigned* sink;
    CHECK(hipMalloc(&R, (size_t)2560 << 20));
    CHECK(hipMalloc(&in, in_total));
    CHECK(hipMalloc(&out, out_total));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(in, 1, in_total));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    printf("{\"probe\": \"record round trip through the MALL\", \"runs\": [\n");
    for (int mix = 0; mix < 2; ++mix) {
        for (size_t mb : sizes_mb) {
            const size_t S = mb << 20;
            const size_t rslice = S / grid & ~(size_t)15;
            // the stream per cycle scales with S as in k=11 (1 B in, 1.7 B row per 2 B record), capped
            size_t islice = mix ? rslice / 2 : 0, oslice = mix ? rslice * 17 / 20 : 0;
            islice &= ~(size_t)15;
            oslice &= ~(size_t)15;
            if (islice * grid > in_total || oslice * grid > out_total) continue;
            for (int warm = 0; warm < 2; ++warm)
                hipLaunchKernelGGL(cycle_kernel, dim3(grid), dim3(1024), 0, 0, R, rslice, in, islice, out, oslice,
                                   (unsigned)warm, sink);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int c = 0; c < cycles_per_run; ++c)
                hipLaunchKernelGGL(cycle_kernel, dim3(grid), dim3(1024), 0, 0, R, rslice, in, islice, out, oslice,
                                   (unsigned)c + 7u, sink);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double per = ms / cycles_per_run * 1e-3;
            const double rbytes = 2.0 * rslice * grid, sbytes = (double)(islice + oslice) * grid;
            printf("  {\"mix\": %d, \"R_MB\": %zu, \"us_per_cycle\": %.1f, \"R_roundtrip_TBps\": %.2f, "
                   "\"all_TBps\": %.2f}%s\n", mix, mb, per * 1e6, rbytes / per / 1e12, (rbytes + sbytes) / per / 1e12,
                   (mix == 1 && mb == sizes_mb[sizeof(sizes_mb) / sizeof(sizes_mb[0]) - 1]) ? "" : ",");
        }
    }
    printf("]}\n");
    return 0;
}
