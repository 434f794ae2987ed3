// Streaming read rate of the K1x load layout (lane L reads bytes 48L + 16q, q = 0..2,
// of a 3 KiB wave block) against the coalesced layout (16L + 1024q), by buffer-load
// cache policy (aux bits: 1 = sc0, 2 = nt, 16 = sc1) and blocks in flight per wave
// (2 = K1x's ring, 4).  256 workgroups x 16 waves, 5.06 GB, best of 5.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ab/cpol_rate tools/cpol_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// LAYOUT 0: 48-byte lanes, 1: coalesced, 2: 32-byte lanes (2 loads of 16 B at 32L + 16q,
// three 2 KiB blocks per 6 KiB).  AUX >= 100: 48-byte lanes with aux 0 on loads q < 2 and
// AUX - 100 on load 2 (the last touch of each line).
template <int LAYOUT, int AUX, int RING>
__global__ void __launch_bounds__(1024) probe(const uint8_t* bytes, uint64_t n, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * 16ull + (threadIdx.x >> 6));
    const uint64_t nwaves = gridDim.x * 16ull;
    constexpr uint32_t kBlock = 3072u;
    // contiguous per-wave spans like the kernel's wave ranges
    const uint64_t nblk = n / kBlock;
    const uint64_t per = nblk / nwaves;
    const uint64_t b0 = wave * per;
    const uint32_t off0 = LAYOUT == 0 ? 48u * lane : (LAYOUT == 2 ? 32u * lane : 16u * lane);
    const uint32_t step = LAYOUT == 0 ? 16u : 1024u;
    uint32_t acc = 0;
    uint4 v[RING][3];
    auto load = [&](uint64_t b, uint4 (&d)[3]) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + b * kBlock), (short)0, (int)kBlock, 0x00020000);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            constexpr int A0 = AUX >= 100 ? 0 : AUX, A2 = AUX >= 100 ? AUX - 100 : AUX;
            // 32-byte lanes: loads (q = 0, 1) of the first 2 KiB, then q = 2 at 2048 + 16 L
            const uint32_t o = LAYOUT == 2 ? (q < 2 ? off0 + 16u * q : 2048u + 16u * lane) : off0 + step * q;
            const auto t = q == 2 ? __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, A2)
                                  : __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, A0);
            d[q] = make_uint4(t[0], t[1], t[2], t[3]);
        }
    };
#pragma unroll
    for (int j = 0; j < RING; ++j) load(b0 + j, v[j]);
    for (uint64_t i = 0; i + RING <= per; i += RING) {
#pragma unroll
        for (int j = 0; j < RING; ++j) {
#pragma unroll
            for (int q = 0; q < 3; ++q) acc ^= v[j][q].x + v[j][q].y + v[j][q].z + v[j][q].w;
            if (i + j + RING < per) load(b0 + i + j + RING, v[j]);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int LAYOUT, int AUX, int RING>
void run(const uint8_t* d, uint64_t n, uint32_t* o, hipEvent_t a, hipEvent_t b) {
    float best = 1e9f;
    for (int it = 0; it < 5; ++it) {
        (void)hipEventRecord(a);
        probe<LAYOUT, AUX, RING><<<256, 1024>>>(d, n, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    printf("%-10s aux %3d ring %d  %.3f ms  %.0f GB/s\n", LAYOUT == 0 ? "48B-lanes" : (LAYOUT == 2 ? "32B-lanes" : "coalesced"), AUX, RING, best,
           (double)n / (best * 1e-3) / 1e9);
}

int main() {
    const uint64_t n = 5062656000ull;
    uint8_t* d = nullptr;
    uint32_t* o = nullptr;
    if (hipMalloc(&d, n + 4096) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    (void)hipMemset(d, 0x41, n + 4096);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) {
        run<0, 0, 2>(d, n, o, a, b);
        run<0, 102, 2>(d, n, o, a, b);
        run<0, 101, 2>(d, n, o, a, b);
        run<0, 116, 2>(d, n, o, a, b);
        run<2, 0, 2>(d, n, o, a, b);
        run<2, 2, 2>(d, n, o, a, b);
        run<1, 0, 2>(d, n, o, a, b);
        run<1, 2, 2>(d, n, o, a, b);
        run<1, 1, 2>(d, n, o, a, b);
        run<1, 16, 2>(d, n, o, a, b);
        run<1, 18, 2>(d, n, o, a, b);
    }
    return 0;
}
