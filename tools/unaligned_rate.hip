// Streaming read rate with unaligned 16-byte buffer loads (K1L design probe):
// every lane reads 96 bytes at byte offset 81 * lane - 16 of a 64-line block
// (5184 bytes per wave iteration), against the same reads at a 96-byte stride
// (aligned) and the production 48-byte stride.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/unaligned_rate tools/unaligned_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int MODE>
__global__ void __launch_bounds__(1024) probe(const uint8_t* bytes, uint64_t n, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * 16ull + (threadIdx.x >> 6));
    const uint64_t nwaves = gridDim.x * 16ull;
    constexpr uint32_t kBlock = MODE == 2 ? 3072u : (MODE == 3 ? 2048u : (MODE == 4 ? 1024u : (MODE == 5 ? 3072u : 5184u)));
    const uint64_t nblk = n / kBlock - 1;
    uint32_t acc = 0;
    // 4 blocks in flight per wave: issue all loads of 4 blocks, then consume
    for (uint64_t b = wave; b + 3 * nwaves < nblk; b += 4 * nwaves) {
        uint4 v[4][6];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t base = 16 + (b + k * nwaves) * kBlock;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + base - 16), (short)0, (int)(kBlock + 64), 0x00020000);
            const uint32_t off = MODE == 0 ? 81u * lane : (MODE == 1 ? 96u * lane : (MODE == 3 ? 32u * lane : (MODE == 4 || MODE == 5 ? 16u * lane : 48u * lane)));
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if ((MODE == 2 || MODE == 5) && q >= 3) break;
                if (MODE == 3 && q >= 2) break;
                if (MODE == 4 && q >= 1) break;
                const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, MODE == 5 ? off + 1024 * q : off + 16 * q, 0, 0);
                v[k][q] = make_uint4(t[0], t[1], t[2], t[3]);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if ((MODE == 2 || MODE == 5) && q >= 3) break;
                if (MODE == 3 && q >= 2) break;
                if (MODE == 4 && q >= 1) break;
                acc ^= v[k][q].x + v[k][q].y + v[k][q].z + v[k][q].w;
            }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t n = 5062656000ull;
    uint8_t* d = nullptr;
    uint32_t* o = nullptr;
    if (hipMalloc(&d, n + 4096) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    hipMemset(d, 0x41, n + 4096);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[6] = {"81-byte stride, unaligned 16-B loads (6 per lane)", "96-byte stride, aligned (6 per lane)",
                            "48-byte stride, aligned (3 per lane, K1x)", "32-byte stride (2 per lane, K1w)",
                            "16-byte stride (1 per lane, K1)", "16-byte stride, 3 KiB per wave (3 per lane, coalesced)"};
    for (int rep = 0; rep < 3; ++rep)
        for (int m = 0; m < 6; ++m) {
            float best = 1e9f;
            for (int it = 0; it < 5; ++it) {
                hipEventRecord(a);
                if (m == 0) probe<0><<<256, 1024>>>(d, n, o);
                if (m == 1) probe<1><<<256, 1024>>>(d, n, o);
                if (m == 2) probe<2><<<256, 1024>>>(d, n, o);
                if (m == 3) probe<3><<<256, 1024>>>(d, n, o);
                if (m == 4) probe<4><<<256, 1024>>>(d, n, o);
                if (m == 5) probe<5><<<256, 1024>>>(d, n, o);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            const double data = (double)n;
            printf("%-52s %.3f ms  %.0f GB/s of input\n", names[m], best, data / (best * 1e-3) / 1e9);
        }
    return 0;
}
