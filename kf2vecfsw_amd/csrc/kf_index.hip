// kf_index.hip -- the FASTA record index of a batch on the device (what the host
// finds per file with kf_index_records, reference path kf2vec/main.py:309-311:
// Jellyfish's record parsing), so that the CLI's readers only copy bytes.
//
// A header is a line that starts with '>' (at a genome start or after '\n'); it
// is excluded up to its '\n' (or the genome end).  Unlike the host index, header
// lines that follow each other stay separate pairs (the count kernels treat
// adjacent ranges like one).  Three launches: per-block header counts, a
// one-workgroup block scan, and a scatter of the pairs in order; the number of
// pairs stays on the device (kf_count_batch_dev reads it there).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kf_internal.h"

namespace kf {
namespace {

constexpr int kIBlock = 256;                   // threads per workgroup
constexpr int kIPer = 16;                      // bytes per thread
constexpr uint32_t kISpan = kIBlock * kIPer;   // 4 KiB per workgroup

// genome of byte i (< goff[n]): the last g with goff[g] <= i
__device__ __forceinline__ int genome_of(const uint64_t* goff, int n, uint64_t i) {
    int lo = 0, hi = n;
    while (hi - lo > 1) {
        const int m = (lo + hi) >> 1;
        if (goff[m] <= i) lo = m;
        else hi = m;
    }
    return lo;
}

// header starts among the thread's 16 bytes (bit q: byte p0 + q)
__device__ __forceinline__ uint32_t thread_heads(const uint8_t* bytes, uint64_t end, const uint64_t* goff, int n,
                                                 uint64_t p0) {
    uint32_t m = 0;
    if (p0 >= end) return 0;
    uint8_t prev = p0 > 0 ? bytes[p0 - 1] : (uint8_t)'\n';
    for (int q = 0; q < kIPer; ++q) {
        const uint64_t i = p0 + q;
        if (i >= end) break;
        const uint8_t c = bytes[i];
        if (c == '>') {
            bool start = prev == '\n' || i == 0;
            if (!start) {   // a genome start (genomes need not end with '\n')
                const int g = genome_of(goff, n, i);
                start = goff[g] == i;
            }
            if (start) m |= 1u << q;
        }
        prev = c;
    }
    return m;
}

__global__ void __launch_bounds__(kIBlock) idx_count_kernel(const uint8_t* bytes, uint64_t end, const uint64_t* goff,
                                                            int n, uint32_t* blk) {
    __shared__ uint32_t red[kIBlock / 64];
    const uint64_t p0 = (uint64_t)blockIdx.x * kISpan + (uint64_t)threadIdx.x * kIPer;
    uint32_t c = (uint32_t)__builtin_popcount(thread_heads(bytes, end, goff, n, p0));
    for (int d = 32; d >= 1; d >>= 1) c += (uint32_t)__shfl_xor((int)c, d, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) blk[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// exclusive scan of nb block counts in place (one workgroup); blk[nb] = total,
// also written to *n_pairs
__global__ void __launch_bounds__(1024) idx_scan_kernel(uint32_t* blk, uint32_t nb, uint64_t* n_pairs) {
    __shared__ uint32_t sh[1024];
    const uint32_t t = threadIdx.x;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += 1024) {
        const uint32_t i = base + t;
        const uint32_t v = i < nb ? blk[i] : 0u;
        sh[t] = v;
        __syncthreads();
        for (uint32_t d = 1; d < 1024; d <<= 1) {
            const uint32_t o = t >= d ? sh[t - d] : 0u;
            __syncthreads();
            sh[t] += o;
            __syncthreads();
        }
        if (i < nb) blk[i] = carry + sh[t] - v;
        carry += sh[1023];
        __syncthreads();
    }
    if (t == 0) {
        blk[nb] = carry;
        *n_pairs = carry;
    }
}

__global__ void __launch_bounds__(kIBlock) idx_scatter_kernel(const uint8_t* bytes, uint64_t end, const uint64_t* goff,
                                                              int n, const uint32_t* blk, uint64_t* excl,
                                                              uint64_t cap) {
    __shared__ uint32_t wsum[kIBlock / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t p0 = (uint64_t)blockIdx.x * kISpan + (uint64_t)threadIdx.x * kIPer;
    uint32_t m = thread_heads(bytes, end, goff, n, p0);
    const uint32_t c = (uint32_t)__builtin_popcount(m);
    uint32_t inc = c;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0;
    for (int x = 0; x < w; ++x) before += wsum[x];
    uint64_t u = (uint64_t)blk[blockIdx.x] + before + inc - c;
    while (m) {
        const int q = __builtin_ctz(m);
        m &= m - 1;
        const uint64_t j = p0 + (uint64_t)q;
        if (u < cap) {
            const uint64_t ge = goff[genome_of(goff, n, j) + 1];
            uint64_t e = j;
            while (e < ge && bytes[e] != '\n') ++e;   // the header line (short)
            excl[2 * u] = j;
            excl[2 * u + 1] = e;
        }
        ++u;
    }
}

}  // namespace
}  // namespace kf

using namespace kf;

extern "C" int kf_index_fasta(const uint8_t* d_bytes, const uint64_t* d_goff, int32_t n_genomes, uint64_t batch_bytes,
                              uint64_t* d_excl, uint64_t cap_pairs, uint64_t* d_n_pairs, uint32_t* d_scratch,
                              uint64_t scratch_words, void* stream) {
    if (n_genomes < 0) return kf_fail(KF_EINVAL, "n_genomes < 0");
    if (!d_n_pairs) return kf_fail(KF_EINVAL, "null device pointer");
    hipStream_t s = (hipStream_t)stream;
    if (n_genomes == 0 || batch_bytes == 0) {
        if (hipMemsetAsync(d_n_pairs, 0, 8, s) != hipSuccess) return kf_fail(KF_EHIP, "memset failed");
        return KF_OK;
    }
    if (!d_bytes || !d_goff || !d_scratch || (cap_pairs && !d_excl)) return kf_fail(KF_EINVAL, "null device pointer");
    const uint64_t nb = (batch_bytes + kISpan - 1) / kISpan;
    if (nb >= (1ull << 31)) return kf_fail(KF_EINVAL, "batch too large");
    if (scratch_words < nb + 1)
        return kf_fail(KF_ERANGE, "scratch needs %llu words", (unsigned long long)(nb + 1));
    hipLaunchKernelGGL(idx_count_kernel, dim3((uint32_t)nb), dim3(kIBlock), 0, s, d_bytes, batch_bytes, d_goff,
                       n_genomes, d_scratch);
    hipLaunchKernelGGL(idx_scan_kernel, dim3(1), dim3(1024), 0, s, d_scratch, (uint32_t)nb, d_n_pairs);
    hipLaunchKernelGGL(idx_scatter_kernel, dim3((uint32_t)nb), dim3(kIBlock), 0, s, d_bytes, batch_bytes, d_goff,
                       n_genomes, d_scratch, d_excl, cap_pairs);
    if (hipGetLastError() != hipSuccess) return kf_fail(KF_EHIP, "record index launch failed");
    return KF_OK;
}
