// kf_chunks.hip -- device pre-pass of kf2vec's `get_chunks` (reference
// kf2vec/main.py:654-929) for MI355X (gfx950).
//
// The reference turns every genome into 10 kbp windows with four external
// tools before counting each window with its own Jellyfish pair:
//   seqtk seq -l 0          linearise each record (main.py:732)
//   awk gsub(/[N|n]+/,"N")  collapse runs of N, n and '|' into one 'N' (:740-742)
//   seqkit seq -m 10000 -g  drop the gap letters "- \t." and contigs < 10 kbp (:753)
//   seqkit sliding          windows of 10 kbp at step 10000 - ovrlap (:813-824)
// Here one compaction pass over the genome's bytes in HBM produces every
// record's processed sequence (kf_chunk_compact), the host plans the windows
// from the record lengths, and one gather lays the windows out back to back
// for kf_count_batch (kf_chunk_gather).
//
// Compaction, per byte i of record r's sequence region [a_r, b_r):
//   dropped: '\n', a '\r' that ends a line (kseq strips it), the gap letters;
//   an N-class byte (N, n, '|') is kept -- as 'N' -- only if the byte before it
//   in the linearised record (newlines and line-end '\r' skipped, gap letters
//   NOT skipped: awk runs before seqkit) is not N-class;
//   every other byte is kept as is (lowercase, IUPAC, stray '>': the counter
//   treats them as it treats them anywhere).
// Three launches: per-block kept counts, one-workgroup block scan, scatter.
// Record r's processed sequence is out[out_se[2r], out_se[2r+1]).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kf_internal.h"

namespace kf {
namespace {

constexpr int kCBlock = 256;                 // threads per workgroup
constexpr int kCPer = 16;                    // bytes per thread
constexpr uint32_t kCSpan = kCBlock * kCPer; // bytes per workgroup (4 KiB)

__device__ __forceinline__ bool is_n(uint8_t c) { return c == 'N' || c == 'n' || c == '|'; }
__device__ __forceinline__ bool is_gap(uint8_t c) { return c == '-' || c == ' ' || c == '\t' || c == '.'; }

// Record of byte i (the last record starting at or before i), or -1; records
// are sorted and disjoint.  Wave-uniform-free binary search (per thread).
__device__ __forceinline__ int32_t rec_of(const uint64_t* se, int32_t n, uint64_t i) {
    int32_t lo = 0, hi = n;   // first record with start > i
    while (lo < hi) {
        const int32_t m = (lo + hi) >> 1;
        if (se[2 * m] <= i) lo = m + 1;
        else hi = m;
    }
    const int32_t r = lo - 1;
    return (r >= 0 && i < se[2 * r + 1]) ? r : -1;
}

// Is byte j (inside [a, b)) dropped as a line break: '\n', or '\r' that ends a line?
__device__ __forceinline__ bool line_break(const uint8_t* bytes, uint64_t j, uint64_t b) {
    const uint8_t c = bytes[j];
    return c == '\n' || (c == '\r' && (j + 1 == b || bytes[j + 1] == '\n'));
}

// Keep byte i of the region [a, b)?  *out receives the byte written.
__device__ __forceinline__ bool keep_byte(const uint8_t* bytes, uint64_t i, uint64_t a, uint64_t b, uint8_t* out) {
    const uint8_t c = bytes[i];
    if (line_break(bytes, i, b) || is_gap(c)) return false;
    if (is_n(c)) {
        uint64_t j = i;
        while (j > a) {   // the linearised predecessor (rarely more than one step back)
            --j;
            if (!line_break(bytes, j, b)) {
                if (is_n(bytes[j])) return false;
                break;
            }
        }
        *out = 'N';
        return true;
    }
    *out = c;
    return true;
}

// Kept bytes of thread t's 16 bytes; records looked up once per thread.
__device__ __forceinline__ uint32_t thread_keep(const uint8_t* bytes, uint64_t len, const uint64_t* se, int32_t n,
                                                uint64_t p0, uint8_t (&ch)[kCPer], uint32_t& mask) {
    uint32_t cnt = 0;
    mask = 0;
    if (p0 >= len) return 0;
    int32_t r = rec_of(se, n, p0);
    for (int q = 0; q < kCPer; ++q) {
        const uint64_t i = p0 + q;
        if (i >= len) break;
        if (r < 0 || i >= se[2 * r + 1]) {   // find the record of i (after a record end)
            r = rec_of(se, n, i);
            if (r < 0) continue;
        }
        uint8_t c;
        if (keep_byte(bytes, i, se[2 * r], se[2 * r + 1], &c)) {
            ch[q] = c;
            mask |= 1u << q;
            ++cnt;
        }
    }
    return cnt;
}

__global__ void __launch_bounds__(kCBlock) chunk_count_kernel(const uint8_t* bytes, uint64_t len, const uint64_t* se,
                                                                int32_t n, uint32_t* blk) {
    __shared__ uint32_t red[kCBlock / 64];
    const uint64_t p0 = (uint64_t)blockIdx.x * kCSpan + (uint64_t)threadIdx.x * kCPer;
    uint8_t ch[kCPer];
    uint32_t mask;
    uint32_t c = thread_keep(bytes, len, se, n, p0, ch, mask);
    for (int d = 32; d >= 1; d >>= 1) c += (uint32_t)__shfl_xor((int)c, d, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) blk[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Exclusive scan of nb block counts in place (one workgroup), blk[nb] = total.
__global__ void __launch_bounds__(1024) chunk_scan_kernel(uint32_t* blk, uint32_t nb) {
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
    if (t == 0) blk[nb] = carry;
}

__global__ void __launch_bounds__(kCBlock) chunk_scatter_kernel(const uint8_t* bytes, uint64_t len, const uint64_t* se,
                                                                  int32_t n, const uint32_t* blk, uint8_t* out) {
    __shared__ uint32_t wsum[kCBlock / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t p0 = (uint64_t)blockIdx.x * kCSpan + (uint64_t)threadIdx.x * kCPer;
    uint8_t ch[kCPer];
    uint32_t mask;
    const uint32_t c = thread_keep(bytes, len, se, n, p0, ch, mask);
    // exclusive prefix of c over the workgroup
    uint32_t inc = c;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0;
    for (int x = 0; x < w; ++x) before += wsum[x];
    uint64_t pos = (uint64_t)blk[blockIdx.x] + before + inc - c;
    for (int q = 0; q < kCPer; ++q)
        if (mask & (1u << q)) out[pos++] = ch[q];
}

// Compacted [start, end) of every record: the kept bytes before a_r and b_r.
__global__ void __launch_bounds__(256) chunk_bounds_kernel(const uint8_t* bytes, uint64_t len, const uint64_t* se,
                                                             int32_t n, const uint32_t* blk, uint64_t* out_se) {
    const int32_t x = blockIdx.x * blockDim.x + threadIdx.x;   // one bound per thread: 2n of them
    if (x >= 2 * n) return;
    const uint64_t p = min(se[x], len);
    const uint64_t b0 = p / kCSpan * kCSpan;
    uint64_t cnt = blk[p / kCSpan];
    // kept bytes of [b0, p): only bytes inside records count
    int32_t r = -1;
    for (uint64_t i = b0; i < p; ++i) {
        if (r < 0 || i >= se[2 * r + 1]) {
            r = rec_of(se, n, i);
            if (r < 0) continue;
        }
        uint8_t c;
        if (keep_byte(bytes, i, se[2 * r], se[2 * r + 1], &c)) ++cnt;
    }
    out_se[x] = cnt;
}

// Window w = src[win_src[w], + win_len) -> dst[w * win_len, + win_len).
__global__ void __launch_bounds__(256) chunk_gather_kernel(const uint8_t* src, const uint64_t* win_src, uint32_t win_len,
                                                             uint8_t* dst) {
    const uint64_t s = win_src[blockIdx.x];
    uint8_t* d = dst + (uint64_t)blockIdx.x * win_len;
    for (uint32_t i = threadIdx.x; i < win_len; i += blockDim.x) d[i] = src[s + i];
}

}  // namespace
}  // namespace kf

using namespace kf;

extern "C" int kf_chunk_compact(const uint8_t* d_bytes, uint64_t len, const uint64_t* d_seq, int32_t n_rec,
                                uint8_t* d_out, uint64_t* d_out_se, uint32_t* d_scratch, uint64_t scratch_words,
                                void* stream) {
    if (n_rec < 0) return kf_fail(KF_EINVAL, "n_rec < 0");
    if (n_rec == 0) return KF_OK;
    if (!d_bytes || !d_seq || !d_out || !d_out_se || !d_scratch) return kf_fail(KF_EINVAL, "null device pointer");
    // block counts, their scan and the record bounds are 32-bit: the processed
    // sequence of one call must stay below 4 GiB
    if (len >= (1ull << 32)) return kf_fail(KF_EINVAL, "input of %llu bytes: at most 4 GiB - 1 per call",
                                            (unsigned long long)len);
    const uint64_t nb = (len + kCSpan - 1) / kCSpan;
    if (scratch_words < nb + 1) return kf_fail(KF_ERANGE, "scratch needs %llu words", (unsigned long long)(nb + 1));
    hipStream_t s = (hipStream_t)stream;
    if (nb) {
        hipLaunchKernelGGL(chunk_count_kernel, dim3((uint32_t)nb), dim3(kCBlock), 0, s, d_bytes, len, d_seq, n_rec,
                           d_scratch);
        hipLaunchKernelGGL(chunk_scan_kernel, dim3(1), dim3(1024), 0, s, d_scratch, (uint32_t)nb);
        hipLaunchKernelGGL(chunk_scatter_kernel, dim3((uint32_t)nb), dim3(kCBlock), 0, s, d_bytes, len, d_seq, n_rec,
                           d_scratch, d_out);
    } else {
        if (hipMemsetAsync(d_scratch, 0, sizeof(uint32_t), s) != hipSuccess) return kf_fail(KF_EHIP, "memset failed");
    }
    hipLaunchKernelGGL(chunk_bounds_kernel, dim3((2 * n_rec + 255) / 256), dim3(256), 0, s, d_bytes, len, d_seq, n_rec,
                       d_scratch, d_out_se);
    if (hipGetLastError() != hipSuccess) return kf_fail(KF_EHIP, "chunk compaction launch failed");
    return KF_OK;
}

extern "C" int kf_chunk_gather(const uint8_t* d_src, const uint64_t* d_win_src, int32_t n_win, uint32_t win_len,
                               uint8_t* d_dst, void* stream) {
    if (n_win < 0) return kf_fail(KF_EINVAL, "n_win < 0");
    if (n_win == 0) return KF_OK;
    if (!d_src || !d_win_src || !d_dst) return kf_fail(KF_EINVAL, "null device pointer");
    hipLaunchKernelGGL(chunk_gather_kernel, dim3((uint32_t)n_win), dim3(256), 0, (hipStream_t)stream, d_src, d_win_src,
                       win_len, d_dst);
    if (hipGetLastError() != hipSuccess) return kf_fail(KF_EHIP, "chunk gather launch failed");
    return KF_OK;
}
