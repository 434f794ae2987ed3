// kf_sparse.hip -- `get_kmers` at any k = 2..31 (reference kf2vec/main.py:112-176)
// for MI355X (gfx950).
//
// The reference runs `jellyfish count -m K -C` + `jellyfish dump -c -t` per genome
// and keeps the PRESENT canonical k-mers only (main.py:133-160); its parser
// accepts k = 2..31 (main.py:81-82, 1006).  A dense 4^k/2-bin row stops being
// possible past k ~ 13 (k = 31: 2^61 bins), so this path sorts instead of
// histogramming:
//   1. emit    one key per input byte: the canonical code of the window ending
//              at that byte (standard 2-bit code A0 C1 G2 T3, canonical = the
//              smaller of the code and its reverse complement, i.e. the
//              lexicographically smaller string), or SENT (= 4^k - 1, the code of
//              T..T, never canonical) where no window ends;
//   2. sort    each genome's keys, a segmented LSD radix sort of 2k bits in
//              ceil(2k/8) passes of equal <= 8-bit digits: one read counts every
//              pass's digits per genome, then each pass is one single-sweep
//              kernel (ranks by LDS atomics, the tile's digit offsets by
//              decoupled look-back over the genome's earlier tiles, the tile
//              re-ordered in LDS so every digit's keys leave as one run);
//   3. unique  run heads of the sorted keys compacted with their positions; a
//              run's count is the distance to the next head.  SENT sorts last and
//              is dropped.
// Keys are u32 for k <= 16 (half the bytes of every pass) and u64 above.
//
// Semantics are those of the dense counter (kf_count_batch): '\n' is
// transparent, any other non-ACGT byte (either case counts) breaks the window,
// the excluded byte ranges (headers, FASTQ '+' / quality lines, from
// kf_index_records) break it too, and a window never spans two genomes.
//
// Layout: genome g owns key slots [goff[g], goff[g+1]) in every buffer (a genome
// has at most as many windows as bytes), cut into tiles (TileOf); tile t of
// the batch belongs to the genome g with tfirst[g] <= t < tfirst[g+1].
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kf_internal.h"

namespace kf {
namespace {

constexpr int kSBlock = 256;                   // threads per workgroup (4 waves)
constexpr int kSWaves = kSBlock / 64;
constexpr int kEB = 32;                        // emit: bytes per thread
// Key slots per tile: 16384 u32 keys or 8192 u64 keys (64 / 32 keys per 8-bit
// digit run on average, 256-byte runs; the scatter stages 64 KiB).  With the
// single-sweep passes fewer, larger tiles win despite 2-3 waves per SIMD
// (profiles/r04/v49_*, v51_*: k = 31 17.1 -> 15.2 ms against u64 4096, k = 16
// 7.14 -> 6.81 against u32 8192).
template <typename KeyT>
struct TileOf {
#ifndef KF_SPARSE_TILE64   // u64 tile (tools/ A/B builds)
#define KF_SPARSE_TILE64 8192
#endif
#ifndef KF_SPARSE_TILE32   // u32 tile (tools/ A/B builds)
#define KF_SPARSE_TILE32 16384
#endif
    static constexpr uint32_t tile = sizeof(KeyT) == 4 ? (uint32_t)KF_SPARSE_TILE32 : (uint32_t)KF_SPARSE_TILE64;
    static constexpr int per = tile / kSBlock;             // slots per thread
    static constexpr uint32_t wave_span = tile / kSWaves;  // slots per wave
    static constexpr int emit_threads = tile / kEB;        // emit: kEB bytes per thread
    static_assert(emit_threads % 64 == 0 && emit_threads <= 1024, "emit: whole waves per tile");
};
constexpr uint32_t tile_for_k(int k) { return k <= 16 ? TileOf<uint32_t>::tile : TileOf<uint64_t>::tile; }

// Standard 2-bit code of a byte: A0 C1 G2 T3 (either case), 4 = '\n', 5 = other.
// Branch-free (a switch compiled to a compare tree with exec-mask branches per
// byte): u = c | 0x20 is a, c, g or t only for those letters in either case
// (bit 5 is the only case bit), bits 0, 2, 6, 19 of 0x80045 mark them, and
// x = (u >> 1) & 3 is a0 c1 g3 t2, so x ^ (x >> 1) is the standard code.
__device__ __forceinline__ uint32_t sp_code(uint8_t c) {
    const uint32_t u = (uint32_t)c | 0x20u, i = u - (uint32_t)'a';
    const bool base = i < 26u && ((0x80045u >> i) & 1u);
    const uint32_t x = (u >> 1) & 3u;
    return base ? (x ^ (x >> 1)) : (c == '\n' ? 4u : 5u);
}

// Genome of tile t (t < tfirst[n]): the last g with tfirst[g] <= t (empty
// genomes share their tfirst with the next genome).
__device__ __forceinline__ int tile_genome(const uint32_t* tfirst, int n, uint32_t t) {
    int lo = 0, hi = n;
    while (hi - lo > 1) {
        const int m = (lo + hi) >> 1;
        if (tfirst[m] <= t) lo = m;
        else hi = m;
    }
    return lo;
}

struct TileSpan {
    uint32_t g, gs, ge, base, cnt;   // genome, its slot range, the tile's first slot and slot count
};

// tfirst[n + 2 + t] = the genome of tile t (sp_tilemap_kernel): one load
// instead of a binary search's chain of dependent loads at every tile's start
__device__ __forceinline__ bool tile_span(const uint64_t* goff, const uint32_t* tfirst, int n, uint32_t t,
                                          TileSpan& ts, uint32_t span) {
    if (t >= tfirst[n]) return false;
    ts.g = tfirst[n + 2 + t];
    ts.gs = (uint32_t)goff[ts.g];
    ts.ge = (uint32_t)goff[ts.g + 1];
    ts.base = ts.gs + (t - tfirst[ts.g]) * span;
    ts.cnt = min(span, ts.ge - ts.base);
    return true;
}

// Exclusive prefix of one value per thread over the 256-thread workgroup.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0;
    for (int x = 0; x < w; ++x) before += wsum[x];
    __syncthreads();
    return before + inc - v;
}

// Ranking inside a wave-instruction of the stable scatter:
//   1 (default): LDS atomics, one returning add per key into the wave's digit
//     counter -- an LDS unit serves the lanes of one instruction that hit the
//     same address in lane order, so ranks follow the keys' order;
//   0: ballot matching (one ballot per digit bit; ~46 VALU per 64 keys), which
//     needs no such ordering.
// The heads kernel checks every genome's final order (a key below its
// predecessor flags the call: all counts come back UINT64_MAX - 1), so an
// ordering the hardware did not keep cannot pass silently.
#ifndef KF_SPARSE_RANK
#define KF_SPARSE_RANK 1
#endif

#if KF_SPARSE_RANK == 0
// Lanes of the wave (among `valid`) whose digit equals this lane's: one ballot
// per digit bit.
__device__ __forceinline__ uint64_t match_digit(uint32_t d, int bits, uint64_t valid) {
    uint64_t m = valid;
    for (int b = 0; b < bits; ++b) {
        const bool one = (d >> b) & 1u;
        const uint64_t bb = __ballot(one);
        m &= one ? bb : ~bb;
    }
    return m;
}
#endif

// ---- tiles: tfirst[g] = exclusive prefix of ceil(len_g / span), tfirst[n] = total.
// A goff that decreases or ends past batch_bytes (the buffers' size) sets
// tfirst[n+1] and leaves every tile count at 0: nothing is read or written, and
// every genome's distinct-k-mer count comes back as UINT64_MAX.
__global__ void __launch_bounds__(1024) sp_tiles_kernel(const uint64_t* goff, int n, uint64_t batch_bytes,
                                                        uint32_t span, uint32_t* tfirst) {
    __shared__ uint32_t sh[1024];
    __shared__ int bad;
    const int t = threadIdx.x;
    if (t == 0) bad = goff[n] > batch_bytes;
    __syncthreads();
    for (int g = t; g < n; g += 1024)
        if (goff[g + 1] < goff[g]) bad = 1;
    __syncthreads();
    const bool ok = !bad;
    uint32_t carry = 0;
    for (int base = 0; base < n; base += 1024) {
        const int g = base + t;
        const uint32_t v = g < n && ok ? (uint32_t)((goff[g + 1] - goff[g] + span - 1) / span) : 0u;
        sh[t] = v;
        __syncthreads();
        for (int d = 1; d < 1024; d <<= 1) {
            const uint32_t o = t >= d ? sh[t - d] : 0u;
            __syncthreads();
            sh[t] += o;
            __syncthreads();
        }
        if (g < n) tfirst[g] = carry + sh[t] - v;
        carry += sh[1023];
        __syncthreads();
    }
    if (t == 0) {
        tfirst[n] = carry;
        tfirst[n + 1] = ok ? 0u : 1u;
    }
}

// ---- tile map: tfirst[n + 2 + t] = genome of tile t; xlo[t] = the first
// excluded range ending after the tile's first slot (xlo[tiles] = n_excl)
__global__ void __launch_bounds__(256) sp_tilemap_kernel(const uint64_t* goff, uint32_t* tfirst, int n,
                                                         const uint64_t* excl, uint32_t n_excl, uint32_t span,
                                                         uint32_t* xlo) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x, nt = tfirst[n];
    if (t > nt) return;
    if (t == nt) {
        xlo[t] = n_excl;
        return;
    }
    const int g = tile_genome(tfirst, n, t);
    tfirst[n + 2 + t] = (uint32_t)g;
    const uint64_t base = goff[g] + (uint64_t)(t - tfirst[g]) * span;
    uint32_t lo = 0, h = n_excl;
    while (lo < h) {
        const uint32_t m = (lo + h) >> 1;
        if (excl[2 * m + 1] <= base) lo = m + 1;
        else h = m;
    }
    xlo[t] = lo;
}

// ---- 1. emit: thread = kEB consecutive bytes of a tile; its k-1 bases
// of context come from a walk back over the bytes before it (newlines skipped; a
// break, an excluded range or the genome start ends the walk), then it rolls
// forward.  32 bytes per thread amortise the walk (up to k-1 + newline bytes).

// The keys go out through LDS: a thread's kEB keys are one row (padded by 16 bytes
// against bank conflicts), read back key by key in lane order so that every store
// instruction writes 256-512 contiguous bytes (a thread storing its own 128-256
// bytes touches 64 lines per instruction).
#ifndef KF_SPARSE_EMIT   // 1: whole rows staged, 2: half rows (half the LDS), 0: direct stores
#define KF_SPARSE_EMIT 2
#endif
template <typename KeyT>
struct EmitStage {
    static constexpr int keys = KF_SPARSE_EMIT == 2 ? kEB / 2 : kEB;   // keys per row per round
    static constexpr int row = keys + 16 / (int)sizeof(KeyT);          // padded row
    static constexpr int elems = KF_SPARSE_EMIT == 0 ? 1 : TileOf<KeyT>::emit_threads * row;
};

// One thread's keys (out[] holds SENT on entry): the windows ending in the kEB
// bytes at p0 = ts.base + threadIdx.x * kEB.
template <typename KeyT>
__device__ __forceinline__ void emit_row(const uint8_t* __restrict__ bytes, const TileSpan& ts, uint32_t n_excl,
                                         const uint64_t* excl, const uint32_t* xlo, int k, KeyT (&out)[kEB]) {
    const uint32_t q0 = threadIdx.x * kEB;
    if (q0 >= ts.cnt) return;
    const uint32_t p0 = ts.base + q0, cnt = min((uint32_t)kEB, ts.cnt - q0);
    using W = KeyT;   // window registers as wide as the key (2k <= 32 bits for u32 keys)
    const W kmask = (W)((1ull << (2 * k)) - 1);
    const int hi = 2 * k - 2;
    uint32_t code[kEB];
    bool any = false;
    if (cnt == (uint32_t)kEB && ((uintptr_t)(bytes + p0) & 15u) == 0) {   // two 16-byte loads
        const uint4 a = *(const uint4*)(bytes + p0), b = *(const uint4*)(bytes + p0 + 16);
        const uint32_t wv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < kEB; ++j) {
            code[j] = sp_code((uint8_t)(wv[j >> 2] >> (8 * (j & 3))));
            any |= code[j] < 4;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kEB; ++j) {
            code[j] = (uint32_t)j < cnt ? sp_code(bytes[p0 + j]) : 4u;
            any |= code[j] < 4;
        }
    }
    if (!any) return;   // no base here: no window ends in these bytes (and no walk back over a newline run)
    // first excluded range ending after p0
    uint32_t ix = 0;
    {
        // the answer lies in [xlo[t], xlo[t + 1]] (sp_tilemap_kernel)
        uint32_t lo = xlo[blockIdx.x], h = xlo[blockIdx.x + 1];
        while (lo < h) {
            const uint32_t m = (lo + h) >> 1;
            if (excl[2 * m + 1] <= p0) lo = m + 1;
            else h = m;
        }
        ix = lo;
    }
    // context: up to k-1 bases before p0 (most recent in the low pair)
    const uint64_t stop = ix > 0 ? excl[2 * ix - 1] : 0;   // end of the last excluded range before p0
    const uint64_t floor_ = max((uint64_t)ts.gs, stop);
    W back = 0;
    int m = 0;
    uint64_t q = p0;
    bool open = true;   // the walk may go on
    if (p0 >= floor_ + kEB && (p0 & 15u) == 0) {
        // the kEB bytes before p0 in two 16-byte loads (no chain of dependent
        // byte loads), walked in registers
        const uint4 a = *(const uint4*)(bytes + p0 - kEB), b = *(const uint4*)(bytes + p0 - 16);
        const uint32_t wv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = kEB - 1; j >= 0; --j) {
            const uint32_t c = sp_code((uint8_t)(wv[j >> 2] >> (8 * (j & 3))));
            if (open && m < k - 1 && c != 4) {
                if (c == 5) open = false;
                else back |= (W)c << (2 * m++);
            }
        }
        q = p0 - kEB;
    }
    for (; open && q > floor_ && m < k - 1;) {
        const uint32_t c = sp_code(bytes[--q]);
        if (c == 4) continue;
        if (c == 5) break;
        back |= (W)c << (2 * m);
        ++m;
    }
    W fw = back, rc = 0;   // fw: the m context bases, most recent lowest
    int len = m;
    for (int i = 0; i < m; ++i) rc |= (W)(3u - ((uint32_t)(back >> (2 * i)) & 3u)) << (hi - 2 * i);
    // the next excluded range's bounds (the thread's bytes rarely meet one)
    uint64_t xs = ix < n_excl ? excl[2 * ix] : ~0ull, xe = ix < n_excl ? excl[2 * ix + 1] : ~0ull;
    // one step of the window, without branches: a base rolls in, '\n' (4) is
    // transparent, anything else (5) breaks the window
    auto roll = [&](int j, uint32_t c) {
        const bool isb = c < 4u;
        const uint32_t cb = c & 3u;
        fw = isb ? (W)(((fw << 2) | cb) & kmask) : fw;
        rc = isb ? (W)((rc >> 2) | ((W)(3u - cb) << hi)) : rc;
        len = c == 5u ? 0 : len + (isb ? 1 : 0);
        out[j] = isb && len >= k ? (KeyT)(fw < rc ? fw : rc) : out[j];
    };
    if (xs >= (uint64_t)p0 + kEB) {   // no excluded byte here (bytes past cnt hold code 4)
#pragma unroll
        for (int j = 0; j < kEB; ++j) roll(j, code[j]);
        return;
    }
#pragma unroll
    for (int j = 0; j < kEB; ++j) {
        const uint32_t p = p0 + j;
        if ((uint32_t)j < cnt) {
            while (p >= xe) {
                ++ix;
                xs = ix < n_excl ? excl[2 * ix] : ~0ull;
                xe = ix < n_excl ? excl[2 * ix + 1] : ~0ull;
            }
            roll(j, p >= xs ? 5u : code[j]);
        }
    }
}

template <typename KeyT>
__global__ void __launch_bounds__(TileOf<KeyT>::emit_threads) sp_emit_kernel(const uint8_t* __restrict__ bytes, const uint64_t* goff,
                                                            const uint32_t* tfirst, int n, const uint64_t* excl,
                                                            uint32_t n_excl, const uint32_t* xlo, int k,
                                                            KeyT* __restrict__ keys) {
    using T = TileOf<KeyT>;
    using S = EmitStage<KeyT>;
    __shared__ __attribute__((aligned(16))) KeyT stage[S::elems];
    TileSpan ts;
    if (!tile_span(goff, tfirst, n, blockIdx.x, ts, T::tile)) return;   // uniform over the workgroup
    const KeyT sent = (KeyT)((1ull << (2 * k)) - 1);
    KeyT out[kEB];
#pragma unroll
    for (int j = 0; j < kEB; ++j) out[j] = sent;
    emit_row(bytes, ts, n_excl, excl, xlo, k, out);
#if KF_SPARSE_EMIT == 0
    (void)stage;
    const uint32_t q0 = threadIdx.x * kEB;
    if (q0 < ts.cnt) {
        KeyT* dst = keys + ts.base + q0;
        const uint32_t cnt = min((uint32_t)kEB, ts.cnt - q0);
        if (cnt == (uint32_t)kEB && ((uintptr_t)dst & 15u) == 0) {
#pragma unroll
            for (int j = 0; j < kEB; j += 16 / (int)sizeof(KeyT)) {
                if constexpr (sizeof(KeyT) == 8) *(ulonglong2*)(dst + j) = make_ulonglong2(out[j], out[j + 1]);
                else *(uint4*)(dst + j) = make_uint4(out[j], out[j + 1], out[j + 2], out[j + 3]);
            }
        } else {
            for (uint32_t j = 0; j < cnt; ++j) dst[j] = out[j];
        }
    }
#else
    KeyT* row = stage + threadIdx.x * S::row;
    KeyT* dst = keys + ts.base;
#pragma unroll
    for (int h = 0; h < kEB / S::keys; ++h) {
        if (h) __syncthreads();   // the previous round's reads are done
#pragma unroll
        for (int j = 0; j < S::keys; j += 16 / (int)sizeof(KeyT)) {
            const int o = h * S::keys + j;
            if constexpr (sizeof(KeyT) == 8) *(ulonglong2*)(row + j) = make_ulonglong2(out[o], out[o + 1]);
            else *(uint4*)(row + j) = make_uint4(out[o], out[o + 1], out[o + 2], out[o + 3]);
        }
        __syncthreads();
        // staged key e = (thread r, key c) is slot r * kEB + h * S::keys + c of the tile
#pragma unroll 4
        for (uint32_t e = threadIdx.x; e < (uint32_t)T::emit_threads * S::keys; e += T::emit_threads) {
            const uint32_t r = e / S::keys, c = e % S::keys, i = r * kEB + h * S::keys + c;
            if (i < ts.cnt) dst[i] = stage[r * S::row + c];
        }
    }
#endif
}

// ---- 2a. per-tile digit histogram (one row per digit: hist[d * hstride + t])
template <typename KeyT>
__global__ void __launch_bounds__(kSBlock) sp_hist_kernel(const KeyT* __restrict__ keys, const uint64_t* goff,
                                                          const uint32_t* tfirst, int n, int shift, int bits,
                                                          uint32_t* hist, uint32_t hstride) {
    using T = TileOf<KeyT>;
    __shared__ uint32_t wc[kSWaves][256];
    TileSpan ts;
    if (!tile_span(goff, tfirst, n, blockIdx.x, ts, T::tile)) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < kSWaves * 256; i += kSBlock) (&wc[0][0])[i] = 0;
    __syncthreads();
    const uint32_t dmask = (1u << bits) - 1u;
    // order does not matter here: one LDS add per key into the wave's counters
    // (the ballot matching of the scatter costs ~60 VALU per 64 keys)
    // every load first (a load per iteration, each waited for before its add,
    // left the waves at HBM latency): indices clamped to the tile's last key
    KeyT x[T::per];
#pragma unroll
    for (int it = 0; it < T::per; ++it) x[it] = keys[ts.base + min(w * T::wave_span + it * 64 + lane, ts.cnt - 1)];
#pragma unroll
    for (int it = 0; it < T::per; ++it) {
        const uint32_t li = w * T::wave_span + it * 64 + lane;
        if (li < ts.cnt) atomicAdd(&wc[w][(uint32_t)(x[it] >> shift) & dmask], 1u);
    }
    __syncthreads();
    if (tid <= (int)dmask) hist[(uint64_t)tid * hstride + blockIdx.x] = wc[0][tid] + wc[1][tid] + wc[2][tid] + wc[3][tid];
}

// ---- 2b. workgroup (g, d): exclusive scan of hist[d][tiles of g] in place;
// gtot[g * 256 + d] = the genome's count of digit d
__global__ void __launch_bounds__(kSBlock) sp_scan_kernel(uint32_t* hist, uint32_t hstride, const uint32_t* tfirst,
                                                          uint32_t* gtot) {
    __shared__ uint32_t wsum[kSWaves];
    __shared__ uint32_t tot;
    const uint32_t g = blockIdx.x, d = blockIdx.y;
    uint32_t* row = hist + (uint64_t)d * hstride;
    const uint32_t t0 = tfirst[g], t1 = tfirst[g + 1];
    uint32_t carry = 0;
    for (uint32_t base = t0; base < t1; base += kSBlock) {
        const uint32_t t = base + threadIdx.x;
        const uint32_t v = t < t1 ? row[t] : 0u;
        const uint32_t ex = block_excl_scan(v, wsum);
        if (t < t1) row[t] = carry + ex;
        if (threadIdx.x == kSBlock - 1) tot = ex + v;   // the chunk's total
        __syncthreads();
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) gtot[g * 256 + d] = carry;
}

// ---- 2c. stable scatter of one tile by digit
// ---- 2'. single-sweep passes (KF_SPARSE_LOOKBACK = 1, the default): no tile
// histogram pass and no scan.  The genome-wide digit counts of EVERY pass come
// from one read of the emitted keys (sp_ghist_kernel); inside a pass, tile t
// learns how many keys of digit d its genome's earlier tiles hold by decoupled
// look-back: it publishes its own count (AGG), adds up its predecessors' words
// back to the first inclusive prefix (INCL), then publishes its own INCL.  A
// status word is (epoch << 34 | flag << 32 | count), one 64-bit store, so count
// and flag are seen together; epoch = pass + 1 tells this pass's words from the
// last pass's (the array is cleared once per call).  Tiles are numbered in the
// order workgroups start (a ticket), so a tile only waits on tiles that are
// already running; a wait that still exceeds ~2^22 polls flags the call (bit 2
// of tfirst[n+1]: every count comes back UINT64_MAX - 1) instead of hanging.
#ifndef KF_SPARSE_LOOKBACK
#define KF_SPARSE_LOOKBACK 1
#endif
#ifndef KF_SPARSE_ABL   // profiling ablations of the scatter (tools/ builds; wrong order by design)
#define KF_SPARSE_ABL 0
#endif
#ifndef KF_SPARSE_LBW   // predecessors read per look-back round trip
#define KF_SPARSE_LBW 1   // 4 and 8 measured the same with the interleaved order (v39)
#endif
constexpr uint64_t kStAgg = 1, kStIncl = 2;

__device__ __forceinline__ void st_publish(uint64_t* w, uint32_t epoch, uint64_t flag, uint32_t v) {
    __hip_atomic_store(w, ((uint64_t)epoch << 34) | (flag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t lookback(uint64_t* status, uint32_t* tfirst, int n, uint32_t t, uint32_t t0,
                                             uint32_t d, uint32_t tot, uint32_t epoch) {
    uint64_t* mine = status + (uint64_t)t * 256 + d;
    if (t == t0) {   // the genome's first tile: its prefix is its count
        st_publish(mine, epoch, kStIncl, tot);
        return 0;
    }
    st_publish(mine, epoch, kStAgg, tot);
    // KF_SPARSE_LBW predecessors per round trip (a status load goes past the
    // XCD's L2: ~1-2 us), nearest first, summed up to the first inclusive word;
    // a word not yet published ends the round there and is polled again
    uint32_t before = 0;
    uint32_t spins = 0;
    uint32_t j = t - 1;   // nearest predecessor not yet added (>= t0)
    for (;;) {
        uint64_t w[KF_SPARSE_LBW];
#pragma unroll
        for (int q = 0; q < KF_SPARSE_LBW; ++q)
            w[q] = __hip_atomic_load(status + (uint64_t)(j >= t0 + (uint32_t)q ? j - (uint32_t)q : t0) * 256 + d, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        bool done = false, stalled = false;
#pragma unroll
        for (int q = 0; q < KF_SPARSE_LBW; ++q) {
            if (done || stalled) continue;
            if ((uint32_t)(w[q] >> 34) != epoch) {   // not published yet
                stalled = true;
                continue;
            }
            before += (uint32_t)w[q];
            if (((w[q] >> 32) & 3u) == kStIncl || j == t0) done = true;
            else --j;
        }
        if (done) break;
        if (stalled) {
            if (++spins > (1u << 22)) {
                atomicOr(&tfirst[n + 1], 2u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    st_publish(mine, epoch, kStIncl, before + tot);
    return before;
}

// gall[(p * n + g) * 256 + d] += keys of genome g with digit d in pass p.
// Workgroup (g, c) takes the c-th of gridDim.y slices of genome g.
template <typename KeyT>
__global__ void __launch_bounds__(kSBlock) sp_ghist_kernel(const KeyT* __restrict__ keys, const uint64_t* goff,
                                                           const uint32_t* tfirst, int n, int passes, int bits,
                                                           uint32_t* gall) {
    __shared__ uint32_t cnt[8][256];
    if (tfirst[n + 1] & 1u) return;   // invalid goff (sp_tiles_kernel): nothing is counted
    const int g = blockIdx.x;
    const uint32_t gs = (uint32_t)goff[g], len = (uint32_t)goff[g + 1] - gs;
    const uint32_t part = (len + gridDim.y - 1) / gridDim.y;
    const uint32_t c0 = gs + min(len, blockIdx.y * part), c1 = gs + min(len, (blockIdx.y + 1) * part);
    if (c0 >= c1) return;
    for (int i = threadIdx.x; i < passes * 256; i += kSBlock) (&cnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t dmask = (1u << bits) - 1u;   // digits above bit 2k are 0
    constexpr int kB = 8;
    for (uint32_t base = c0; base < c1; base += kSBlock * kB) {
        KeyT x[kB];
#pragma unroll
        for (int j = 0; j < kB; ++j) x[j] = keys[min(base + j * kSBlock + threadIdx.x, c1 - 1)];
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            if (base + j * kSBlock + threadIdx.x < c1) {
                for (int p = 0; p < passes; ++p) atomicAdd(&cnt[p][(uint32_t)(x[j] >> (p * bits)) & dmask], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < passes * 256; i += kSBlock) {
        const uint32_t v = (&cnt[0][0])[i];
        if (v) atomicAdd(&gall[((uint64_t)(i >> 8) * n + g) * 256 + (i & 255)], v);
    }
}

// Ticket -> tile for the single-sweep passes: tiles ordered by (index inside
// the genome, genome), so the tiles running at once spread over the genomes'
// independent look-back chains instead of queueing on one genome's chain.
// Inside a genome the order is kept (what the look-back's progress needs).
// O(n) per tile: used up to KF_SPARSE_ORDER_MAXN genomes (identity above).
#ifndef KF_SPARSE_ORDER_MAXN
#define KF_SPARSE_ORDER_MAXN 4096
#endif
__global__ void __launch_bounds__(kSBlock) sp_order_kernel(const uint32_t* tfirst, int n, uint32_t* order) {
    const uint32_t t = blockIdx.x * kSBlock + threadIdx.x;
    if (t >= tfirst[n]) return;
    const int g = (int)tfirst[n + 2 + t];
    const uint32_t r = t - tfirst[g];
    uint32_t pos = 0;
    for (int h = 0; h < n; ++h) {
        const uint32_t nt = tfirst[h + 1] - tfirst[h];
        pos += min(nt, r) + (h < g && nt > r ? 1u : 0u);
    }
    order[pos] = t;
}

template <typename KeyT, bool LB>
__global__ void __launch_bounds__(kSBlock) sp_scatter_kernel(const KeyT* __restrict__ in, KeyT* __restrict__ out,
                                                             const uint64_t* goff, uint32_t* tfirst, int n,
                                                             int shift, int bits, const uint32_t* hist,
                                                             uint32_t hstride, const uint32_t* gtot,
                                                             uint64_t* status, uint32_t* ticket, uint32_t epoch,
                                                             const uint32_t* order) {
    using T = TileOf<KeyT>;
    __shared__ uint32_t wc[kSWaves][256];   // per wave: digit counts, then the wave's base inside the digit
    __shared__ uint32_t lbase[256];         // tile-local start of each digit
    __shared__ uint32_t gdst[256];          // global slot of the digit's first key in this tile, minus lbase
    __shared__ uint32_t wsum[kSWaves];
    __shared__ uint32_t tix;
    extern __shared__ __attribute__((aligned(16))) uint8_t sp_dyn[];
    KeyT* stage = (KeyT*)sp_dyn;   // T::tile keys (dynamic LDS: 32 KiB)
    uint32_t t = blockIdx.x;
    if constexpr (LB) {   // tiles in the order workgroups start: a tile only waits on started tiles
        if (threadIdx.x == 0) {
            const uint32_t x = atomicAdd(ticket, 1u);
            tix = order && x < tfirst[n] ? order[x] : x;
        }
        __syncthreads();
        t = tix;
    }
    TileSpan ts;
    if (!tile_span(goff, tfirst, n, t, ts, T::tile)) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < kSWaves * 256; i += kSBlock) (&wc[0][0])[i] = 0;
    __syncthreads();
    const uint32_t dmask = (1u << bits) - 1u;
    const uint64_t lt = (1ull << lane) - 1;
    KeyT key[T::per];
    uint32_t rank[T::per];
#pragma unroll
    for (int it = 0; it < T::per; ++it) key[it] = in[ts.base + min(w * T::wave_span + it * 64 + lane, ts.cnt - 1)];
#pragma unroll
    for (int it = 0; it < T::per; ++it) {
        const uint32_t li = w * T::wave_span + it * 64 + lane;
        const bool v = li < ts.cnt;
        const KeyT x = key[it];
        const uint32_t d = (uint32_t)(x >> shift) & dmask;
#if KF_SPARSE_RANK == 0
        const uint64_t m = match_digit(d, bits, __ballot(v));
        const uint32_t r = (uint32_t)__popcll(m & lt);
        const uint32_t prior = wc[w][d];
        if (v && r == 0) wc[w][d] = prior + (uint32_t)__popcll(m);
        rank[it] = prior + r;
#else
        (void)lt;
#if KF_SPARSE_ABL == 3   // profiling only: no rank atomics
        rank[it] = 0u;
        if (v && lane == 0) wc[w][d] += 64u;
#else
        rank[it] = v ? atomicAdd(&wc[w][d], 1u) : 0u;
#endif
#endif
    }
    __syncthreads();
    {
        const int d = tid;   // one digit per thread (bits <= 8)
        const uint32_t c0 = wc[0][d], c1 = wc[1][d], c2 = wc[2][d], c3 = wc[3][d];
        const bool live = d <= (int)dmask;
        const uint32_t tot = c0 + c1 + c2 + c3;
        const uint32_t gt = live ? gtot[ts.g * 256 + d] : 0u;
        uint32_t before;   // keys of digit d in the genome's earlier tiles
        if constexpr (LB) {
#if KF_SPARSE_ABL == 1   // profiling only (wrong order): no look-back
            before = 0u;
            (void)status;
            (void)epoch;
#else
            before = live ? lookback(status, tfirst, n, t, tfirst[ts.g], d, tot, epoch) : 0u;
#endif
        } else {
            before = live ? hist[(uint64_t)d * hstride + t] : 0u;
        }
        const uint32_t lb = block_excl_scan(tot, wsum);
        const uint32_t gb = block_excl_scan(gt, wsum);
        wc[0][d] = 0;
        wc[1][d] = c0;
        wc[2][d] = c0 + c1;
        wc[3][d] = c0 + c1 + c2;
        lbase[d] = lb;
        gdst[d] = live ? ts.gs + gb + before - lb : 0u;
    }
    __syncthreads();
    for (int it = 0; it < T::per; ++it) {
        const uint32_t li = w * T::wave_span + it * 64 + lane;
        if (li < ts.cnt) {
            const uint32_t d = (uint32_t)(key[it] >> shift) & dmask;
            stage[lbase[d] + wc[w][d] + rank[it]] = key[it];
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < ts.cnt; i += kSBlock) {
        const KeyT x = stage[i];
#if KF_SPARSE_ABL == 2   // profiling only: no global stores (one per tile)
        if (i == 0)
#endif
        out[gdst[(uint32_t)(x >> shift) & dmask] + i] = x;
    }
}

// The key before slot li of the wave-span layout (li = w * wave_span + it * 64 +
// lane): lane - 1 of the same load, lane 63 of the previous one, or for the
// wave's first slot one extra (wave-uniform) load -- one key load per slot
// instead of two.
template <typename KeyT>
__device__ __forceinline__ KeyT wave_shfl(KeyT v, int src, bool up) {
    if constexpr (sizeof(KeyT) == 8) {
        const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
        const uint32_t l = (uint32_t)(up ? __shfl_up((int)lo, 1, 64) : __shfl((int)lo, src, 64));
        const uint32_t h = (uint32_t)(up ? __shfl_up((int)hi, 1, 64) : __shfl((int)hi, src, 64));
        return ((KeyT)h << 32) | l;
    } else {
        return (KeyT)(up ? __shfl_up((int)v, 1, 64) : __shfl((int)v, src, 64));
    }
}

// every key of the lane first; returns the key before the wave's first slot
template <typename KeyT>
__device__ __forceinline__ KeyT load_keys(const KeyT* __restrict__ keys, const TileSpan& ts, int w, int lane,
                                          KeyT (&x)[TileOf<KeyT>::per]) {
    using T = TileOf<KeyT>;
#pragma unroll
    for (int it = 0; it < T::per; ++it) x[it] = keys[ts.base + min(w * T::wave_span + it * 64 + lane, ts.cnt - 1)];
    const uint32_t p0 = ts.base + min(w * T::wave_span, ts.cnt - 1);
    return keys[max(p0, ts.gs + 1) - 1];   // unused when p0 == gs (a head)
}

template <typename KeyT>
__device__ __forceinline__ KeyT prev_key(const KeyT (&x)[TileOf<KeyT>::per], int it, int lane, KeyT first_prev) {
    const KeyT up = wave_shfl(x[it], 0, true);
    const KeyT last = it ? wave_shfl(x[it > 0 ? it - 1 : 0], 63, false) : first_prev;
    return lane ? up : last;
}

// ---- 3a. run heads per tile (into hist row 0)
template <typename KeyT>
__global__ void __launch_bounds__(kSBlock) sp_heads_kernel(const KeyT* __restrict__ keys, const uint64_t* goff,
                                                           uint32_t* tfirst, int n, uint32_t* heads) {
    using T = TileOf<KeyT>;
    __shared__ uint32_t wsum[kSWaves];
    TileSpan ts;
    if (!tile_span(goff, tfirst, n, blockIdx.x, ts, T::tile)) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // every load first (slot and predecessor; indices clamped into the tile / genome)
    KeyT x[T::per];
    const KeyT fp = load_keys(keys, ts, w, lane, x);
    uint32_t c = 0;
    bool disorder = false;
#pragma unroll
    for (int it = 0; it < T::per; ++it) {
        const uint32_t li = w * T::wave_span + it * 64 + lane, p = ts.base + li;
        const KeyT y = prev_key(x, it, lane, fp);
        if (li < ts.cnt) {
            c += p == ts.gs || x[it] != y ? 1u : 0u;
            disorder |= p > ts.gs && x[it] < y;
        }
    }
    if (__ballot(disorder) && (threadIdx.x & 63) == 0) atomicOr(&tfirst[n + 1], 2u);   // the sort's self-check
    for (int d = 32; d >= 1; d >>= 1) c += (uint32_t)__shfl_xor((int)c, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) heads[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// ---- 3b. heads -> unique keys and their first slots (genome-relative)
template <typename KeyT>
__global__ void __launch_bounds__(kSBlock) sp_unique_kernel(const KeyT* __restrict__ keys, const uint64_t* goff,
                                                            const uint32_t* tfirst, int n, const uint32_t* heads,
                                                            uint64_t* __restrict__ ukeys, uint32_t* __restrict__ upos) {
    using T = TileOf<KeyT>;
    __shared__ uint32_t wsum[kSWaves];
    TileSpan ts;
    if (!tile_span(goff, tfirst, n, blockIdx.x, ts, T::tile)) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t lt = (1ull << lane) - 1;
    static_assert(T::per <= 64, "head flags: one bit per slot of the lane");
    uint64_t hm = 0;   // head flags of this lane's slots
    uint32_t mine = 0;
    KeyT x[T::per];
    {
        const KeyT fp = load_keys(keys, ts, w, lane, x);
#pragma unroll
        for (int it = 0; it < T::per; ++it) {
            const uint32_t li = w * T::wave_span + it * 64 + lane, p = ts.base + li;
            const KeyT y = prev_key(x, it, lane, fp);
            const bool h = li < ts.cnt && (p == ts.gs || x[it] != y);
            hm |= (h ? 1ull : 0ull) << it;
            mine += (uint32_t)__popcll(__ballot(h));
        }
    }
    if (lane == 0) wsum[w] = mine;
    __syncthreads();
    uint32_t u = heads[blockIdx.x];
    for (int x = 0; x < w; ++x) u += wsum[x];
#pragma unroll
    for (int it = 0; it < T::per; ++it) {
        const bool h = (hm >> it) & 1u;
        const uint64_t b = __ballot(h);
        if (h) {
            const uint32_t li = w * T::wave_span + it * 64 + lane;
            const uint32_t j = u + (uint32_t)__popcll(b & lt);
            ukeys[ts.gs + j] = (uint64_t)x[it];
            upos[ts.gs + j] = ts.base + li - ts.gs;
        }
        u += (uint32_t)__popcll(b);
    }
}

// ---- 3c. counts = distance to the next head; tiles index unique slots here
template <uint32_t Span>
__global__ void __launch_bounds__(kSBlock) sp_counts_kernel(const uint64_t* goff, const uint32_t* tfirst, int n,
                                                            const uint32_t* nfull, const uint32_t* upos,
                                                            uint32_t* __restrict__ counts) {
    constexpr int per = Span / kSBlock;
    TileSpan ts;
    if (!tile_span(goff, tfirst, n, blockIdx.x, ts, Span)) return;
    const uint32_t nf = nfull[ts.g * 256];
    const uint32_t len = ts.ge - ts.gs;
    const uint32_t u0 = ts.base - ts.gs;   // the tile's first unique index
    if (u0 >= nf) return;
    const uint32_t* up = upos + ts.gs;
    uint32_t a[per], b[per];
#pragma unroll
    for (int it = 0; it < per; ++it) {   // every load first (indices clamped below nf)
        const uint32_t u = min(u0 + it * kSBlock + threadIdx.x, nf - 1);
        a[it] = up[u];
        b[it] = up[min(u + 1, nf - 1)];
    }
#pragma unroll
    for (int it = 0; it < per; ++it) {
        const uint32_t i = it * kSBlock + threadIdx.x, u = u0 + i;
        if (i < ts.cnt && u < nf) counts[ts.gs + u] = (u + 1 < nf ? b[it] : len) - a[it];
    }
}

// ---- 3d. distinct k-mers per genome (SENT dropped)
template <typename KeyT>
__global__ void __launch_bounds__(256) sp_nuniq_kernel(const KeyT* keys, const uint64_t* goff, int n,
                                                       const uint32_t* nfull, const uint32_t* tfirst, KeyT sent,
                                                       uint64_t* nuniq) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    if (tfirst[n + 1] & 1u) {   // invalid goff (sp_tiles_kernel): nothing was counted
        nuniq[g] = ~0ull;
        return;
    }
    if (tfirst[n + 1] & 2u) {   // the final order check failed (sp_heads_kernel)
        nuniq[g] = ~1ull;
        return;
    }
    uint32_t nf = nfull[g * 256];
    const uint64_t ge = goff[g + 1];
    if (nf > 0 && keys[ge - 1] == sent) --nf;
    nuniq[g] = nf;
}

// Workspace carve-up (byte offsets, 256-aligned).
struct SpLayout {
    uint64_t tfirst, xlo, keys, hist, gtot, upos, gall, ticket, order, total;   // hist doubles as the look-back status
    uint32_t hstride;
};

uint64_t al256(uint64_t x) { return (x + 255) & ~255ull; }

SpLayout sp_layout(int k, uint64_t batch_bytes, int32_t n) {
    SpLayout L;
    const uint64_t ks = k <= 16 ? 4 : 8;
    L.hstride = (uint32_t)(batch_bytes / tile_for_k(k) + (uint64_t)n + 1);
    uint64_t o = 0;
    L.tfirst = o;   // tfirst[0..n], the flags word, then the tile -> genome map
    o = al256(o + 4ull * ((uint64_t)n + 2 + L.hstride));
    L.xlo = o;
    o = al256(o + 4ull * ((uint64_t)L.hstride + 1));
    L.keys = o;
    o = al256(o + ks * batch_bytes);
    L.hist = o;
    o = al256(o + (KF_SPARSE_LOOKBACK ? 8ull : 4ull) * 256 * L.hstride);
    L.gtot = o;
    o = al256(o + 4ull * 256 * (uint64_t)n);
    L.upos = o;
    o = al256(o + 4ull * batch_bytes);
    L.gall = o;   // passes x n x 256 genome digit counts (look-back)
    o = al256(o + 4ull * 8 * 256 * (uint64_t)n);
    L.ticket = o;   // a tile counter per pass
    o = al256(o + 4ull * 8);
    L.order = o;    // ticket -> tile
    o = al256(o + 4ull * L.hstride);
    L.total = o;
    return L;
}

template <typename KeyT>
int sp_prepare() {   // the scatter's staging tile is dynamic LDS (64 KiB for u64 keys)
    static bool done = false;
    if (done) return KF_OK;
    if (hipFuncSetAttribute((const void*)&sp_scatter_kernel<KeyT, KF_SPARSE_LOOKBACK != 0>,
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(TileOf<KeyT>::tile * sizeof(KeyT))) != hipSuccess)
        return kf_fail(KF_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    done = true;
    return KF_OK;
}

template <typename KeyT>
int sp_run(const uint8_t* d_bytes, const uint64_t* d_goff, int32_t n, uint64_t batch_bytes, const uint64_t* d_excl,
           uint64_t n_excl, int k, uint8_t* work, const SpLayout& L, uint64_t* d_keys, uint32_t* d_counts,
           uint64_t* d_nuniq, hipStream_t s) {
    if (const int rc = sp_prepare<KeyT>()) return rc;
    uint32_t* tfirst = (uint32_t*)(work + L.tfirst);
    KeyT* kw = (KeyT*)(work + L.keys);     // the sorted keys end here
    KeyT* ka = (KeyT*)d_keys;              // d_keys doubles as the other sort buffer
    uint32_t* hist = (uint32_t*)(work + L.hist);
    uint32_t* gtot = (uint32_t*)(work + L.gtot);
    uint32_t* upos = (uint32_t*)(work + L.upos);
    const uint32_t grid = L.hstride;       // >= the batch's tile count
    const int bits_total = 2 * k;
    const int passes = (bits_total + 7) / 8;
    const int bits = (bits_total + passes - 1) / passes;
    hipLaunchKernelGGL(sp_tiles_kernel, dim3(1), dim3(1024), 0, s, d_goff, n, batch_bytes, TileOf<KeyT>::tile, tfirst);
    uint32_t* xlo = (uint32_t*)(work + L.xlo);
    hipLaunchKernelGGL(sp_tilemap_kernel, dim3(grid / 256 + 1), dim3(256), 0, s, d_goff, tfirst, n, d_excl,
                       (uint32_t)n_excl, TileOf<KeyT>::tile, xlo);
    // the last pass must write kw: start in kw for an even number of passes
    KeyT* src = (passes % 2 == 0) ? kw : ka;
    KeyT* dst = (passes % 2 == 0) ? ka : kw;
    hipLaunchKernelGGL(sp_emit_kernel<KeyT>, dim3(grid), dim3(TileOf<KeyT>::emit_threads), 0, s, d_bytes, d_goff, tfirst, n, d_excl,
                       (uint32_t)n_excl, xlo, k, src);
#if KF_SPARSE_LOOKBACK
    uint64_t* status = (uint64_t*)(work + L.hist);
    uint32_t* gall = (uint32_t*)(work + L.gall);
    uint32_t* ticket = (uint32_t*)(work + L.ticket);
    if (hipMemsetAsync(status, 0, 8ull * 256 * L.hstride, s) != hipSuccess ||
        hipMemsetAsync(gall, 0, L.order - L.gall, s) != hipSuccess)   // gall and the tickets
        return kf_fail(KF_EHIP, "memset failed");
    const uint32_t slices = (uint32_t)max(1, min(1024, 4096 / max(1, (int)n)));
    hipLaunchKernelGGL(sp_ghist_kernel<KeyT>, dim3((uint32_t)n, slices), dim3(kSBlock), 0, s, src, d_goff, tfirst, n,
                       passes, bits, gall);
    uint32_t* order = nullptr;
    if (n > 1 && n <= KF_SPARSE_ORDER_MAXN) {
        order = (uint32_t*)(work + L.order);
        hipLaunchKernelGGL(sp_order_kernel, dim3((grid + kSBlock - 1) / kSBlock), dim3(kSBlock), 0, s, tfirst, n, order);
    }
#endif
    for (int p = 0; p < passes; ++p) {
        const int shift = p * bits;
        const int b = min(bits, bits_total - shift);
#if KF_SPARSE_LOOKBACK
        hipLaunchKernelGGL((sp_scatter_kernel<KeyT, true>), dim3(grid), dim3(kSBlock), TileOf<KeyT>::tile * sizeof(KeyT),
                           s, src, dst, d_goff, tfirst, n, shift, b, nullptr, L.hstride,
                           gall + (uint64_t)p * n * 256, status, ticket + p, (uint32_t)p + 1, order);
#else
        hipLaunchKernelGGL(sp_hist_kernel<KeyT>, dim3(grid), dim3(kSBlock), 0, s, src, d_goff, tfirst, n, shift, b,
                           hist, L.hstride);
        hipLaunchKernelGGL(sp_scan_kernel, dim3((uint32_t)n, 1u << b), dim3(kSBlock), 0, s, hist, L.hstride, tfirst,
                           gtot);
        hipLaunchKernelGGL((sp_scatter_kernel<KeyT, false>), dim3(grid), dim3(kSBlock), TileOf<KeyT>::tile * sizeof(KeyT),
                           s, src, dst, d_goff, tfirst, n, shift, b, hist, L.hstride, gtot, nullptr, nullptr, 0u,
                           nullptr);
#endif
        KeyT* t = src;
        src = dst;
        dst = t;
    }
    // src == kw: sorted
    hipLaunchKernelGGL(sp_heads_kernel<KeyT>, dim3(grid), dim3(kSBlock), 0, s, kw, d_goff, tfirst, n, hist);
    hipLaunchKernelGGL(sp_scan_kernel, dim3((uint32_t)n, 1), dim3(kSBlock), 0, s, hist, L.hstride, tfirst, gtot);
    hipLaunchKernelGGL(sp_unique_kernel<KeyT>, dim3(grid), dim3(kSBlock), 0, s, kw, d_goff, tfirst, n, hist, d_keys,
                       upos);
    hipLaunchKernelGGL(sp_counts_kernel<TileOf<KeyT>::tile>, dim3(grid), dim3(kSBlock), 0, s, d_goff, tfirst, n, gtot,
                       upos, d_counts);
    const KeyT sent = (KeyT)((1ull << (2 * k)) - 1);
    hipLaunchKernelGGL(sp_nuniq_kernel<KeyT>, dim3((n + 255) / 256), dim3(256), 0, s, kw, d_goff, n, gtot, tfirst, sent,
                       d_nuniq);
    return KF_OK;
}

}  // namespace
}  // namespace kf

using namespace kf;

extern "C" uint64_t kf_sparse_workspace_bytes(int k, uint64_t batch_bytes, int32_t n_genomes) {
    if (k < 2 || k > KF_SPARSE_MAX_K || n_genomes < 0) return 0;
    return sp_layout(k, batch_bytes, n_genomes).total;
}

extern "C" int kf_sparse_count(const uint8_t* d_bytes, const uint64_t* d_goff, int32_t n_genomes,
                               uint64_t batch_bytes, const uint64_t* d_excl, uint64_t n_excl, int k, void* d_work,
                               uint64_t work_bytes, uint64_t* d_keys, uint32_t* d_counts, uint64_t* d_nuniq,
                               void* stream) {
    if (k < 2 || k > KF_SPARSE_MAX_K) return kf_fail(KF_EINVAL, "k=%d out of range [2, %d]", k, KF_SPARSE_MAX_K);
    if (n_genomes < 0) return kf_fail(KF_EINVAL, "n_genomes < 0");
    if (n_genomes == 0) return KF_OK;
    if (batch_bytes >= (1ull << 32))
        return kf_fail(KF_EINVAL, "batch of %llu bytes: at most 4 GiB - 1 per call", (unsigned long long)batch_bytes);
    if (n_excl >= (1ull << 31)) return kf_fail(KF_EINVAL, "too many excluded ranges");
    if (!d_bytes || !d_goff || (n_excl && !d_excl) || !d_work || !d_keys || !d_counts || !d_nuniq)
        return kf_fail(KF_EINVAL, "null device pointer");
    if ((uintptr_t)d_bytes & 15u)   // as kf_count_batch: the emit's 16-byte loads assume it
        return kf_fail(KF_EINVAL, "d_bytes must be 16-byte aligned");
    const SpLayout L = sp_layout(k, batch_bytes, n_genomes);
    if (work_bytes < L.total)
        return kf_fail(KF_ERANGE, "workspace needs %llu bytes (kf_sparse_workspace_bytes)",
                       (unsigned long long)L.total);
    hipStream_t s = (hipStream_t)stream;
    const int rc = k <= 16 ? sp_run<uint32_t>(d_bytes, d_goff, n_genomes, batch_bytes, d_excl, n_excl, k,
                                              (uint8_t*)d_work, L, d_keys, d_counts, d_nuniq, s)
                           : sp_run<uint64_t>(d_bytes, d_goff, n_genomes, batch_bytes, d_excl, n_excl, k,
                                              (uint8_t*)d_work, L, d_keys, d_counts, d_nuniq, s);
    if (rc != KF_OK) return rc;
    if (hipGetLastError() != hipSuccess) return kf_fail(KF_EHIP, "sparse count launch failed");
    return KF_OK;
}
