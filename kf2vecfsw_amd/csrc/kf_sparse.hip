// kf_sparse.hip -- `get_kmers` at any k = 2..31 (reference kf2vec/main.py:112-176)
// for MI355X (gfx950).
//
// The reference runs `jellyfish count -m K -C` + `jellyfish dump -c -t` per genome
// and keeps the PRESENT canonical k-mers only (main.py:133-160); its parser
// accepts k = 2..31 (main.py:81-82, 1006).  A dense 4^k/2-bin row stops being
// possible past k ~ 13 (k = 31: 2^61 bins), so this path sorts instead of
// histogramming.  Round 5: one most-significant-digit split in HBM, then the
// sort of each bucket group inside one CU's LDS (rounds 4's form was an LSD
// radix sort of 2k bits with one HBM read + write of every key per 8-bit digit,
// 8 passes at k = 31):
//   A. count    every window's canonical key (standard 2-bit code A0 C1 G2 T3,
//               canonical = the smaller of the code and its reverse complement,
//               i.e. the lexicographically smaller string) is computed from the
//               input bytes and counted by its top D <= 10 bits (its bucket) per
//               genome; nothing is written but the genome x bucket totals;
//   B. scatter  the keys are computed again (the input is 1 B per key, a key 4-8 B)
//               and written bucket by bucket: per tile of 16,384 bytes, ranks by
//               LDS atomics, each bucket's place among the genome's earlier tiles
//               by decoupled look-back, the tile re-ordered in LDS so every
//               bucket's keys leave as one run;
//   C. chunks   consecutive buckets of a genome are grouped into chunks of at most
//               C keys (128 KiB of LDS); one workgroup loads a chunk, sorts it in
//               LDS (LSD passes of 8 bits over the bits below the chunk's first
//               bucket), run-length encodes it, learns how many distinct k-mers
//               the genome's earlier chunks hold (look-back) and writes its
//               (key, count) pairs in place.  A bucket with more than C keys
//               (low-complexity sequence: poly-A puts a genome's every window in
//               one bucket) is copied to an overflow area, sorted there by the
//               round-4 LSD passes (single sweep, look-back) and run-length
//               encoded by one workgroup streaming it.
// Keys are u32 for k <= 16 and u64 above.  Windows that end nowhere (no base,
// a break) produce no key (round 4 sorted a sentinel per byte).
//
// Semantics are those of the dense counter (kf_count_batch): '\n' is
// transparent, any other non-ACGT byte (either case counts) breaks the window,
// the excluded byte ranges (headers, FASTQ '+' / quality lines, from
// kf_index_records) break it too, and a window never spans two genomes.
//
// Layout: genome g owns slots [goff[g], goff[g+1]) of every key buffer (a genome
// has at most as many windows as bytes); its bucketed keys fill the first
// gkeys[g] of them, bucket b from gbase[g][b].
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <cstdio>

#include "kf_internal.h"

namespace kf {
namespace {

constexpr int kSBlock = 256;                   // LSD (overflow) kernels: threads per workgroup
constexpr int kSWaves = kSBlock / 64;
constexpr int kEB = 32;                        // emit: bytes per thread
// LSD tiles (the overflow sort): 16384 u32 keys or 8192 u64 keys (the scatter
// stages 64 KiB; profiles/r04/v49_*, v51_*).
template <typename KeyT>
struct TileOf {
    static constexpr uint32_t tile = sizeof(KeyT) == 4 ? 16384u : 8192u;
    static constexpr int per = tile / kSBlock;             // slots per thread
    static constexpr uint32_t wave_span = tile / kSWaves;  // slots per wave
};

// Phase A / B tiles: 16,384 input bytes, 512 threads x kEB bytes.
constexpr uint32_t kTB = 16384;
constexpr int kBBlock = (int)kTB / kEB;        // 512
constexpr int kBWaves = kBBlock / 64;          // 8
// Buckets: the top D bits of a 2k-bit key, D = min(10, 2k).
constexpr int kBD = 10;
constexpr uint32_t kNB = 1u << kBD;
__host__ __device__ constexpr int sp_dbits(int k) { return 2 * k < kBD ? 2 * k : kBD; }
// Phase C: chunks of at most 32 keys per thread (16,384 at 512 threads: 128 KiB
// of LDS for u64 keys), up to 256 VGPRs per thread (1024 threads spilled at 128).
// tools/ A/B builds: KF_SP_CBLOCK = 256, 8,192-key chunks, two workgroups per CU;
// KF_SP_CBLOCK = 768 with KF_SP_CPER = 16 keys per thread, 12,288-key chunks
// and 12 waves per CU.
#ifndef KF_SP_CBLOCK
#define KF_SP_CBLOCK 512
#endif
#ifndef KF_SP_CPER
#define KF_SP_CPER 32
#endif
constexpr int kCBlock = KF_SP_CBLOCK;
constexpr int kCWaves = kCBlock / 64;
constexpr uint32_t kCCap = (uint32_t)KF_SP_CPER * (uint32_t)kCBlock;
constexpr int kCPerCU = kCBlock >= 512 ? 1 : 512 / kCBlock;   // resident chunk workgroups per CU
// u32 keys (k <= 16): 24 keys per thread, 12,288-key chunks, so a chunk
// workgroup needs <= 80 KiB of LDS and two share a CU (4 waves per SIMD; the
// 128-VGPR budget spills ~140 B per lane): k = 13 5.67-5.68 ms against
// 5.84 with one 16,384-key workgroup per CU, k = 16 5.86-5.87 against 5.95
// (processes alternated, profiles/r06/v33_sparse_u32_2wg_ab.jsonl)
#ifndef KF_SP_CPER4
#define KF_SP_CPER4 24
#endif
constexpr uint32_t kNoOvf = 0xFFFFFFFFu;
// 8-bit MSD passes over the top bits of a chunk's keys before the run fix-up
// (tools/ A/B builds: KF_SP_MSD=3 sorts 24 bits, leaving almost no runs).
#ifndef KF_SP_MSD
#define KF_SP_MSD 2
#endif
// Digit width of the chunk sort's passes (KF_SP_DIGIT = 8 or 10): 10-bit MSD
// passes sort the top 20 bits, so a 16,384-key chunk over 2^20 values leaves
// runs of equal top bits for ~1.6 % of its keys instead of ~22 %, and a chunk
// whose keys span R = 2k - D + ceil(log2 buckets) <= 20 bits is sorted whole in
// the two passes (D = 10 bucket bits: k <= 15 for a one-bucket chunk, k <= 14
// for the usual two to four buckets per chunk).  64 x 5 Mbp (profiles/r05/v19_*):
// k = 31 7.69 -> 7.23 ms, k = 13 6.37 -> 5.97 (fix-up 0.69e9 -> 0.38e9 cycles,
// the passes unchanged; 16 KiB of counters per workgroup instead of 4).
// Phase A loads a workgroup's next tile's bytes while it makes this tile's keys
// (KF_SP_PREFETCH_A=0: when the tile starts).
#ifndef KF_SP_PREFETCH_A
#define KF_SP_PREFETCH_A 1
#endif
// Unroll of the chunk kernel's mask sweep and run-length stores (tools/ A/B).
#ifndef KF_SP_UNROLL_SWEEP
#define KF_SP_UNROLL_SWEEP 4
#endif
#ifndef KF_SP_UNROLL_STORES
#define KF_SP_UNROLL_STORES 4
#endif
#ifndef KF_SP_DIGIT
#define KF_SP_DIGIT 10
#endif
constexpr int kDB = KF_SP_DIGIT;
constexpr uint32_t kND = 1u << kDB;          // digits
constexpr uint32_t kNWW = kND / 2;           // packed u16 counter words per wave
template <typename KeyT>
struct ChunkOf {
    static constexpr int per = sizeof(KeyT) == 4 ? KF_SP_CPER4 : KF_SP_CPER;   // keys per thread
    static constexpr uint32_t cap = (uint32_t)per * (uint32_t)kCBlock;         // keys
    static constexpr uint32_t wave_span = cap / kCWaves;
    // LDS: the key stage, the digit counters, the head-mask prefixes, wsum, cid
    static constexpr uint32_t lds = cap * (uint32_t)sizeof(KeyT) + kCWaves * kNWW * 4 + (cap / 32) * 4 +
                                    kCWaves * 4 + 16;
    static constexpr int per_cu = kCPerCU == 1 && 2 * lds <= 160u * 1024u ? 2 : kCPerCU;
    static constexpr int waves_per_eu = (kCWaves * per_cu + 3) / 4;
};
struct Chunk {          // one LDS sort unit: buckets [blo, blo + nb) of one genome
    uint32_t start;     // first slot in the bucketed keys
    uint32_t nkeys;
    uint16_t blo, nb;
    uint32_t ovf;       // kNoOvf, or the big bucket's first slot in the overflow area
};

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

// Segment of tile t (t < tfirst[n]): the last g with tfirst[g] <= t (empty
// segments share their tfirst with the next one).
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
    uint32_t g, gs, ge, base, cnt;   // segment, its slot range, the tile's first slot and slot count
};

// tfirst[n + 2 + t] = the segment of tile t (sp_tilemap_kernel): one load
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

// Barrier for LDS traffic only: outstanding global loads and stores stay in
// flight across it (__syncthreads() is a workgroup fence too, which waits for
// every outstanding global access of the wave first).
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Inclusive prefix sum over a whole (fully active) wave on the VALU: DPP row
// shifts and row broadcasts instead of __shfl_up's six ds_bpermute round trips.
__device__ __forceinline__ uint32_t wave_incl_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

// Exclusive prefix of one value per thread over an NW-wave workgroup; *total
// (optional) gets the sum.  Contains two barriers (LDS-only ones if LDSB).
template <int NW, bool LDSB = false>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total = nullptr) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_dpp(v);
    if (lane == 63) wsum[w] = inc;
    if (LDSB) lds_sync();
    else __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int x = 0; x < NW; ++x) {
        const uint32_t s = wsum[x];
        before += x < w ? s : 0u;
        all += s;
    }
    if (total) *total = all;
    if (LDSB) lds_sync();
    else __syncthreads();
    return before + inc - v;
}

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

// ---- tile map: tfirst[n + 2 + t] = segment of tile t; xlo[t] = the first
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

// ---- keys of the windows ending in kEB bytes: thread = kEB consecutive bytes
// of tile tix (span kTB); its k-1 bases of context come from a walk back over
// the bytes before it (newlines skipped; a break, an excluded range or the
// genome start ends the walk), then it rolls forward.  32 bytes per thread
// amortise the walk (up to k-1 + newline bytes).  out[] holds SENT on entry
// (4^k - 1 = T..T, never canonical: its reverse complement A..A is smaller) and
// keeps it where no window ends.
// The bytes a thread's emit reads, loaded ahead: its kEB bytes and the kEB before
// them, four 16-byte loads at addresses clamped into the buffer (every load
// unconditional: the caller keeps them in flight while it finishes a tile).
struct EmitIn {
    uint4 a, b, c, d;
};
__device__ __forceinline__ EmitIn emit_load(const uint8_t* __restrict__ bytes, const TileSpan& ts, uint64_t nbytes) {
    EmitIn e;
    if (nbytes < 2 * kEB) {   // (uniform) a tiny batch: emit_row reads byte by byte
        e.a = e.b = e.c = e.d = make_uint4(0u, 0u, 0u, 0u);
        return e;
    }
    const uint64_t lim = (nbytes - 2 * kEB) & ~15ull;
    const uint64_t p0 = (uint64_t)ts.base + threadIdx.x * kEB;
    const uint64_t pm = min(p0, lim), pc = min(p0 >= kEB ? p0 - kEB : 0ull, lim);
    e.a = *(const uint4*)(bytes + pm);
    e.b = *(const uint4*)(bytes + pm + 16);
    e.c = *(const uint4*)(bytes + pc);
    e.d = *(const uint4*)(bytes + pc + 16);
    return e;
}

// BK (phase A): out[] gets each window's bucket (the key's top D = 2k - bshift
// bits) instead of its key: the top bits of min(code, reverse complement) are the
// min of the two top bits, so the reverse complement is kept as its top D bits
// only (one 32-bit register) and out[] is 32-bit (fewer VGPRs for u64 keys).
template <typename KeyT, bool BK = false, typename OutT = KeyT>
__device__ __forceinline__ void emit_row(const uint8_t* __restrict__ bytes, const TileSpan& ts, uint32_t tix,
                                         uint32_t n_excl, const uint64_t* excl, const uint32_t* xlo, int k,
                                         uint64_t nbytes, const EmitIn& in, OutT (&out)[kEB], int bshift = 0) {
    const uint32_t q0 = threadIdx.x * kEB;
    if (q0 >= ts.cnt) return;
    const uint32_t p0 = ts.base + q0, cnt = min((uint32_t)kEB, ts.cnt - q0);
    using W = KeyT;   // window registers as wide as the key (2k <= 32 bits for u32 keys)
    const W kmask = (W)((1ull << (2 * k)) - 1);
    const int hi = 2 * k - 2;
    uint32_t code[kEB];
    bool any = false;
    // (emit_load's clamp never moves a full, 16-byte aligned row: p0 + 2 kEB <= nbytes)
    if (cnt == (uint32_t)kEB && (p0 & 15u) == 0 && (uint64_t)p0 + 2 * kEB <= nbytes) {   // the preloaded row
        const uint4 a = in.a, b = in.b;
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
    // first excluded range ending after p0: in [xlo[tix], xlo[tix + 1]] (sp_tilemap_kernel)
    uint32_t ix = 0;
    {
        uint32_t lo = xlo[tix], h = xlo[tix + 1];
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
    if (p0 >= floor_ + kEB && (p0 & 15u) == 0 && (uint64_t)p0 - kEB <= ((nbytes - 2 * kEB) & ~15ull) &&
        nbytes >= 2 * kEB) {
        // the kEB bytes before p0, preloaded (no chain of dependent byte loads),
        // walked in registers
        const uint4 a = in.c, b = in.d;
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
    W fw = back, rc;   // fw: the m context bases, most recent lowest
    int len = m;
    {
        // rc: the context's reverse complement, most recent base's complement at
        // bits hi..hi+1: complement the m pairs, reverse the pair order of the word
        // (bit reversal, then swap the two bits of every pair), align to k pairs
        const W cm = m ? (W)(back ^ ((W)~(W)0 >> (8 * sizeof(W) - 2 * m))) : (W)0;
        W r;
        if constexpr (sizeof(W) == 8) r = (W)__builtin_bitreverse64((uint64_t)cm);
        else r = (W)__builtin_bitreverse32((uint32_t)cm);
        const W m55 = (W)0x5555555555555555ull;
        r = ((r >> 1) & m55) | ((r & m55) << 1);
        rc = r >> (8 * sizeof(W) - 2 * k);
    }
    const int dtop = 2 * k - bshift - 2;       // BK: the top pair's shift in the D-bit top
    uint32_t rtop = (uint32_t)(rc >> bshift);  // BK: the reverse complement's top D bits
    // the next excluded range's bounds (the thread's bytes rarely meet one)
    uint64_t xs = ix < n_excl ? excl[2 * ix] : ~0ull, xe = ix < n_excl ? excl[2 * ix + 1] : ~0ull;
    // one step of the window, without branches: a base rolls in, '\n' (4) is
    // transparent, anything else (5) breaks the window
    auto roll = [&](int j, uint32_t c) {
        const bool isb = c < 4u;
        const uint32_t cb = c & 3u;
        fw = isb ? (W)(((fw << 2) | cb) & kmask) : fw;
        len = c == 5u ? 0 : len + (isb ? 1 : 0);
        if constexpr (BK) {
            rtop = isb ? (rtop >> 2) | ((3u - cb) << dtop) : rtop;
            const uint32_t ft = (uint32_t)(fw >> bshift);
            out[j] = isb && len >= k ? (OutT)min(ft, rtop) : out[j];
        } else {
            rc = isb ? (W)((rc >> 2) | ((W)(3u - cb) << hi)) : rc;
            out[j] = isb && len >= k ? (OutT)(fw < rc ? fw : rc) : out[j];
        }
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

// ---- decoupled look-back (phase B per bucket, phase C per chunk, the LSD
// passes per digit).  A status word is (epoch << 34 | flag << 32 | count), one
// 64-bit store, so count and flag are seen together; epoch tells this pass's
// words from an earlier pass's (the arrays are cleared once per call).  Units
// are taken in ticket order, so a unit only waits on units already running; a
// wait that still exceeds ~2^22 polls sets bit 1 of *flags (every count then
// comes back UINT64_MAX - 1) instead of hanging.
constexpr uint64_t kStAgg = 1, kStIncl = 2;

__device__ __forceinline__ void st_publish(uint64_t* w, uint32_t epoch, uint64_t flag, uint32_t v) {
    __hip_atomic_store(w, ((uint64_t)epoch << 34) | (flag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Unit t's exclusive prefix of one counter (unit u's word at status[u * stride]),
// its chain starting at unit t0; publishes t's inclusive prefix.
__device__ __forceinline__ uint32_t lookback(uint64_t* status, uint32_t stride, uint32_t* flags, uint32_t t,
                                             uint32_t t0, uint32_t tot, uint32_t epoch) {
    uint64_t* mine = status + (uint64_t)t * stride;
    if (t == t0) {   // the chain's first unit: its prefix is its count
        st_publish(mine, epoch, kStIncl, tot);
        return 0;
    }
    st_publish(mine, epoch, kStAgg, tot);
    uint32_t before = 0, spins = 0;
    uint32_t j = t - 1;   // nearest predecessor not yet added (>= t0)
    for (;;) {
        const uint64_t w = __hip_atomic_load(status + (uint64_t)j * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(w >> 34) != epoch) {   // not published yet
            if (++spins > (1u << 22)) {
                atomicOr(flags, 2u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        before += (uint32_t)w;
        if (((w >> 32) & 3u) == kStIncl || j == t0) break;
        --j;
    }
    st_publish(mine, epoch, kStIncl, before + tot);
    return before;
}

// ---- LSD passes (the overflow sort of big buckets; round 4's sort of whole genomes)
// gall[(p * n + g) * 256 + d] += keys of segment g with digit d in pass p: bits
// [p bits, min((p + 1) bits, sbits)) of the key, the same digit the scatter of
// pass p takes (a big bucket's keys carry its bucket index above sbits, so the
// last pass's digit must stop at sbits too).
// Workgroups loop over the segments (most are empty when nothing overflows).
template <typename KeyT>
__global__ void __launch_bounds__(kSBlock) sp_ghist_kernel(const KeyT* __restrict__ keys, const uint64_t* goff,
                                                           const uint32_t* tfirst, int n, int passes, int bits,
                                                           int sbits, uint32_t* gall) {
    __shared__ uint32_t cnt[8][256];
    if (tfirst[n + 1] & 1u) return;   // invalid goff (sp_tiles_kernel): nothing is counted
    const uint32_t dmask = (1u << bits) - 1u;
    const int lshift = (passes - 1) * bits;
    const uint32_t lmask = (1u << (sbits - lshift)) - 1u;   // the last pass's digit
    for (int g = blockIdx.x; g < n; g += gridDim.x) {
        const uint32_t c0 = (uint32_t)goff[g], c1 = (uint32_t)goff[g + 1];
        if (c0 >= c1) continue;   // uniform
        for (int i = threadIdx.x; i < passes * 256; i += kSBlock) (&cnt[0][0])[i] = 0;
        __syncthreads();
        constexpr int kB = 8;
        for (uint32_t base = c0; base < c1; base += kSBlock * kB) {
            KeyT x[kB];
#pragma unroll
            for (int j = 0; j < kB; ++j) x[j] = keys[min(base + j * kSBlock + threadIdx.x, c1 - 1)];
#pragma unroll
            for (int j = 0; j < kB; ++j) {
                if (base + j * kSBlock + threadIdx.x < c1) {
                    for (int p = 0; p < passes; ++p)
                        atomicAdd(&cnt[p][(uint32_t)(x[j] >> (p * bits)) & (p + 1 < passes ? dmask : lmask)], 1u);
                }
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < passes * 256; i += kSBlock) {
            const uint32_t v = (&cnt[0][0])[i];
            if (v) atomicAdd(&gall[((uint64_t)(i >> 8) * n + g) * 256 + (i & 255)], v);
        }
        __syncthreads();
    }
}

// Ticket -> unit (tiles of the passes, tiles of phase B, chunks of phase C):
// units ordered by (index inside the segment, segment), so the units running at
// once spread over the segments' independent look-back chains instead of
// queueing on one chain.  Inside a segment the order is kept (what the
// look-back's progress needs).  O(n) per unit: used up to KF_SPARSE_ORDER_MAXN
// segments (identity above).  ufirst: prefix of units per segment, the total at
// [n], the unit -> segment map from [n + 2].
#ifndef KF_SPARSE_ORDER_MAXN
#define KF_SPARSE_ORDER_MAXN 4096
#endif
__global__ void __launch_bounds__(kSBlock) sp_order_kernel(const uint32_t* ufirst, int n, uint32_t* order) {
    const uint32_t t = blockIdx.x * kSBlock + threadIdx.x;
    if (t >= ufirst[n]) return;
    const int g = (int)ufirst[n + 2 + t];
    const uint32_t r = t - ufirst[g];
    uint32_t pos = 0;
    for (int h = 0; h < n; ++h) {
        const uint32_t nt = ufirst[h + 1] - ufirst[h];
        pos += min(nt, r) + (h < g && nt > r ? 1u : 0u);
    }
    order[pos] = t;
}

// One single-sweep LSD pass (stable scatter by one digit): a tile loads its keys,
// ranks them with one returning LDS add per key into its wave's digit counter,
// learns how many keys of each digit its segment's earlier tiles hold by
// look-back, re-orders the tile in LDS by digit and writes every digit's keys as
// one run.  Persistent: the workgroups loop over tickets (an empty overflow area
// costs one ticket per workgroup).  The ranks rely on an LDS unit serving the
// lanes of one instruction that hit the same address in lane order (ranks then
// follow the keys' order); the run-length encoding checks the final order and
// flags the call if it is broken.
template <typename KeyT>
__global__ void __launch_bounds__(kSBlock) sp_scatter_kernel(const KeyT* __restrict__ in, KeyT* __restrict__ out,
                                                             const uint64_t* goff, uint32_t* tfirst, int n,
                                                             int shift, int bits, const uint32_t* gtot,
                                                             uint64_t* status, uint32_t* ticket, uint32_t epoch,
                                                             const uint32_t* order) {
    using T = TileOf<KeyT>;
    __shared__ uint32_t wc[kSWaves][256];   // per wave: digit counts, then the wave's base inside the digit
    __shared__ uint32_t lbase[256];         // tile-local start of each digit
    __shared__ uint32_t gdst[256];          // global slot of the digit's first key in this tile, minus lbase
    __shared__ uint32_t wsum[kSWaves];
    __shared__ uint32_t tix;
    extern __shared__ __attribute__((aligned(16))) uint8_t sp_dyn[];
    KeyT* stage = (KeyT*)sp_dyn;   // T::tile keys (dynamic LDS: 64 KiB)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t dmask = (1u << bits) - 1u;
    for (;;) {
        if (tid == 0) {
            const uint32_t x = atomicAdd(ticket, 1u);
            tix = order && x < tfirst[n] ? order[x] : x;
        }
        __syncthreads();
        const uint32_t t = tix;
        TileSpan ts;
        if (!tile_span(goff, tfirst, n, t, ts, T::tile)) return;   // uniform: no tiles left
        for (int i = tid; i < kSWaves * 256; i += kSBlock) (&wc[0][0])[i] = 0;
        __syncthreads();
        KeyT key[T::per];
        uint32_t rank[T::per];
#pragma unroll
        for (int it = 0; it < T::per; ++it) key[it] = in[ts.base + min(w * T::wave_span + it * 64 + lane, ts.cnt - 1)];
#pragma unroll
        for (int it = 0; it < T::per; ++it) {
            const uint32_t li = w * T::wave_span + it * 64 + lane;
            const uint32_t d = (uint32_t)(key[it] >> shift) & dmask;
            rank[it] = li < ts.cnt ? atomicAdd(&wc[w][d], 1u) : 0u;
        }
        __syncthreads();
        {
            const int d = tid;   // one digit per thread (bits <= 8)
            const uint32_t c0 = wc[0][d], c1 = wc[1][d], c2 = wc[2][d], c3 = wc[3][d];
            const bool live = d <= (int)dmask;
            const uint32_t tot = c0 + c1 + c2 + c3;
            const uint32_t gt = live ? gtot[ts.g * 256 + d] : 0u;
            const uint32_t before =
                live ? lookback(status + (uint64_t)d, 256, &tfirst[n + 1], t, tfirst[ts.g], tot, epoch) : 0u;
            const uint32_t lb = block_excl_scan<kSWaves>(tot, wsum);
            const uint32_t gb = block_excl_scan<kSWaves>(gt, wsum);
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
            out[gdst[(uint32_t)(x >> shift) & dmask] + i] = x;
        }
        __syncthreads();   // stage, gdst and tix are reused by the next tile
    }
}

// ============================================================================
// Round-5 form: A count, B scatter by bucket, C chunk sort in LDS
// ============================================================================

// ---- A. genome x bucket totals.  Workgroup (g, y) takes every gridDim.y-th
// tile of genome g (a whole row of counts per workgroup keeps the global adds
// few: one per bucket per workgroup).
template <typename KeyT>
__global__ void __launch_bounds__(kBBlock) sp2_count_kernel(const uint8_t* __restrict__ bytes, const uint64_t* goff,
                                                            const uint32_t* tfirst, int n, const uint64_t* excl,
                                                            uint32_t n_excl, const uint32_t* xlo, int k, int bshift,
                                                            uint64_t nbytes, uint32_t* gtot) {
    __shared__ uint32_t h[kNB];
    if (tfirst[n + 1] & 1u) return;   // invalid goff: nothing is counted
    const int g = blockIdx.x;
    const uint32_t t0 = tfirst[g], t1 = tfirst[g + 1];
    if (t0 + blockIdx.y >= t1) return;   // uniform
    for (uint32_t i = threadIdx.x; i < kNB; i += kBBlock) h[i] = 0;
    __syncthreads();
    TileSpan ts;
    tile_span(goff, tfirst, n, t0 + blockIdx.y, ts, kTB);
    EmitIn in = emit_load(bytes, ts, nbytes);
    for (uint32_t t = t0 + blockIdx.y; t < t1; t += gridDim.y) {
        // this workgroup's next tile's bytes go out before this tile's keys are made
        // (KF_SP_PREFETCH_A=0, tools/ builds: loaded when the tile starts)
        TileSpan tn = ts;
        EmitIn inn = in;
        if (!KF_SP_PREFETCH_A) in = emit_load(bytes, ts, nbytes);
        if (KF_SP_PREFETCH_A && t + gridDim.y < t1) {
            tile_span(goff, tfirst, n, t + gridDim.y, tn, kTB);
            inn = emit_load(bytes, tn, nbytes);
        }
        if constexpr (sizeof(KeyT) == 8) {   // u64 keys: buckets only (146 VGPRs instead of 173)
            uint32_t out[kEB];                  // (0xFFFFFFFF: no window ends here)
#pragma unroll
            for (int j = 0; j < kEB; ++j) out[j] = 0xFFFFFFFFu;
            emit_row<KeyT, true, uint32_t>(bytes, ts, t, n_excl, excl, xlo, k, nbytes, in, out, bshift);
#pragma unroll
            for (int j = 0; j < kEB; ++j)
                if (out[j] != 0xFFFFFFFFu) atomicAdd(&h[out[j]], 1u);
        } else {                                // u32 keys: the keys themselves (fewer VGPRs so)
            const KeyT sent = (KeyT)((1ull << (2 * k)) - 1);
            KeyT out[kEB];
#pragma unroll
            for (int j = 0; j < kEB; ++j) out[j] = sent;
            emit_row<KeyT>(bytes, ts, t, n_excl, excl, xlo, k, nbytes, in, out);
#pragma unroll
            for (int j = 0; j < kEB; ++j)
                if (out[j] != sent) atomicAdd(&h[(uint32_t)(out[j] >> bshift)], 1u);
        }
        if (KF_SP_PREFETCH_A) {
            ts = tn;
            in = inn;
        } else if (t + gridDim.y < t1) {
            tile_span(goff, tfirst, n, t + gridDim.y, ts, kTB);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kNB; i += kBBlock)
        if (h[i]) atomicAdd(&gtot[(uint64_t)g * kNB + i], h[i]);
}

// ---- A'. per genome: gbase[g][b] = goff[g] + keys of buckets < b; gkeys[g] = all
__global__ void __launch_bounds__(1024) sp2_gbase_kernel(const uint64_t* goff, const uint32_t* gtot, int n,
                                                         uint32_t* gbase, uint32_t* gkeys) {
    __shared__ uint32_t wsum[16];
    const int g = blockIdx.x;
    const uint32_t v = gtot[(uint64_t)g * kNB + threadIdx.x];
    uint32_t tot;
    const uint32_t ex = block_excl_scan<16>(v, wsum, &tot);
    gbase[(uint64_t)g * kNB + threadIdx.x] = (uint32_t)goff[g] + ex;
    if (threadIdx.x == 0) gkeys[g] = tot;
}

// ---- B. scatter by bucket.  Persistent workgroups (one per CU: 128 KiB of
// staging for u64 keys) take tiles by ticket; per tile: the keys again from the
// bytes (32 per thread, in registers), ranks by packed u16 LDS adds into the
// wave's bucket counters, a tile-local scan, the look-back of each bucket over
// the genome's earlier tiles, the tile re-ordered in LDS by bucket, and every
// bucket's keys written as one run at gbase[g][b] + the earlier tiles' keys.
template <typename KeyT>
__global__ void __launch_bounds__(kBBlock) sp2_scatter_kernel(const uint8_t* __restrict__ bytes, const uint64_t* goff,
                                                              uint32_t* tfirst, int n, const uint64_t* excl,
                                                              uint32_t n_excl, const uint32_t* xlo, int k,
                                                              int bshift, uint64_t nbytes, const uint32_t* gbase, uint64_t* status,
                                                              uint32_t* ticket, const uint32_t* order,
                                                              KeyT* __restrict__ out, unsigned long long* prof) {
    __shared__ uint32_t wc[kBWaves][kNB / 2];   // per wave: packed u16 bucket counts, then the wave's base
    __shared__ uint32_t lbase[kNB];             // tile-local start of each bucket
    __shared__ uint32_t gdst[kNB];              // slot of the bucket's first key in this tile, minus lbase
    __shared__ uint32_t wsum[kBWaves];
    __shared__ uint32_t tix, nvalid;
    extern __shared__ __attribute__((aligned(16))) uint8_t sp_dyn[];
    KeyT* stage = (KeyT*)sp_dyn;   // kTB keys
    const int tid = threadIdx.x, w = tid >> 6;
    const KeyT sent = (KeyT)((1ull << (2 * k)) - 1);
    const uint32_t nbe = 1u << sp_dbits(k);
    // KF_SPARSE_PROFILE (profiling builds): thread 0's cycles per phase, summed
    // over workgroups: ticket + emit, rank, scan + look-back, stage, stores
    unsigned long long pt[5] = {0, 0, 0, 0, 0}, tmark = 0;
    auto tick = [&](int ph) {
        if (prof && tid == 0) {
            const unsigned long long tn = __builtin_amdgcn_s_memtime();
            if (ph >= 0) pt[ph] += tn - tmark;
            tmark = tn;
        }
    };
    // Tickets run one tile ahead (as the chunk kernel's): the next tile's bytes are
    // loaded as soon as this tile's keys are made, and stay in flight through its
    // ranks, look-back, re-order and stores; the ticket after that is taken then
    // and published (tix) at the tile's last barrier.
    auto take = [&](uint32_t x) -> uint32_t { return order && x < tfirst[n] ? order[x] : x; };
    if (tid == 0) tix = take(atomicAdd(ticket, 1u));
    __syncthreads();
    uint32_t t = tix;
    __syncthreads();   // every thread has t before tix changes
    TileSpan ts{0u, 0u, 0u, 0u, 0u};
    bool have = tile_span(goff, tfirst, n, t, ts, kTB);
    EmitIn in = emit_load(bytes, ts, nbytes);
    if (tid == 0 && have) tix = take(atomicAdd(ticket, 1u));
    __syncthreads();
    uint32_t tn = tix;
    for (;;) {
        tick(-1);
        if (!have) {   // uniform: no tiles left
            if (prof && tid == 0)
                for (int x = 0; x < 5; ++x) atomicAdd(&prof[x], pt[x]);
            return;
        }
        KeyT key[kEB];
#pragma unroll
        for (int j = 0; j < kEB; ++j) key[j] = sent;
        emit_row<KeyT>(bytes, ts, t, n_excl, excl, xlo, k, nbytes, in, key);
        TileSpan tsn{0u, 0u, 0u, 0u, 0u};
        const bool hn = tile_span(goff, tfirst, n, tn, tsn, kTB);
        EmitIn inn = in;
        if (hn) inn = emit_load(bytes, tsn, nbytes);
        uint32_t xt = 0;
        if (tid == 0 && hn) xt = atomicAdd(ticket, 1u);   // the tile after tn (published at the end)
        for (int i = tid; i < kBWaves * (int)kNB / 2; i += kBBlock) (&wc[0][0])[i] = 0;
        lds_sync();
        tick(0);
        uint32_t rk[kEB];
#pragma unroll
        for (int j = 0; j < kEB; ++j) {
            const uint32_t b = (uint32_t)(key[j] >> bshift), sh = (b & 1u) << 4;
            rk[j] = key[j] != sent ? (atomicAdd(&wc[w][b >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
        }
        lds_sync();
        tick(1);
        {
            // thread tid: buckets 2 tid, 2 tid + 1 (word tid of every wave's row)
            uint32_t run = 0;
#pragma unroll
            for (int x = 0; x < kBWaves; ++x) {   // packed: both halves stay below 2^16
                const uint32_t c = wc[x][tid];
                wc[x][tid] = run;
                run += c;
            }
            const uint32_t t0c = run & 0xFFFFu, t1c = run >> 16;
            uint32_t all;
            const uint32_t ex = block_excl_scan<kBWaves, true>(t0c + t1c, wsum, &all);
            const uint32_t b0 = 2u * (uint32_t)tid, b1 = b0 + 1u;
            lbase[b0] = ex;
            lbase[b1] = ex + t0c;
            const uint32_t tf = tfirst[ts.g];
            uint32_t bf0 = 0, bf1 = 0;
            if (b0 < nbe) bf0 = lookback(status + b0, kNB, &tfirst[n + 1], t, tf, t0c, 1u);
            if (b1 < nbe) bf1 = lookback(status + b1, kNB, &tfirst[n + 1], t, tf, t1c, 1u);
            gdst[b0] = b0 < nbe ? gbase[(uint64_t)ts.g * kNB + b0] + bf0 - ex : 0u;
            gdst[b1] = b1 < nbe ? gbase[(uint64_t)ts.g * kNB + b1] + bf1 - (ex + t0c) : 0u;
            if (tid == 0) nvalid = all;
        }
        lds_sync();
        tick(2);
#pragma unroll
        for (int j = 0; j < kEB; ++j) {
            if (key[j] != sent) {
                const uint32_t b = (uint32_t)(key[j] >> bshift), sh = (b & 1u) << 4;
                stage[lbase[b] + ((wc[w][b >> 1] >> sh) & 0xFFFFu) + rk[j]] = key[j];
            }
        }
        lds_sync();
        tick(3);
        const uint32_t nv = nvalid;
        for (uint32_t i = tid; i < nv; i += kBBlock) {
            const KeyT x = stage[i];
            out[gdst[(uint32_t)(x >> bshift)] + i] = x;
        }
        if (tid == 0 && hn) tix = take(xt);
        lds_sync();   // stage, gdst, tix are reused by the next tile
        tick(4);
        t = tn;
        ts = tsn;
        have = hn;
        in = inn;
        tn = tix;
    }
}

// ---- C0. chunk plan, one wave per genome.  Buckets are taken in order and
// grouped greedily into chunks of at most cap keys; a bucket of more than cap
// keys is a chunk of its own, sorted in the overflow area.  mode 0 counts
// (nch, nbig, bigkeys per genome); mode 1 writes the chunks at cfirst[g] (and
// the chunk -> genome map at cfirst[n + 2 + c]), the big chunks' overflow slots
// at seg_off[bfirst[g] + i] and their chunk ids at bigc[].
__global__ void __launch_bounds__(64) sp2_plan_kernel(const uint32_t* gtot, const uint32_t* gbase, int n, int k,
                                                      uint32_t cap, int mode, uint32_t* nch, uint32_t* nbig,
                                                      uint32_t* bigkeys, uint32_t* cfirst, const uint32_t* bfirst,
                                                      const uint32_t* obase, Chunk* chunks, uint64_t* seg_off,
                                                      uint32_t* bigc) {
    const int g = blockIdx.x, lane = threadIdx.x;
    const uint32_t nbe = 1u << sp_dbits(k);
    uint32_t nc = 0, nb = 0, bk = 0;   // chunks, big chunks, big keys so far (wave-uniform)
    uint32_t cur_lo = 0, cur_hi = 0, cur_n = 0;
    const uint32_t c0 = mode ? cfirst[g] : 0u, bf0 = mode ? bfirst[g] : 0u, ob0 = mode ? obase[g] : 0u;
    auto emit = [&](uint32_t lo, uint32_t hi, uint32_t cnt, bool big) {
        if (mode && lane == 0) {
            Chunk c;
            c.start = gbase[(uint64_t)g * kNB + lo];
            c.nkeys = cnt;
            c.blo = (uint16_t)lo;
            c.nb = (uint16_t)(hi - lo);
            c.ovf = big ? ob0 + bk : kNoOvf;
            chunks[c0 + nc] = c;
            cfirst[n + 2 + c0 + nc] = (uint32_t)g;
            if (big) {
                seg_off[bf0 + nb] = ob0 + bk;
                bigc[bf0 + nb] = c0 + nc;
            }
        }
        ++nc;
        if (big) {
            ++nb;
            bk += cnt;
        }
    };
    for (uint32_t b0 = 0; b0 < nbe; b0 += 64) {
        const uint32_t v = b0 + lane < nbe ? gtot[(uint64_t)g * kNB + b0 + lane] : 0u;
        for (int i = 0; i < 64 && b0 + i < nbe; ++i) {
            const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, i), b = b0 + i;
            if (c == 0) continue;
            if (c > cap) {
                if (cur_n) emit(cur_lo, cur_hi, cur_n, false);
                cur_n = 0;
                emit(b, b + 1, c, true);
            } else if (cur_n + c > cap) {
                emit(cur_lo, cur_hi, cur_n, false);
                cur_lo = b;
                cur_hi = b + 1;
                cur_n = c;
            } else {
                if (!cur_n) cur_lo = b;
                cur_hi = b + 1;
                cur_n += c;
            }
        }
    }
    if (cur_n) emit(cur_lo, cur_hi, cur_n, false);
    if (!mode && lane == 0) {
        nch[g] = nc;
        nbig[g] = nb;
        bigkeys[g] = bk;
    }
}

// ---- C0'. prefixes over genomes (one workgroup): cfirst (chunks; total at [n],
// [n + 1] = 0), bfirst (big chunks), obase (overflow keys); the unused overflow
// segments [big total, smax] are empty at the end of the area.
__global__ void __launch_bounds__(1024) sp2_cscan_kernel(const uint32_t* nch, const uint32_t* nbig,
                                                         const uint32_t* bigkeys, int n, uint32_t smax,
                                                         uint32_t* cfirst, uint32_t* bfirst, uint32_t* obase,
                                                         uint64_t* seg_off) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry[3];
    if (threadIdx.x < 3) carry[threadIdx.x] = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024) {
        const int g = base + (int)threadIdx.x;
        const uint32_t a = g < n ? nch[g] : 0u, b = g < n ? nbig[g] : 0u, c = g < n ? bigkeys[g] : 0u;
        uint32_t ta, tb, tc;
        const uint32_t ea = block_excl_scan<16>(a, wsum, &ta);
        const uint32_t eb = block_excl_scan<16>(b, wsum, &tb);
        const uint32_t ec = block_excl_scan<16>(c, wsum, &tc);
        if (g < n) {
            cfirst[g] = carry[0] + ea;
            bfirst[g] = carry[1] + eb;
            obase[g] = carry[2] + ec;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            carry[0] += ta;
            carry[1] += tb;
            carry[2] += tc;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        cfirst[n] = carry[0];
        cfirst[n + 1] = 0;
        bfirst[n] = carry[1];
        obase[n] = carry[2];
    }
    for (uint32_t i = carry[1] + threadIdx.x; i <= smax; i += 1024) seg_off[i] = carry[2];
}

// ---- C1. big buckets -> the overflow area (workgroups loop over the big chunks)
template <typename KeyT>
__global__ void __launch_bounds__(256) sp2_gather_kernel(const KeyT* __restrict__ kb, const Chunk* chunks,
                                                         const uint32_t* bigc, const uint32_t* bfirst, int n,
                                                         KeyT* __restrict__ ovf) {
    const uint32_t nbig = bfirst[n];
    for (uint32_t i = blockIdx.x; i < nbig; i += gridDim.x) {
        const Chunk c = chunks[bigc[i]];
        for (uint32_t j = threadIdx.x; j < c.nkeys; j += 256) ovf[c.ovf + j] = kb[c.start + j];
    }
}

__device__ __forceinline__ uint32_t ceil_log2(uint32_t x) { return x <= 1 ? 0u : 32u - (uint32_t)__builtin_clz(x - 1); }

// ---- C2. chunk sort + run-length encoding (persistent, one 512-thread
// workgroup per CU).  A chunk's keys (minus its first bucket's base: R = B +
// ceil(log2 nb) bits) are loaded striped, 32 per thread, and sorted in LDS by
// stable 10-bit passes (KF_SP_DIGIT): per pass a returning packed-u16 LDS add per
// key into its wave's digit counter (stable: an LDS unit serves one
// instruction's lanes in lane order, and keys are striped so lane, then
// iteration, then wave is slot order), every thread turns two digits' 8 counters
// into slots (a block scan over the digits), the keys go to their slots and come
// back striped.  For R > 20 only the top 20 bits are sorted that way (two
// passes): a chunk of <= 16,384 keys over 2^20 values of those bits leaves a few
// runs of keys with equal top bits, each sorted by the thread
// owning the mask word of its start (insertion sort in LDS); a run longer than
// kRun whose keys are not all equal (repeats make long runs of EQUAL keys, which
// need nothing) sends the chunk through every pass (LSD takes any order).  One
// striped sweep sets the run-start and head bits (a key unlike its predecessor)
// in LDS masks; a block scan over the head words numbers the heads; the chunk
// learns the genome's distinct k-mers before it by look-back, and every head
// writes (key, distance to the next head), consecutive lanes at consecutive
// outputs.  The next chunk's keys are loaded into the (dead) key registers as
// soon as a chunk is sorted and first used when its sort starts, so their
// latency hides behind the encoding.
template <typename KeyT>
__global__ void __launch_bounds__(kCBlock) __attribute__((amdgpu_waves_per_eu(ChunkOf<KeyT>::waves_per_eu))) sp2_chunk_kernel(const KeyT* __restrict__ kb, const KeyT* __restrict__ ovf,
                                                            const Chunk* chunks, const uint32_t* cfirst, int n,
                                                            int bshift, const uint64_t* goff, uint32_t* flags,
                                                            uint64_t* cstatus, uint32_t* ticket,
                                                            const uint32_t* order, uint64_t* __restrict__ okeys,
                                                            uint32_t* __restrict__ ocounts, uint64_t* unq,
                                                            unsigned long long* prof) {
    using CO = ChunkOf<KeyT>;
    constexpr int PER = CO::per;
    constexpr uint32_t kWords = CO::cap / 32;   // mask words of a chunk
    static_assert(kWords <= (uint32_t)kCBlock && kCWaves * kNWW >= 2 * kWords && kNWW <= (uint32_t)kCBlock,
                  "at most one mask word per thread");
    const bool word_owner = threadIdx.x < kWords;   // (threads past kWords own no mask word)
    __shared__ uint32_t wc[kCWaves][kNWW];   // packed u16 digit counters per wave; after the sort: start | head masks
    __shared__ uint32_t wpre[kWords];       // heads before each head-mask word
    __shared__ uint32_t wsum[kCWaves];
    __shared__ uint32_t cid, before_s;
    extern __shared__ __attribute__((aligned(16))) uint8_t sp_dyn[];
    KeyT* stage = (KeyT*)sp_dyn;   // cap keys
    uint32_t* hs = &wc[0][0];          // run starts (top bits differ), kWords words
    uint32_t* hh = &wc[0][0] + kWords; // heads (keys differ)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // KF_SPARSE_PROFILE (profiling builds): per-phase cycles of thread 0, added up
    // per workgroup: first pass (+ waits on the keys), second pass, masks + fix-up,
    // head count, look-back, stores
    unsigned long long pt[7] = {0, 0, 0, 0, 0, 0, 0};
    unsigned long long tmark = 0;
    auto tick = [&](int ph) {
        if (prof && tid == 0) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (ph >= 0) pt[ph] += t - tmark;
            tmark = t;
        }
    };
    const uint32_t total = cfirst[n];
    uint32_t li0 = (uint32_t)w * CO::wave_span + (uint32_t)lane;   // striped slot li0 + 64 it
    KeyT* srow = stage + li0;
    KeyT y[PER];
    uint32_t rk[PER];
    // Tickets run one chunk ahead: while chunk c is sorted, the next chunk cn's
    // descriptor and genome are already loading, its keys are loaded right after
    // the sort, and the ticket of the chunk after it is taken then and published
    // (cid) at the chunk's last barrier, so no step waits on a global round trip.
    auto take = [&](uint32_t x) -> uint32_t { return order && x < total ? order[x] : x; };
    if (tid == 0) cid = take(atomicAdd(ticket, 1u));
    __syncthreads();
    uint32_t cn = cid;          // the next chunk (>= total: none)
    uint32_t c = 0xFFFFFFFFu;   // the chunk being worked on (none in the first iteration)
    Chunk ch;
    ch.ovf = kNoOvf;
    uint32_t g = 0, c0 = 0;
    bool last = false;
    for (;;) {
        const bool have = c < total;
        // (vector loads: an LDS-only barrier waits for scalar loads, not for these)
        Chunk chn;
        chn.ovf = kNoOvf;
        uint32_t gn = 0;
        if (cn < total) {   // used after this chunk's sort
            chn = chunks[cn];
            gn = cfirst[n + 2 + cn];
        }
        uint32_t nk = 0;
        KeyT base = 0;
        if (have) {
            tick(-1);
            nk = ch.nkeys;
            base = (KeyT)ch.blo << bshift;
        }
        if (have && ch.ovf == kNoOvf) {
            // ------------------------------------------------ in-LDS sort (y loaded)
            {
                const int rem = (int)nk - (int)li0;
#pragma unroll
                for (int it = 0; it < PER; ++it)   // padding sorts last (all ones below R bits and above)
                    y[it] = it * 64 < rem ? (KeyT)(y[it] - base) : (KeyT)~(KeyT)0;
            }
            const uint32_t R = (uint32_t)bshift + ceil_log2(ch.nb);
            auto pass = [&](int sh8, bool reload) __attribute__((always_inline)) {
                for (int i = tid; i < kCWaves * (int)kNWW; i += kCBlock) (&wc[0][0])[i] = 0;
                lds_sync();
#pragma unroll
                for (int it = 0; it < PER; ++it) {
                    const uint32_t d = (uint32_t)(y[it] >> sh8) & (kND - 1u), sh = (d & 1u) << 4;
                    rk[it] = (atomicAdd(&wc[w][d >> 1], 1u << sh) >> sh) & 0xFFFFu;
                }
                lds_sync();
                {
                    // thread t: digits 2t, 2t + 1 (word t of every wave's row), all waves at
                    // once.  Every counter becomes its keys' first slot: the digit's start
                    // plus the counts of the earlier waves (packed halves: <= cap < 2^16).
                    const bool own = tid < (int)kNWW;
                    const int j = own ? tid : 0;
                    uint32_t a[kCWaves], r = 0;
#pragma unroll
                    for (int x = 0; x < kCWaves; ++x) {
                        a[x] = own ? wc[x][j] : 0u;
                        r += a[x];
                    }
                    const uint32_t d0 = r & 0xFFFFu;
                    const uint32_t ex = block_excl_scan<kCWaves, true>(d0 + (r >> 16), wsum);
                    uint32_t q = ex | ((ex + d0) << 16);
                    if (own) {
#pragma unroll
                        for (int x = 0; x < kCWaves; ++x) {
                            wc[x][j] = q;
                            q += a[x];
                        }
                    }
                }
                lds_sync();
#pragma unroll
                for (int it = 0; it < PER; ++it) {
                    const uint32_t d = (uint32_t)(y[it] >> sh8) & (kND - 1u), sh = (d & 1u) << 4;
                    stage[((wc[w][d >> 1] >> sh) & 0xFFFFu) + rk[it]] = y[it];
                }
                lds_sync();
                if (reload) {
#pragma unroll
                    for (int it = 0; it < PER; ++it) y[it] = srow[it * 64];
                }
            };
            constexpr uint32_t kRun = 32;
            for (int round = 0; round < 2; ++round) {
                const bool msd = round == 0 && R > (uint32_t)(kDB * KF_SP_MSD);
                const int lo = msd ? (int)R - kDB * KF_SP_MSD : 0;
                const int np = msd ? KF_SP_MSD : (int)((R + kDB - 1) / kDB);
                if (np == 0) {   // one key value: already sorted
#pragma unroll
                    for (int it = 0; it < PER; ++it) srow[it * 64] = y[it];
                    lds_sync();
                }
                for (int p = 0; p < np; ++p) {
                    pass(lo + kDB * p, p + 1 < np);
                    tick(p == 0 ? 0 : 1);
                }
                // one striped sweep: run starts (the top bits above `lo` differ) and heads
                // (the keys differ); the order check on the sorted bits (every key is in
                // order when lo = 0).  Consecutive lanes read consecutive slots.
                bool disorder = false;
#pragma unroll KF_SP_UNROLL_SWEEP
                for (int it = 0; it < PER; ++it) {
                    const uint32_t i = li0 + (uint32_t)it * 64;
                    const KeyT v = srow[it * 64], pv = i ? stage[i - 1] : (KeyT)0;
                    const bool in = i < nk, lead = i == 0;
                    disorder |= in && !lead && (v >> lo) < (pv >> lo);
                    const uint64_t bs = __ballot(in && (lead || (v >> lo) != (pv >> lo)));
                    const uint64_t bh = __ballot(in && (lead || v != pv));
                    if (lane == 0) {
                        hs[i >> 5] = (uint32_t)bs;
                        hs[(i >> 5) + 1] = (uint32_t)(bs >> 32);
                        hh[i >> 5] = (uint32_t)bh;
                        hh[(i >> 5) + 1] = (uint32_t)(bh >> 32);
                    }
                }
                if (__ballot(disorder) && lane == 0) atomicOr(flags, 2u | 16u);   // the sort's self-check
                lds_sync();
                if (!msd) break;
                // runs of two or more keys start where a start bit is followed by a clear
                // one: rare; the thread owning the start's word sorts the run and
                // recomputes the head bits inside it
                bool lng = false;
                {
                    const uint32_t m = word_owner ? hs[tid] : 0u, nb0 = tid + 1 < (int)kWords ? hs[tid + 1] & 1u : 0u;
                    for (uint32_t cand = m & ~((m >> 1) | (nb0 << 31)); cand; cand &= cand - 1u) {
                        const uint32_t st = 32u * (uint32_t)tid + (uint32_t)__builtin_ctz(cand);
                        uint32_t en = nk;   // the next run start (bits past nk are 0)
                        for (uint32_t pos = st + 1; pos < nk; pos = (pos | 31u) + 1u) {
                            const uint32_t wd = hs[pos >> 5] >> (pos & 31u);
                            if (wd) {
                                en = pos + (uint32_t)__builtin_ctz(wd);
                                break;
                            }
                        }
                        if (st >= nk || en - st < 2) continue;
                        if (en - st > kRun) {   // long: fine only if every key equals the first
                            const KeyT f = stage[st];
                            for (uint32_t i = st + 1; i < en && !lng; ++i) lng = stage[i] != f;
                            continue;
                        }
                        for (uint32_t i = st + 1; i < en; ++i) {   // insertion sort
                            const KeyT v = stage[i];
                            uint32_t j = i;
                            while (j > st && stage[j - 1] > v) {
                                stage[j] = stage[j - 1];
                                --j;
                            }
                            stage[j] = v;
                        }
                        for (uint32_t i = st + 1; i < en; ++i) {   // the run's head bits, in order now
                            const uint32_t bit = 1u << (i & 31u);
                            if (stage[i] != stage[i - 1]) atomicOr(&hh[i >> 5], bit);
                            else atomicAnd(&hh[i >> 5], ~bit);
                        }
                    }
                }
                const bool again = __syncthreads_or(lng);
                tick(2);
                if (!again) break;
#pragma unroll
                for (int it = 0; it < PER; ++it) y[it] = srow[it * 64];
                lds_sync();
            }
        }
        // ---------------------------------------------------- next chunk: its keys into y now
        uint32_t xt = 0, c0n = 0, c1n = 0;
        if (cn < total) {
            if (tid == 0) xt = atomicAdd(ticket, 1u);   // the chunk after cn (published at the end)
            c0n = cfirst[gn];
            c1n = cfirst[gn + 1];
            if (chn.ovf == kNoOvf) {
                // every load unconditional (slots past the chunk re-read its last key), so
                // the 32 loads leave back to back: a load under a lane test is a branch,
                // and the compiler waits for each such load before the next one
                // (raw keys: the base is taken off when the sort starts, so nothing
                // waits for these loads before then)
                uint32_t l = li0;
                asm volatile("" : "+v"(l));   // per chunk: nothing derived from it is hoisted out of the loop
                const KeyT* src = kb + chn.start;
                const uint32_t lastk = chn.nkeys - 1u;   // nkeys >= 1
#pragma unroll
                for (int it = 0; it < PER; ++it) y[it] = src[min(l + (uint32_t)it * 64u, lastk)];
            }
        }
        if (have && ch.ovf == kNoOvf) {
            // ------------------------------------------------ run-length encoding
            // (LDS-only barriers from here on: the next chunk's key loads stay in flight)
            uint32_t nu;
            const uint32_t wx = block_excl_scan<kCWaves, true>(word_owner ? (uint32_t)__builtin_popcount(hh[tid]) : 0u,
                                                               wsum, &nu);
            if (word_owner) wpre[tid] = wx;
            tick(3);
            if (tid == 0) {
                const uint32_t bf = lookback(cstatus, 1, flags, c, c0, nu, 1u);
                before_s = bf;
                if (last) unq[g] = (uint64_t)bf + nu;
            }
            lds_sync();
            tick(4);
            const uint64_t o0 = goff[g] + before_s;
#pragma unroll KF_SP_UNROLL_STORES
            for (int it = 0; it < PER; ++it) {
                const uint32_t i = li0 + (uint32_t)it * 64;
                if (i >= nk) continue;
                const uint32_t wd = hh[i >> 5];
                if (!((wd >> (i & 31u)) & 1u)) continue;
                const uint32_t j = wpre[i >> 5] + (uint32_t)__builtin_popcount(wd & ((1u << (i & 31u)) - 1u));
                uint32_t nx = nk;
                for (uint32_t pos = i + 1; pos < nk; pos = (pos | 31u) + 1u) {
                    const uint32_t w2 = hh[pos >> 5] >> (pos & 31u);
                    if (w2) {
                        nx = pos + (uint32_t)__builtin_ctz(w2);
                        break;
                    }
                }
                okeys[o0 + j] = (uint64_t)(srow[it * 64] + base);
                ocounts[o0 + j] = min(nx, nk) - i;
            }
            if (tid == 0 && cn < total) cid = take(xt);
            lds_sync();   // stage, masks, cid are reused by the next chunk
            tick(5);
        } else if (have) {
            // ------------------------------------------------ big bucket (sorted in the overflow area)
            const KeyT* x = ovf + ch.ovf;
            uint32_t cnt = 0;
            bool disorder = false;
            for (uint32_t i = tid; i < nk; i += kCBlock) {
                const KeyT a = x[i], pv = i ? x[i - 1] : a;
                cnt += (i == 0 || a != pv) ? 1u : 0u;
                disorder |= a < pv;
            }
            if (__ballot(disorder) && lane == 0) atomicOr(flags, 2u | 32u);
            uint32_t nu;
            (void)block_excl_scan<kCWaves>(cnt, wsum, &nu);
            if (tid == 0) {
                const uint32_t bf = lookback(cstatus, 1, flags, c, c0, nu, 1u);
                before_s = bf;
                if (last) unq[g] = (uint64_t)bf + nu;
            }
            __syncthreads();
            const uint64_t o0 = goff[g] + before_s;
            // heads in order: key and (temporarily) its slot
            uint32_t run = 0;
            for (uint32_t r = 0; r < nk; r += kCBlock) {
                const uint32_t i = r + (uint32_t)tid;
                const KeyT a = i < nk ? x[i] : (KeyT)0, pv = i && i < nk ? x[i - 1] : a;
                const bool hd = i < nk && (i == 0 || a != pv);
                uint32_t tot;
                const uint32_t e = block_excl_scan<kCWaves>(hd ? 1u : 0u, wsum, &tot);
                if (hd) {
                    okeys[o0 + run + e] = (uint64_t)a;
                    ocounts[o0 + run + e] = i;
                }
                run += tot;
            }
            // counts = next head's slot - this one's (reads before writes, per round)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            for (uint32_t r = 0; r < nu; r += kCBlock) {
                const uint32_t jj = r + (uint32_t)tid;
                uint32_t a = 0, b = 0;
                if (jj < nu) {
                    a = __builtin_nontemporal_load(ocounts + o0 + jj);
                    b = jj + 1 < nu ? __builtin_nontemporal_load(ocounts + o0 + jj + 1) : nk;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (jj < nu) ocounts[o0 + jj] = b - a;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
            if (tid == 0 && cn < total) cid = take(xt);
            __syncthreads();
        } else {
            // no chunk yet (first iteration): every thread has read cid by now
            lds_sync();
            if (tid == 0 && cn < total) cid = take(xt);
            lds_sync();
        }
        if (cn >= total) {
            if (prof && tid == 0)
                for (int x = 0; x < 7; ++x) atomicAdd(&prof[x], pt[x]);
            return;
        }
        c = cn;
        ch = chn;
        g = gn;
        c0 = c0n;
        last = cn + 1 == c1n;
        cn = cid;
    }
}

// ---- C3. distinct k-mers per genome (the last chunk's inclusive prefix; 0
// for a genome without windows) or the failure codes.
__global__ void __launch_bounds__(256) sp2_final_kernel(const uint32_t* tfirst, int n, const uint32_t* oflags,
                                                        const uint64_t* unq, uint64_t* nuniq) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint32_t f = tfirst[n + 1] | (*oflags & 2u);
    nuniq[g] = (f & 1u) ? ~0ull : (f & 2u) ? ~1ull : unq[g];
}

// Workspace carve-up (byte offsets, 256-aligned).
struct SpLayout {
    // phase A / B: tiles of kTB bytes
    uint64_t tfirst, xlo, gtot, gbase, gkeys, bstatus, bticket, border;
    // phase C: chunks
    uint64_t nch, nbig, bigkeys, cfirst, bfirst, obase, chunks, bigc, cstatus, cticket, corder, unq;
    // overflow LSD sort of big buckets
    uint64_t seg_off, otfirst, oxlo, ostatus, ogall, oticket, oorder;
    uint64_t kb, ovf, total;   // bucketed keys, overflow keys
    uint32_t tiles, cmax, smax, otiles;
};

uint64_t al256(uint64_t x) { return (x + 255) & ~255ull; }

SpLayout sp_layout(int k, uint64_t batch_bytes, int32_t n) {
    SpLayout L;
    const uint64_t ks = k <= 16 ? 4 : 8;
    const uint64_t cap = ks == 4 ? ChunkOf<uint32_t>::cap : ChunkOf<uint64_t>::cap;
    L.tiles = (uint32_t)(batch_bytes / kTB + (uint64_t)n + 1);
    // greedy packing: two consecutive chunks hold more than cap keys together
    L.cmax = (uint32_t)(2 * batch_bytes / cap + (uint64_t)n + 1);
    L.smax = (uint32_t)(batch_bytes / (cap + 1) + 1);   // big buckets hold more than cap keys
    L.otiles = (uint32_t)(batch_bytes / (ks == 4 ? TileOf<uint32_t>::tile : TileOf<uint64_t>::tile) + L.smax + 1);
    const uint64_t nn = (uint64_t)n;
    uint64_t o = 0;
    auto put = [&](uint64_t& f, uint64_t bytes) {
        f = o;
        o = al256(o + bytes);
    };
    put(L.tfirst, 4ull * (nn + 2 + L.tiles));
    put(L.xlo, 4ull * (L.tiles + 1));
    put(L.gtot, 4ull * nn * kNB);
    put(L.gbase, 4ull * nn * kNB);
    put(L.gkeys, 4ull * nn);
    put(L.bstatus, 8ull * kNB * L.tiles);
    put(L.bticket, 4ull * 4);
    put(L.border, 4ull * L.tiles);
    put(L.nch, 4ull * nn);
    put(L.nbig, 4ull * nn);
    put(L.bigkeys, 4ull * nn);
    put(L.cfirst, 4ull * (nn + 2 + L.cmax));
    put(L.bfirst, 4ull * (nn + 1));
    put(L.obase, 4ull * (nn + 1));
    put(L.chunks, sizeof(Chunk) * (uint64_t)L.cmax);
    put(L.bigc, 4ull * L.smax);
    put(L.cstatus, 8ull * L.cmax);
    put(L.cticket, 4ull * 4);
    put(L.corder, 4ull * L.cmax);
    put(L.unq, 8ull * nn);
    put(L.seg_off, 8ull * (L.smax + 1));
    put(L.otfirst, 4ull * (L.smax + 2 + L.otiles));
    put(L.oxlo, 4ull * (L.otiles + 1));
    put(L.ostatus, 8ull * 256 * L.otiles);
    put(L.ogall, 4ull * 8 * 256 * L.smax);
    put(L.oticket, 4ull * 8);
    put(L.oorder, 4ull * L.otiles);
    put(L.kb, ks * batch_bytes);
    put(L.ovf, ks * batch_bytes);
    L.total = o;
    return L;
}

template <typename KeyT>
int sp_prepare() {   // dynamic LDS: phase B staging, phase C chunk, LSD staging
    static bool done = false;
    if (done) return KF_OK;
    if (hipFuncSetAttribute((const void*)&sp2_scatter_kernel<KeyT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(kTB * sizeof(KeyT))) != hipSuccess ||
        hipFuncSetAttribute((const void*)&sp2_chunk_kernel<KeyT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(ChunkOf<KeyT>::cap * sizeof(KeyT))) != hipSuccess ||
        hipFuncSetAttribute((const void*)&sp_scatter_kernel<KeyT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(TileOf<KeyT>::tile * sizeof(KeyT))) != hipSuccess)
        return kf_fail(KF_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    done = true;
    return KF_OK;
}

int sp_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0)
            cus = c;
        else
            cus = 256;
    }
    return cus;
}

template <typename KeyT>
int sp_run(const uint8_t* d_bytes, const uint64_t* d_goff, int32_t n, uint64_t batch_bytes, const uint64_t* d_excl,
           uint64_t n_excl, int k, uint8_t* work, const SpLayout& L, uint64_t* d_keys, uint32_t* d_counts,
           uint64_t* d_nuniq, hipStream_t s) {
    if (const int rc = sp_prepare<KeyT>()) return rc;
    auto at32 = [&](uint64_t off) { return (uint32_t*)(work + off); };
    uint32_t* tfirst = at32(L.tfirst);
    uint32_t* xlo = at32(L.xlo);
    const int D = sp_dbits(k), B = 2 * k - D;
    const int cus = sp_cus();
    // clear what is accumulated or polled: bucket totals, look-back words, tickets
    if (hipMemsetAsync(work + L.gtot, 0, 4ull * n * kNB, s) != hipSuccess ||
        hipMemsetAsync(work + L.bstatus, 0, L.border - L.bstatus, s) != hipSuccess ||   // status + ticket
        hipMemsetAsync(work + L.cstatus, 0, L.corder - L.cstatus, s) != hipSuccess ||   // status + ticket
        hipMemsetAsync(work + L.unq, 0, 8ull * n, s) != hipSuccess ||
        hipMemsetAsync(work + L.ostatus, 0, L.oorder - L.ostatus, s) != hipSuccess)     // status, gall, tickets
        return kf_fail(KF_EHIP, "memset failed");
    // tiles of kTB bytes per genome, their genome and first excluded range
    hipLaunchKernelGGL(sp_tiles_kernel, dim3(1), dim3(1024), 0, s, d_goff, n, batch_bytes, kTB, tfirst);
    hipLaunchKernelGGL(sp_tilemap_kernel, dim3(L.tiles / 256 + 1), dim3(256), 0, s, d_goff, tfirst, n, d_excl,
                       (uint32_t)n_excl, kTB, xlo);
    // A: genome x bucket totals
    const uint32_t slices = (uint32_t)max(1, min(64, 1024 / max(1, (int)n)));
    hipLaunchKernelGGL(sp2_count_kernel<KeyT>, dim3((uint32_t)n, slices), dim3(kBBlock), 0, s, d_bytes, d_goff, tfirst,
                       n, d_excl, (uint32_t)n_excl, xlo, k, B, batch_bytes, at32(L.gtot));
    hipLaunchKernelGGL(sp2_gbase_kernel, dim3((uint32_t)n), dim3(1024), 0, s, d_goff, at32(L.gtot), n, at32(L.gbase),
                       at32(L.gkeys));
    unsigned long long* prof = nullptr;   // [0, 8): chunk kernel phases, [8, 16): bucket scatter phases
#ifdef KF_PROFILE_BUILD
    const char* pe = getenv("KF_SPARSE_PROFILE");   // debugging aid: synchronous, prints to stderr
    if (pe && *pe == '1' && (hipMalloc((void**)&prof, 128) != hipSuccess || hipMemsetAsync(prof, 0, 128, s) != hipSuccess))
        return kf_fail(KF_EHIP, "profile buffer");
#endif
    // B: scatter by bucket
    uint32_t* border = nullptr;
    if (n > 1 && n <= KF_SPARSE_ORDER_MAXN) {
        border = at32(L.border);
        hipLaunchKernelGGL(sp_order_kernel, dim3(L.tiles / kSBlock + 1), dim3(kSBlock), 0, s, tfirst, n, border);
    }
    KeyT* kb = (KeyT*)(work + L.kb);
    KeyT* ovf = (KeyT*)(work + L.ovf);
    hipLaunchKernelGGL(sp2_scatter_kernel<KeyT>, dim3((uint32_t)cus), dim3(kBBlock), kTB * sizeof(KeyT), s, d_bytes,
                       d_goff, tfirst, n, d_excl, (uint32_t)n_excl, xlo, k, B, batch_bytes, at32(L.gbase),
                       (uint64_t*)(work + L.bstatus), at32(L.bticket), border, kb, prof ? prof + 8 : nullptr);
    // C0: chunk plan
    const uint32_t cap = ChunkOf<KeyT>::cap;
    uint64_t* seg_off = (uint64_t*)(work + L.seg_off);
    hipLaunchKernelGGL(sp2_plan_kernel, dim3((uint32_t)n), dim3(64), 0, s, at32(L.gtot), at32(L.gbase), n, k, cap, 0,
                       at32(L.nch), at32(L.nbig), at32(L.bigkeys), at32(L.cfirst), at32(L.bfirst), at32(L.obase),
                       (Chunk*)(work + L.chunks), seg_off, at32(L.bigc));
    hipLaunchKernelGGL(sp2_cscan_kernel, dim3(1), dim3(1024), 0, s, at32(L.nch), at32(L.nbig), at32(L.bigkeys), n,
                       L.smax, at32(L.cfirst), at32(L.bfirst), at32(L.obase), seg_off);
    hipLaunchKernelGGL(sp2_plan_kernel, dim3((uint32_t)n), dim3(64), 0, s, at32(L.gtot), at32(L.gbase), n, k, cap, 1,
                       at32(L.nch), at32(L.nbig), at32(L.bigkeys), at32(L.cfirst), at32(L.bfirst), at32(L.obase),
                       (Chunk*)(work + L.chunks), seg_off, at32(L.bigc));
    // C1: big buckets -> overflow area, LSD-sorted there on their low B bits
    // (nothing to do, and every workgroup leaves at once, unless a bucket
    // holds more than cap keys)
    const int passes = (B + 7) / 8;
    if (passes > 0) {
        const int bits = (B + passes - 1) / passes;
        // the sorted keys must end in ovf: gather into ovf for an even number of passes
        KeyT* src = (passes % 2 == 0) ? ovf : (KeyT*)d_keys;
        KeyT* dst = (passes % 2 == 0) ? (KeyT*)d_keys : ovf;
        hipLaunchKernelGGL(sp2_gather_kernel<KeyT>, dim3((uint32_t)cus), dim3(256), 0, s, kb,
                           (const Chunk*)(work + L.chunks), at32(L.bigc), at32(L.bfirst), n, src);
        uint32_t* otfirst = at32(L.otfirst);
        const int S = (int)L.smax;
        hipLaunchKernelGGL(sp_tiles_kernel, dim3(1), dim3(1024), 0, s, seg_off, S, batch_bytes, TileOf<KeyT>::tile,
                           otfirst);
        hipLaunchKernelGGL(sp_tilemap_kernel, dim3(L.otiles / 256 + 1), dim3(256), 0, s, seg_off, otfirst, S,
                           (const uint64_t*)nullptr, 0u, TileOf<KeyT>::tile, at32(L.oxlo));
        uint32_t* gall = at32(L.ogall);
        hipLaunchKernelGGL(sp_ghist_kernel<KeyT>, dim3((uint32_t)min(S, 4 * cus)), dim3(kSBlock), 0, s, src, seg_off,
                           otfirst, S, passes, bits, B, gall);
        uint32_t* oorder = nullptr;
        if (S > 1 && S <= KF_SPARSE_ORDER_MAXN) {
            oorder = at32(L.oorder);
            hipLaunchKernelGGL(sp_order_kernel, dim3(L.otiles / kSBlock + 1), dim3(kSBlock), 0, s, otfirst, S, oorder);
        }
        for (int p = 0; p < passes; ++p) {
            const int shift = p * bits;
            const int b = min(bits, B - shift);
            hipLaunchKernelGGL(sp_scatter_kernel<KeyT>, dim3((uint32_t)(2 * cus)), dim3(kSBlock),
                               TileOf<KeyT>::tile * sizeof(KeyT), s, src, dst, seg_off, otfirst, S, shift, b,
                               gall + (uint64_t)p * S * 256, (uint64_t*)(work + L.ostatus), at32(L.oticket) + p,
                               (uint32_t)p + 1, oorder);
            KeyT* t = src;
            src = dst;
            dst = t;
        }
    } else {
        // B == 0 (k <= 5): a bucket is one key value; a big bucket is sorted as it stands
        hipLaunchKernelGGL(sp2_gather_kernel<KeyT>, dim3((uint32_t)cus), dim3(256), 0, s, kb,
                           (const Chunk*)(work + L.chunks), at32(L.bigc), at32(L.bfirst), n, ovf);
    }
    // C2: chunks
    uint32_t* corder = nullptr;
    if (n > 1 && n <= KF_SPARSE_ORDER_MAXN) {
        corder = at32(L.corder);
        hipLaunchKernelGGL(sp_order_kernel, dim3(L.cmax / kSBlock + 1), dim3(kSBlock), 0, s, at32(L.cfirst), n, corder);
    }
    hipLaunchKernelGGL(sp2_chunk_kernel<KeyT>, dim3((uint32_t)(cus * ChunkOf<KeyT>::per_cu)), dim3(kCBlock),
                       ChunkOf<KeyT>::cap * sizeof(KeyT), s,
                       kb, ovf, (const Chunk*)(work + L.chunks), at32(L.cfirst), n, B, d_goff, &tfirst[n + 1],
                       (uint64_t*)(work + L.cstatus), at32(L.cticket), corder, d_keys, d_counts,
                       (uint64_t*)(work + L.unq), prof);
    // the overflow sort's flag word (look-back stall) when it ran, else the main one
    const uint32_t* oflags = passes > 0 ? at32(L.otfirst) + L.smax + 1 : &tfirst[n + 1];
#ifdef KF_PROFILE_BUILD
    if (prof) {
        unsigned long long h[16] = {0};
        if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(h, prof, 128, hipMemcpyDeviceToHost) != hipSuccess)
            return kf_fail(KF_EHIP, "profile readback");
        (void)hipFree(prof);
        fprintf(stderr, "[kf_sparse k=%d] chunk kernel, cycles summed over workgroups (thread 0): pass0+load %.3g "
                "pass1 %.3g fixup %.3g heads %.3g lookback %.3g stores %.3g\n", k, (double)h[0], (double)h[1],
                (double)h[2], (double)h[3], (double)h[4], (double)h[5]);
        fprintf(stderr, "[kf_sparse k=%d] bucket scatter, cycles summed over workgroups (thread 0): ticket+emit %.3g "
                "rank %.3g scan+lookback %.3g stage %.3g stores %.3g\n", k, (double)h[8], (double)h[9],
                (double)h[10], (double)h[11], (double)h[12]);
    }
    if (getenv("KF_SPARSE_DEBUG")) {   // which check flagged the call (2: any; 16: chunk order; 32: big-bucket order)
        uint32_t f[2] = {0, 0};
        if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(&f[0], &tfirst[n + 1], 4, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(&f[1], oflags, 4, hipMemcpyDeviceToHost) != hipSuccess)
            return kf_fail(KF_EHIP, "debug readback");
        fprintf(stderr, "[kf_sparse k=%d] flags main 0x%x overflow 0x%x (passes %d, big keys area %u segments)\n", k,
                f[0], f[1], passes, L.smax);
    }
#endif
    hipLaunchKernelGGL(sp2_final_kernel, dim3((n + 255) / 256), dim3(256), 0, s, tfirst, n, oflags,
                       (const uint64_t*)(work + L.unq), d_nuniq);
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
