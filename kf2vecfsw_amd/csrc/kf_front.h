// kf_front.h -- per-lane front end shared by the count kernels (kf_count.hip)
// and the bucket kernels (kf_bucket.hip): byte classification, newline
// compaction, lane tails / context, masks for genome edges and excluded
// intervals, and the window register of one 1 KiB chunk.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kf {

constexpr int kWave = 64;
constexpr int kChunk = 1024;       // bytes per wave iteration (64 lanes x 16 B)

struct CountArgs {
    const uint8_t* bytes;
    const uint64_t* goff;
    const uint64_t* excl;          // [s0,e0,s1,e1,...]
    uint64_t n_excl;
    const uint32_t* code2col;
    const uint32_t* col2rep;
    uint32_t* counts;
    unsigned long long* totals;
    uint32_t nbins;
    int32_t n_genomes;
    uint32_t flags;                // kf_count_batch flags (KF_ACCUMULATE)
};

// ---------------------------------------------------------------- tails
// A "tail" summarises a stretch of the compacted entry stream:
//   codes [0,22): the last <= k-1 entries' 2-bit codes (last entry lowest)
//   n     [22,27): length of the trailing run of valid bases (capped at 31)
//   ne    [27,32): number of entries (capped at 31)
__device__ __forceinline__ uint32_t tail_pack(uint32_t codes, uint32_t n, uint32_t ne) {
    return codes | (min(n, 31u) << 22) | (min(ne, 31u) << 27);
}
__device__ __forceinline__ uint32_t t_codes(uint32_t t) { return t & 0x3FFFFFu; }
__device__ __forceinline__ uint32_t t_n(uint32_t t) { return (t >> 22) & 31u; }
__device__ __forceinline__ uint32_t t_ne(uint32_t t) { return t >> 27; }

template <int K>
__device__ __forceinline__ uint32_t tail_combine(uint32_t a, uint32_t b) {
    constexpr uint32_t TM = (K > 1) ? ((1u << (2 * (K - 1))) - 1u) : 0u;
    const uint32_t bn = t_n(b), bne = t_ne(b);
    const uint32_t n = (bn < bne) ? bn : min(t_n(a) + bn, 31u);
    const uint32_t codes =
        (bne >= (uint32_t)(K - 1)) ? t_codes(b) : (((t_codes(a) << (2 * bne)) | t_codes(b)) & TM);
    return tail_pack(codes, n, t_ne(a) + bne);
}
template <int K>
__device__ __forceinline__ bool tail_complete(uint32_t t) {
    return t_n(t) < t_ne(t) || t_n(t) >= (uint32_t)(K - 1);
}

// ---------------------------------------------------------------- classify
// 16 bytes -> codes C (byte i at bits 2(15-i)), invalid mask INV and
// not-newline mask NNL (byte i at bit 15-i).  Valid bases: ACGTacgt.
//   cb = (b >> 1) & 3            kf code (A0 C1 T2 G3)
//   y  = (b ^ TBL[cb]) & 0xDF    == 0x0C iff b is the base cb (either case)
//   perm(-1,-1,sel) yields 0x00 for sel == 12 and 0xFF for every other byte
//   dot4 packs four codes / four flags into one byte / nibble in memory order.
__device__ __forceinline__ void classify16(const uint4 d, uint32_t& C, uint32_t& INV, uint32_t& NNL) {
    const uint32_t w[4] = {d.x, d.y, d.z, d.w};
    uint32_t pc[4], vf[4], nf[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = w[q];
        const uint32_t cb = (x >> 1) & 0x03030303u;
        const uint32_t ex = __builtin_amdgcn_perm(0u, 0x4B584F4Du, cb);   // "ACTG" ^ 0x0C
        const uint32_t y = (x ^ ex) & 0xDFDFDFDFu;
        vf[q] = __builtin_amdgcn_perm(0xFFFFFFFFu, 0xFFFFFFFFu, y);          // 0x00 valid base
        nf[q] = __builtin_amdgcn_perm(0xFFFFFFFFu, 0xFFFFFFFFu, x ^ 0x06060606u);   // 0x00 newline
        pc[q] = __builtin_amdgcn_udot4(cb, 0x01041040u, 0u, false);
    }
    // codes: byte q of C (from the top) = pc[q]
    const uint32_t c01 = __builtin_amdgcn_perm(pc[0], pc[1], 0x0C0C0400u);
    const uint32_t c23 = __builtin_amdgcn_perm(pc[2], pc[3], 0x0C0C0400u);
    C = (c01 << 16) | c23;
    // flag bytes are 0x00 / 0xFF (= -1 signed).  Weights -8,-4,-2,-1 give dword
    // q+1's nibble and -128,-64,-32,-16 dword q's nibble one position up, so one
    // accumulating dot pair packs a byte of the mask.
    auto pair = [](const uint32_t a, const uint32_t b) -> uint32_t {
        return (uint32_t)__builtin_amdgcn_sdot4((int)a, (int)0xF0E0C080u,
                                               __builtin_amdgcn_sdot4((int)b, (int)0xFFFEFCF8u, 0, false), false);
    };
    INV = (pair(vf[0], vf[1]) << 8) | pair(vf[2], vf[3]);
    NNL = (pair(nf[0], nf[1]) << 8) | pair(nf[2], nf[3]);   // not-newline mask
}

// Fast-path flavour of classify16: codes C, not-newline mask NNL, and `bad`,
// non-zero iff some byte is neither a base nor a newline: z = (b ^ TBL[cb]) & 0xDF
// with TBL = "ACTG" is 0 exactly for a base (either case), and newline bytes are
// masked out by nf (one v_perm per word less than testing z with a v_perm).
__device__ __forceinline__ void classify16_fast(const uint4 d, uint32_t& C, uint32_t& NNL, uint32_t& bad) {
    const uint32_t w[4] = {d.x, d.y, d.z, d.w};
    uint32_t pc[4], nf[4];
    bad = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = w[q];
        const uint32_t cb = (x >> 1) & 0x03030303u;
        const uint32_t ex = __builtin_amdgcn_perm(0u, 0x47544341u, cb);   // "ACTG"
        const uint32_t z = (x ^ ex) & 0xDFDFDFDFu;
        nf[q] = __builtin_amdgcn_perm(0xFFFFFFFFu, 0xFFFFFFFFu, x ^ 0x06060606u);
        bad |= z & nf[q];
        pc[q] = __builtin_amdgcn_udot4(cb, 0x01041040u, 0u, false);
    }
    const uint32_t c01 = __builtin_amdgcn_perm(pc[0], pc[1], 0x0C0C0400u);
    const uint32_t c23 = __builtin_amdgcn_perm(pc[2], pc[3], 0x0C0C0400u);
    C = (c01 << 16) | c23;
    auto pair = [](const uint32_t a, const uint32_t b) -> uint32_t {
        return (uint32_t)__builtin_amdgcn_sdot4((int)a, (int)0xF0E0C080u,
                                               __builtin_amdgcn_sdot4((int)b, (int)0xFFFEFCF8u, 0, false), false);
    };
    NNL = (pair(nf[0], nf[1]) << 8) | pair(nf[2], nf[3]);
}

// Remove newline entries (compaction).  C: 2-bit entries, V/EN: 1-bit masks,
// entry r at bits [2r, 2r+2) / bit r.  The lowest newline is removed branch-free
// (r = 16 sentinel when there is none: every mask becomes the identity); any
// further newline in the same 16 bytes (lines shorter than 16) takes the loop.
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

template <bool MASKED>
__device__ __forceinline__ void remove_entry(uint32_t r, uint32_t& C, uint32_t& V, uint32_t& EN, uint32_t& nl) {
    const uint32_t lo1 = (1u << r) - 1u;          // entries below r stay
    const uint32_t lo2 = lo1 | (lo1 << r);         // (1 << 2r) - 1, also for r = 16
    V = bfi(lo1, V, V >> 1);
    if (MASKED) EN = bfi(lo1, EN, EN >> 1);
    C = bfi(lo2, C, C >> 2);
    nl = (nl >> 1) & ~lo1;                         // drop bit r, shift the rest down
}

template <bool MASKED>
__device__ __forceinline__ void compact(uint32_t nl, uint32_t& C, uint32_t& V, uint32_t& EN) {
    remove_entry<MASKED>((uint32_t)__builtin_ctz(nl | 0x10000u), C, V, EN, nl);
    while (nl) remove_entry<MASKED>((uint32_t)__builtin_ctz(nl), C, V, EN, nl);
}

__device__ __forceinline__ uint32_t revpairs(uint32_t x) {
    const uint32_t t = __builtin_bitreverse32(x);
    return ((t << 1) & 0xAAAAAAAAu) | ((t >> 1) & 0x55555555u);
}

// reverse complement of a K-mer in kf code (complement = code ^ 2)
template <int K>
__device__ __forceinline__ uint32_t kf_revcomp(uint32_t x) {
    return (revpairs(x) >> (32 - 2 * K)) ^ (0xAAAAAAAAu >> (32 - 2 * K));
}

template <int K>
__device__ __forceinline__ uint32_t run_mask(uint32_t E) {
    // bit r set iff entries r .. r+K-1 are all valid
    uint32_t R = E;
    int a = 1;
#pragma unroll
    for (int it = 0; it < 5; ++it) {
        if (a < K) {
            const int s = (a < K - a) ? a : (K - a);
            R &= R >> s;
            a += s;
        }
    }
    return R;
}

// Atomic add to the LDS word at byte address `a`.  The histogram is the whole
// dynamic LDS allocation and the kernel declares no static LDS, so it starts at
// LDS address 0 (checked once per kernel): a raw address-space-3 pointer avoids a
// base add per k-mer.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ void lds_add(uint32_t a, uint32_t v) {
    __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ uint32_t wave_shr1(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// Inclusive prefix sum over the wave on the VALU (DPP row shifts and row
// broadcasts; no LDS traffic, unlike __shfl_up's ds_bpermute).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

// Exclusive scan of lane tails with a carry-in (slow path: some lane's block has
// fewer than k-1 entries and no reset, e.g. very short FASTA lines).
template <int K>
__device__ __noinline__ uint32_t scan_ctx(uint32_t own, uint32_t carry, int lane) {
    uint32_t v = own;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, kWave);
        if (lane >= d) v = tail_combine<K>(o, v);
    }
    const uint32_t ex = __shfl_up(v, 1, kWave);
    return lane == 0 ? carry : tail_combine<K>(carry, ex);
}

// Load a wave-uniform 64-bit word and pin it in SGPRs: compares against it then
// never wait on the vector-memory counter shared with the byte-stream prefetch.
__device__ __forceinline__ uint64_t uload64(const uint64_t* p) {
    const uint64_t v = *p;
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

struct ChunkMask {
    // byte-position bounds for masked chunks (absolute offsets)
    uint64_t glo;   // bytes < glo are invalid (previous genome)
    uint64_t lo;    // count only windows ending at bytes in [lo, hi)
    uint64_t hi;
};

__device__ __forceinline__ uint32_t range_bits(int64_t a, int64_t b) {
    // bits for bytes [a, b) of a 16-byte block (byte i at bit 15-i), a,b clamped to [0,16]
    a = a < 0 ? 0 : (a > 16 ? 16 : a);
    b = b < 0 ? 0 : (b > 16 ? 16 : b);
    if (b <= a) return 0u;
    const uint32_t n = (uint32_t)(b - a);
    return ((n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u)) << (16 - (uint32_t)b)) & 0xFFFFu;
}

// Apply genome start / count window / excluded intervals to one lane's block.
__device__ __forceinline__ void apply_masks(const CountArgs& A, uint64_t chunk, int lane,
                                            const ChunkMask& m, uint64_t iv0,
                                            uint32_t& INV, uint32_t& EN) {
    const int64_t b0 = (int64_t)(chunk + 16u * (uint32_t)lane);
    INV |= range_bits(-1, (int64_t)m.glo - b0);
    EN = range_bits((int64_t)m.lo - b0, (int64_t)m.hi - b0);
    const uint64_t cend = chunk + kChunk;
    for (uint64_t i = iv0; i < A.n_excl; ++i) {      // wave-uniform loop
        const uint64_t s = uload64(A.excl + 2 * i), e = uload64(A.excl + 2 * i + 1);
        if (s >= cend) break;
        INV |= range_bits((int64_t)s - b0, (int64_t)e - b0);
    }
}

// Buffer descriptor of the chunk at c, clamped to the genome end rounded up to
// 16 bytes: the hardware range check zeroes a whole dword/vector that straddles
// num_records, so an exact (unaligned) end would drop the genome's last bases.
// Bytes in [ghi, align16(ghi)) are read but never counted (they lie past hi).
// c = c0 + rel; end_r = align16(ghi) - c0 (32-bit: see process_range)
#ifndef KF_CHUNK_CPOL
#define KF_CHUNK_CPOL 2   // 1 KiB chunk stream: non-temporal (k=5 -1.3 %, k=9 -1.7 %, k=11 same; v10_lib_ab_*_chunk_nt)
#endif
__device__ __forceinline__ uint4 load_chunk(const uint8_t* bytes, uint64_t c0, uint32_t rel, uint32_t end_r,
                                            int lane) {
    const uint32_t rec = end_r > rel ? min(end_r - rel, (uint32_t)kChunk) : 0u;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + c0 + rel), (short)0, (int)rec, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, 0, KF_CHUNK_CPOL);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// Tail of one lane's block; compaction shifts zeros into V above entry ne-1,
// so ctz(~V) <= ne <= 16.
template <int K>
__device__ __forceinline__ uint32_t own_tail(uint32_t C, uint32_t V, uint32_t ne) {
    constexpr uint32_t TM = (K > 1) ? ((1u << (2 * (K - 1))) - 1u) : 0u;
    return (C & TM) | ((uint32_t)__builtin_ctz(~V) << 22) | (ne << 27);
}

// Per-lane front end shared by every path: block -> (C, V, EN, ne, own tail).
template <int K, bool MASKED, bool OWN = true>
__device__ __forceinline__ void front_end(const uint4 d, const CountArgs& A, uint64_t chunk, int lane,
                                          const ChunkMask& m, uint64_t iv0,
                                          uint32_t& C, uint32_t& V, uint32_t& EN, uint32_t& ne,
                                          uint32_t& own) {
    uint32_t INV, NNL;
    classify16(d, C, INV, NNL);
    EN = 0xFFFFu;
    if (MASKED) apply_masks(A, chunk, lane, m, iv0, INV, EN);
    V = ~INV & 0xFFFFu;
    ne = (uint32_t)__builtin_popcount(NNL);
    compact<MASKED>(NNL ^ 0xFFFFu, C, V, EN);
    if (OWN) own = own_tail<K>(C, V, ne);
}

// Index of the first element of a non-decreasing sequence key(0..n) with
// key(i) > x (n if none), by a 64-way wave-parallel search: one load latency per
// 64x narrowing instead of one per halving (log64 n vs log2 n dependent loads).
// Wave-uniform arguments; every lane must be active.
template <class KeyF>
__device__ __forceinline__ uint64_t wave_upper_bound(uint64_t n, uint64_t x, int lane, KeyF key) {
    uint64_t a = 0, b = n;   // the answer lies in [a, b]
    while (b - a > (uint64_t)kWave) {
        const uint64_t step = (b - a + kWave - 1) / kWave;
        const uint64_t i = a + step * (uint64_t)lane;
        const uint32_t cnt = (uint32_t)__builtin_popcountll(__ballot(i < b && key(i) <= x));
        const uint64_t na = cnt ? a + step * (cnt - 1) + 1 : a;
        b = min(b, a + step * cnt);
        a = na;
    }
    const uint64_t i = a + (uint64_t)lane;
    return a + (uint64_t)__builtin_popcountll(__ballot(i < b && key(i) <= x));
}

// Lane block of the 1 KiB chunk at p for chunk_tail_data (bytes before the
// genome's aligned start read as zero, so p may lie before the buffer).
__device__ __forceinline__ uint4 chunk_tail_load(const uint8_t* bytes, int64_t p, uint64_t glo, int lane) {
    const int64_t b0 = p + 16 * lane;
    uint4 d = make_uint4(0u, 0u, 0u, 0u);
    if (b0 >= (int64_t)(glo & ~(uint64_t)15)) d = *(const uint4*)(bytes + b0);
    return d;
}

// Inclusive tail of the 1 KiB chunk starting at p whose lane block d is already
// loaded (warm-up only; bytes before glo are invalid).
template <int K>
__device__ __noinline__ uint32_t chunk_tail_data(const uint4 d, const uint8_t* bytes, const uint64_t* excl,
                                                 uint64_t n_excl, int64_t p, uint64_t glo, int lane) {
    CountArgs A{};
    A.bytes = bytes;
    A.excl = excl;
    A.n_excl = n_excl;
    // first excluded interval that ends after the chunk start
    const uint64_t key = p < 0 ? 0 : (uint64_t)p;
    const uint64_t lo = wave_upper_bound(A.n_excl, key, lane, [&](uint64_t i) { return A.excl[2 * i + 1]; });
    ChunkMask m{glo, 0, 0};
    uint32_t C, V, EN, ne, own;
    front_end<K, true>(d, A, (uint64_t)p, lane, m, lo, C, V, EN, ne, own);
    uint32_t v = own;
#pragma unroll
    for (int dd = 1; dd < kWave; dd <<= 1) {
        const uint32_t o = __shfl_up(v, dd, kWave);
        if (lane >= dd) v = tail_combine<K>(o, v);
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)v, kWave - 1);
}

// Inclusive tail of the 1 KiB chunk starting at p (warm-up only; p may lie
// before glo or even before the buffer: those bytes read as invalid).
template <int K>
__device__ __forceinline__ uint32_t chunk_tail(const uint8_t* bytes, const uint64_t* excl, uint64_t n_excl, int64_t p,
                                               uint64_t glo, int lane) {
    return chunk_tail_data<K>(chunk_tail_load(bytes, p, glo, lane), bytes, excl, n_excl, p, glo, lane);
}


// One wave's byte range [lo, hi) of genome [glo, ghi), walked in 1 KiB chunks
// at c0 + rel (rel = 0, 1024, ...).  Chunk bookkeeping is in 32-bit offsets from
// c0 (a wave range is far below 4 GiB): gfx9 SALU has no 64-bit ordered
// compare, so 64-bit bounds tests would run on the VALU once per chunk.
struct Range {
    uint64_t c0, glo, ghi, lo, hi;
    uint32_t lo_r, hi_r, end_r, nch;
    uint64_t iv;              // first excluded interval ending after the chunk
    uint32_t ivs_r, ive_r;    // its bounds relative to c0 (clamped)
    uint64_t ivs_a, ive_a;    // and absolute (~0 if none)
    uint32_t carry;           // tail before the next chunk

    __device__ __forceinline__ uint32_t rel_of(uint64_t x) const {
        return x <= c0 ? 0u : (x - c0 >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)(x - c0));
    }
    // Addresses only (no loads), so the chunk stream can be put in flight before
    // the warm-up's dependent loads.  Requires lo < hi.
    __device__ __forceinline__ void init(uint64_t glo_, uint64_t ghi_, uint64_t lo_, uint64_t hi_) {
        glo = glo_, ghi = ghi_, lo = lo_, hi = hi_;
        c0 = lo & ~(uint64_t)15;
        lo_r = (uint32_t)(lo - c0);
        hi_r = (uint32_t)(hi - c0);
        end_r = rel_of((ghi + 15) & ~(uint64_t)15);
        nch = (hi_r + kChunk - 1) / kChunk;
    }
    template <int K>
    __device__ __forceinline__ void begin(const CountArgs& A, uint64_t glo_, uint64_t ghi_, uint64_t lo_,
                                          uint64_t hi_, int lane) {
        init(glo_, ghi_, lo_, hi_);
        warm<K>(A, lane);
    }
    // Lane block of the chunk before c0 (the first warm-up step), so its load can
    // be issued early; pass it to warm_from.
    __device__ __forceinline__ uint4 ctx_load(const uint8_t* bytes, int lane) const {
        return c0 > glo ? chunk_tail_load(bytes, (int64_t)c0 - kChunk, glo, lane) : make_uint4(0u, 0u, 0u, 0u);
    }
    // Context and first interval (after init).
    template <int K>
    __device__ __forceinline__ void warm(const CountArgs& A, int lane) {
        // warm-up: exact k-1 context before c0 (walk back until complete)
        carry = tail_pack(0, 0, 0);
        for (int64_t p = (int64_t)c0; p > (int64_t)glo && !tail_complete<K>(carry);) {
            p -= kChunk;
            carry = tail_combine<K>(chunk_tail<K>(A.bytes, A.excl, A.n_excl, p, glo, lane), carry);
        }
        find_interval(A, lane);
    }
    // As warm, from the 16 bytes before c0 and one interval search (the common
    // case: they lie inside the genome, outside every excluded interval, and end
    // in >= k-1 bases); anything else takes warm.  Same carry as warm for every
    // use (codes of the last k-1 entries, a run of >= k-1).
    template <int K>
    __device__ __forceinline__ void warm16(const CountArgs& A, int lane) {
        if (c0 < glo + 16) {   // the genome start is within reach
            warm<K>(A, lane);
            return;
        }
        const uint64_t p16 = c0 - 16;
        const uint4 d = *(const uint4*)(A.bytes + p16);   // the same 16 bytes in every lane
        uint64_t s_iv = ~0ull, e_iv = ~0ull;
        iv = wave_upper_bound(A.n_excl, p16, lane, [&](uint64_t i) { return A.excl[2 * i + 1]; });
        if (iv < A.n_excl) {
            s_iv = uload64(A.excl + 2 * iv);
            e_iv = uload64(A.excl + 2 * iv + 1);
        }
        uint32_t C, V, EN, ne, own;
        const ChunkMask m{glo, 0, 0};
        front_end<K, false>(d, A, p16, lane, m, iv, C, V, EN, ne, own);
        if (s_iv < c0 || t_n(own) < (uint32_t)(K - 1)) {   // an interval ends past p16 but starts before c0
            warm<K>(A, lane);
            return;
        }
        carry = own;
        ivs_r = iv < A.n_excl ? rel_of(s_iv) : 0xFFFFFFFFu;
        ive_r = iv < A.n_excl ? rel_of(e_iv) : 0xFFFFFFFFu;
        ivs_a = s_iv, ive_a = e_iv;
    }
    // As warm, with the first chunk before c0 already loaded (ctx_load).
    template <int K>
    __device__ __forceinline__ void warm_from(const CountArgs& A, const uint4 dctx, int lane) {
        carry = tail_pack(0, 0, 0);
        int64_t p = (int64_t)c0;
        if (p > (int64_t)glo) {
            p -= kChunk;
            carry = chunk_tail_data<K>(dctx, A.bytes, A.excl, A.n_excl, p, glo, lane);
        }
        for (; p > (int64_t)glo && !tail_complete<K>(carry);) {   // rare: a short chunk of context
            p -= kChunk;
            carry = tail_combine<K>(chunk_tail<K>(A.bytes, A.excl, A.n_excl, p, glo, lane), carry);
        }
        find_interval(A, lane);
    }
    __device__ __forceinline__ void find_interval(const CountArgs& A, int lane) {
        // first excluded interval ending after c0; its bounds live in registers so
        // the chunk loop issues no vector loads besides the byte stream (a VMEM load
        // there would force vmcnt(0) and drain the prefetch ring)
        iv = wave_upper_bound(A.n_excl, c0, lane, [&](uint64_t i) { return A.excl[2 * i + 1]; });
        ivs_r = ive_r = 0xFFFFFFFFu;
        ivs_a = ive_a = ~0ull;
        if (iv < A.n_excl) {
            ivs_a = uload64(A.excl + 2 * iv);
            ive_a = uload64(A.excl + 2 * iv + 1);
            ivs_r = rel_of(ivs_a);
            ive_r = rel_of(ive_a);
        }
    }
    // true if the chunk at rel needs the masked path (range edge or an excluded
    // interval inside); advances the interval pointer past finished intervals
    __device__ __forceinline__ bool masked(const CountArgs& A, uint32_t rel) {
        if (rel >= ive_r) {   // passed the current interval (rare)
            const uint64_t cc = c0 + rel;
            do { ++iv; } while (iv < A.n_excl && uload64(A.excl + 2 * iv + 1) <= cc);
            ivs_a = iv < A.n_excl ? uload64(A.excl + 2 * iv) : ~0ull;
            ive_a = iv < A.n_excl ? uload64(A.excl + 2 * iv + 1) : ~0ull;
            ivs_r = iv < A.n_excl ? rel_of(ivs_a) : 0xFFFFFFFFu;
            ive_r = iv < A.n_excl ? rel_of(ive_a) : 0xFFFFFFFFu;
        }
        return ivs_r < rel + kChunk || rel < lo_r || rel + kChunk > hi_r;
    }
    // as masked, for the span [rel, rel + len) (len a multiple of kChunk)
    __device__ __forceinline__ bool masked_span(const CountArgs& A, uint32_t rel, uint32_t len) {
        if (rel >= ive_r) return masked(A, rel) || ivs_r < rel + len || rel + len > hi_r;
        return ivs_r < rel + len || rel < lo_r || rel + len > hi_r;
    }
    __device__ __forceinline__ ChunkMask mask() const { return ChunkMask{glo, lo, hi}; }
    __device__ __forceinline__ uint4 load(const uint8_t* bytes, uint32_t rel, int lane) const {
        return load_chunk(bytes, c0, rel, end_r, lane);
    }
};

// Split [plo, phi) into n contiguous 16-byte-aligned parts (monotone, covering).
__device__ __forceinline__ uint64_t split_at(uint64_t plo, uint64_t phi, uint64_t w, uint64_t n) {
    if (w == 0) return plo;
    if (w >= n) return phi;
    const uint64_t len = phi - plo;
    const uint64_t s = (plo + len / n * w + (len % n) * w / n) & ~(uint64_t)15;
    return min(max(s, plo), phi);
}

// As split_at with wave w's part proportional to byte (w >> 2) of `wts` (the
// wave's age slot on its SIMD: the SIMD issues oldest-first, so slot 0 runs
// fastest); n = 16.  wts = 0x01010101 is an equal split.
//   Split once per kernel into a 2^-20 fixed-point fraction (wave_frac), then per
// piece one 64-bit multiply (split_at_frac): a 64x32/32 division per wave and
// piece is a long SALU sequence that the CU's 16 waves serialise on.
__device__ __forceinline__ uint32_t wave_frac(uint32_t w, uint32_t wts) {
    if (w == 0) return 0u;
    if (w >= 16) return 1u << 20;
    const uint32_t b0 = wts & 0xFFu, b1 = (wts >> 8) & 0xFFu, b2 = (wts >> 16) & 0xFFu, b3 = wts >> 24;
    const uint32_t tot = 4u * (b0 + b1 + b2 + b3);
    // prefix weight of waves 0..w-1: full slots below w's slot plus w's own slot members
    const uint32_t s = w >> 2, r = w & 3u;
    uint32_t cum = 0;
    cum += (s > 0 ? 4u * b0 : (r ? r * b0 : 0u));
    cum += (s > 1 ? 4u * b1 : (s == 1 ? r * b1 : 0u));
    cum += (s > 2 ? 4u * b2 : (s == 2 ? r * b2 : 0u));
    cum += (s == 3 ? r * b3 : 0u);
    return (cum << 20) / tot;   // cum <= 15 x 255 = 3825 < 2^12: cum << 20 fits in u32
}

// [plo, phi) at fraction fr / 2^20 (phi - plo < 2^44), 16-byte aligned; the
// same fr gives the same point, so adjacent waves' parts are monotone and covering.
__device__ __forceinline__ uint64_t split_at_frac(uint64_t plo, uint64_t phi, uint32_t fr) {
    if (fr >= (1u << 20)) return phi;
    const uint64_t x = (plo + (((phi - plo) * fr) >> 20)) & ~(uint64_t)15;
    return min(max(x, plo), phi);
}

// Window register of one lane's block (general path): context from lane L-1
// (lane 0: `carry`), exact even through lanes with fewer than k-1 entries.
//   W = context codes << 2ne | C (entry 0 = last byte, lowest), window r = the
//   k-mer ending at entry r = bits [2r, 2r+2K) of W, first base highest;
//   R bit r = window r is counted; `next` = the wave's inclusive tail (carry
//   for the next chunk).
struct Windows {
    uint32_t wlo, whi, R, next;
};
template <int K, bool MASKED>
__device__ __forceinline__ Windows windows(uint32_t C, uint32_t V, uint32_t EN, uint32_t ne, uint32_t carry,
                                           int lane) {
    constexpr uint32_t TM = (K > 1) ? ((1u << (2 * (K - 1))) - 1u) : 0u;
    const uint32_t own = own_tail<K>(C, V, ne);
    // A block is incomplete (needs the exact scan) only if it has fewer than k-1
    // entries and no reset; ne < k-1 needs >= 17-k newlines in 16 bytes, so test
    // that first (one compare) and refine only when it fires.
    uint32_t ctx = wave_shr1(carry, own);
    if (__ballot(ne < (uint32_t)(K - 1)) != 0) {
        const uint64_t inc_mask = __ballot(!tail_complete<K>(own)) & 0x7FFFFFFFFFFFFFFFull;
        if (inc_mask) ctx = scan_ctx<K>(own, carry, lane);
    }
    const uint64_t W = ((uint64_t)t_codes(ctx) << (2 * ne)) | (uint64_t)C;
    Windows w;
    w.wlo = (uint32_t)W;
    w.whi = (uint32_t)(W >> 32);
    const uint32_t ctxlen = min(t_n(ctx), (uint32_t)(K - 1));
    const uint32_t E = (((1u << ctxlen) - 1u) << ne) | V;
    w.R = run_mask<K>(E) & ((1u << ne) - 1u);
    if (MASKED) w.R &= EN;
    const uint32_t incl = tail_pack(w.wlo & TM, (uint32_t)__builtin_ctz(~E), 31u);
    w.next = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
    return w;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
    return v;
}

// Large k: two-phase LDS bucket counting (kf_bucket.hip).  Count rows are
// written whole (no memset needed unless accumulating); the caller zeroes totals.
int bucket_launch(const CountArgs& A, int k, uint32_t flags, hipStream_t s);
int bucket_launch_info(int k, int* grid, int* block, int* lds);
int bucket_reserve(int k, int32_t max_genomes);

}  // namespace kf
