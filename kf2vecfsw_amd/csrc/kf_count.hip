// kf_count.hip -- canonical k-mer counting kernels for k <= 8 on MI355X
// (gfx950, CDNA4), the device half of kf_count_batch (include/kf2vec_gpu.h).
//
// Replaces the Jellyfish shell-out of kf2vec's get_frequencies (reference
// kf2vec/main.py:309-328: `jellyfish count -C` + `jellyfish dump -c` + the
// pandas merge onto the sorted vocabulary).  k >= 9 is kf_bucket.hip.
//
// Work decomposition:
//   * the batch [goff[0], goff[n)) is cut into gridDim.x equal 16-byte-aligned
//     byte spans, one per 1024-thread workgroup (16 waves); a span may cross
//     genome boundaries;
//   * each genome piece of a span is cut into 16 wave ranges; a wave walks its
//     range with buffer loads (a register ring keeps the next loads in flight),
//     classifies the bytes with v_perm / v_dot4 (no table loads), removes
//     newlines, takes the k-1 bases of context from lane L-1 by DPP (lane 0
//     from the wave's carry) and counts FORWARD k-mers into LDS; a k-mer and its
//     reverse complement are merged into their canonical column at the flush;
//   * FASTA headers / FASTQ non-sequence lines arrive as a sorted interval list
//     (kf_index_records) and are invalid bytes (a k-mer reset).
//
// Kernels:
//   K1x k1x_kernel<K>  (k = 2 .. 7): 3 KiB per wave iteration read as three
//       coalesced 1 KiB regions (lane L: bytes 16L + 1024q, non-temporal
//       buffer loads, xc_load); windows are formed per 16-byte region, the
//       k-1 bases of context from lane L-1 by DPP.  Two consecutive k-mer
//       windows are one (k+1)-mer counted once in P (4^(k+1) u16 counters:
//       128 KiB at k = 7), a window left unpaired goes to S (4^k u16 by
//       forward k-mer): half the LDS atomics of one add per window; every add
//       returns the old word and a u16 half that reaches its threshold is moved
//       to the count row (exact: see xc_fast);
//   K1x8 k1x_kernel<8> (k = 8): the K1x front end with every window an 8-mer
//       in P (one pass over the bytes).
//   K9b  k1x_kernel<9> (k = 9, round 6): the K1x front end, every window's
//       canonical class once, all 131,072 classes as u8 counters in LDS whose
//       byte carries are corrected exactly from the adds' returns (see "K9b").
// (Rounds 1-3 counted k <= 6 with one u32 LDS add per window, K1.)
// Rejected alternatives and their measurements live in tools/zoo/ (DESIGN.md).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <mutex>

#include "kf_front.h"
#include "kf_internal.h"

namespace kf {

constexpr int kBlock = 1024;             // threads per workgroup
// K1x: a genome piece's share per wave by the wave's age slot on its SIMD (the
// SIMD issues oldest-first; slot 0 runs ~2.4x faster than slot 3), 8 bits each
#ifndef KF_WAVE_WEIGHTS
#define KF_WAVE_WEIGHTS (20u | 17u << 8 | 11u << 16 | 6u << 24)
#endif
constexpr uint32_t kWaveWeights = KF_WAVE_WEIGHTS;
constexpr int kXRing = 2;    // K1x: 3 KiB iterations in the register ring

__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t a, uint32_t v) {
    return __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Workgroup barrier ordering LDS only: waits for this wave's LDS operations, not
// for its vector-memory ones (__syncthreads waits for vmcnt(0) too, i.e. for the
// ring's prefetches and the flush's row stores; nothing here reads global
// memory another wave of the workgroup wrote).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Byte span [lo, hi) of workgroup b of G over the batch (16-byte aligned).
__device__ __forceinline__ void wg_span(const CountArgs& A, uint64_t& lo, uint64_t& hi) {
    const uint64_t base = A.goff[0];
    const uint64_t total = A.goff[A.n_genomes] - base;
    const uint64_t G = gridDim.x, b = blockIdx.x;
    lo = base + ((total / G * b + (total % G) * b / G) & ~(uint64_t)15);
    hi = (b + 1 == G) ? base + total : base + ((total / G * (b + 1) + (total % G) * (b + 1) / G) & ~(uint64_t)15);
}

// ---------------------------------------------------------------- K1x (k = 2 .. 8)
// LDS layout: P = u16 counters of (k+1)-mers at 0 ((k+1)-mer y in half y & 1 of
// word y >> 1), then S = u16 singles by forward k-mer.  k = 7 takes the whole
// 160 KiB of a CU (P 128 KiB, S 32 KiB); k = 8 counts every window as an 8-mer in
// P (65,536 u16) and its S area only holds the flush's drain flags.
template <int K>
struct XL {
    static constexpr uint32_t P = K >= 8 ? (1u << 17) : (2u << (2 * (K + 1)));   // P bytes = byte offset of S
    static constexpr uint32_t S = K >= 8 ? (1u << 15) : (2u << (2 * K));         // S bytes
    static constexpr uint32_t bytes = P + S;                                      // dynamic LDS of the kernel
};
constexpr int kXChunk = 3 * kChunk;                    // bytes per wave iteration
// u16 exactness (xc_fast): k = 7 checks every add's return against 0x4000 and
// moves 0x4000 at a time; k = 8 (48 adds per lane per iteration) against 0x2000;
// k <= 6 (small tables, frequent crossings) against 0x8000: a half then stays
// below 0x8000 + 16 waves x 1536 adds = 0xE000.
constexpr uint32_t kHot7 = 0xC000C000u, kStep7 = 0x4000u;
constexpr uint32_t kHot8 = 0xE000E000u, kStep8 = 0x2000u;
constexpr uint32_t kHot6 = 0x80008000u, kStep6 = 0x8000u;
template <int K>
constexpr uint32_t x_hot() { return K >= 8 ? kHot8 : (K == 7 ? kHot7 : kHot6); }
template <int K>
constexpr uint32_t x_step() { return K >= 8 ? kStep8 : (K == 7 ? kStep7 : kStep6); }

// ---------------------------------------------------------------- k = 9 classes
// k = 9 has 131,072 canonical classes (4^9 / 2: k odd, no palindromes).  Class
// of a 9-mer y (kf code, first base highest): its orientation whose middle base
// is A or C, i.e. kf-code bit 9 clear -- the reverse complement flips that bit --
// so c = bit9(y) ? rc(y) : y.  Its index is c without bit 9,
// i = (c & 0x1FF) | (c >> 1 & 0x1FE00) (17 bits); k9_code_of(i) gives c back.
__device__ __forceinline__ uint32_t k9_code_of(uint32_t i) { return ((i >> 9) << 10) | (i & 0x1FFu); }

__device__ __forceinline__ uint32_t half_one(uint32_t i) { return 1u << ((i & 1u) << 4); }

// 1 << byte B of h (the byte is 0 or 16): one SDWA shift.
template <int B>
__device__ __forceinline__ uint32_t shl1_byte(uint32_t h, uint32_t one) {
    uint32_t r;
    if constexpr (B == 0)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
            : "=v"(r) : "v"(h), "v"(one));
    else if constexpr (B == 1)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
            : "=v"(r) : "v"(h), "v"(one));
    else if constexpr (B == 2)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
            : "=v"(r) : "v"(h), "v"(one));
    else
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
            : "=v"(r) : "v"(h), "v"(one));
    return r;
}

// Rare path: move STEP out of each half of the LDS word at byte address a that
// has reached it (HOT = the halves' bits at or above STEP) into the count row,
// until both halves are below STEP (compare-and-swap: exact under concurrent
// adds).  k <= 7: a P half is the (k+1)-mer of two windows (older k-mer = bin >> 2,
// newer = bin mod 4^k), an S half one forward k-mer; k = 8: a P half is one 8-mer.
template <int K>
__device__ __noinline__ void x_drain(uint32_t a, const uint32_t* __restrict__ code2col, uint32_t* gcounts) {
    constexpr uint32_t HOT = x_hot<K>(), STEP = x_step<K>();
    constexpr uint32_t PB = XL<K>::P;
    lds_u32* p = (lds_u32*)(uintptr_t)a;
    uint32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (cur & HOT) {
        const uint32_t sub = ((cur & (HOT & 0xFFFF0000u)) ? (STEP << 16) : 0u) | ((cur & (HOT & 0xFFFFu)) ? STEP : 0u);
        uint32_t seen = cur;
        if (__hip_atomic_compare_exchange_strong(p, &seen, cur - sub, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
            const bool single = a >= PB;
            const uint32_t w = (single ? a - PB : a) >> 2;
            for (uint32_t h = 0; h < 2; ++h) {
                if (!((sub >> (16 * h)) & 0xFFFFu)) continue;
                const uint32_t bin = 2 * w + h;
                if (K == 8 || single) {
                    atomicAdd(gcounts + code2col[bin], STEP);
                } else {
                    atomicAdd(gcounts + code2col[bin >> 2], STEP);                      // older k-mer
                    atomicAdd(gcounts + code2col[bin & ((1u << (2 * K)) - 1u)], STEP);  // newer k-mer
                }
            }
            cur -= sub;
        } else {
            cur = seen;
        }
    }
}
// Drain every hot word of P (and S) -- one wave, the whole table.
template <int K>
__device__ __noinline__ void x_scan_drain(const uint32_t* __restrict__ code2col, uint32_t* gcounts, int lane) {
    constexpr uint32_t HOT = x_hot<K>();
    for (uint32_t w = (uint32_t)lane; w < (K >= 8 ? XL<K>::P : XL<K>::bytes) / 4; w += kWave) {
        const uint32_t v = __hip_atomic_load((lds_u32*)(uintptr_t)(4 * w), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        if (v & HOT) x_drain<K>(4 * w, code2col, gcounts);
    }
}

// Classification per dword x (4 bytes), no per-byte newline compare:
//   s  = x & 7 per byte: A/a 1, C/c 3, T/t 4, G/g 7, '\n' 2 (distinct)
//   e  = kXTab[s] (one v_perm): the lowercase base, 0x0B for '\n', and values
//        whose low three bits differ from s elsewhere
//   z  = bitop3(x, e, 0xDF..): bits other than 5 as x ^ e, bit 5 as x & ~e, so a
//        base of either case gives 0 (e has bit 5 set: case ignored), '\n' gives
//        exactly 1 ('*', which folds onto '\n', gives 0x21), and every other
//        byte a value outside {0, 1}
//   codes: (x & 6) = 2 x code (A0 C1 T2 G3), packed by v_dot4 (the factor two
//   drops out of the shifts that merge four of them).
constexpr uint32_t kXTabLo = 0x630B6102u;   // e0..e3 = 0x02, 'a', 0x0B, 'c'
constexpr uint32_t kXTabHi = 0x67000074u;   // e4..e7 = 't', 0x00, 0x00, 'g'

struct XBlock {
    uint4 q[3];   // lane L: bytes [16L + 1024 i, 16L + 1024 i + 16) of the 3 KiB iteration
};
// z = bits other than 5 (c = 1): x ^ e; bit 5 (c = 0): x & ~e  (one v_bitop3)
__device__ __forceinline__ uint32_t x_zmap(uint32_t x, uint32_t e, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x38" : "=v"(r) : "v"(x), "v"(e), "v"(c));
    return r;
}

// ---------------------------------------------------------------- K1x, coalesced layout
// The 3 KiB iteration is read as three 1 KiB regions, lane L holding
// bytes [16L, 16L+16) of each, so every load instruction reads 1 KiB contiguous,
// with the non-temporal cache policy.  Measured streaming rate of the two layouts
// (tools/cpol_rate.hip, profiles/r03/v8_cpol_rate.txt): 6.8 TB/s coalesced + nt vs
// 5.6-5.8 TB/s for rounds 1-2's 48-byte lanes, which the nt bit slows to 4.5.  Windows are
// formed and paired per 16-byte region: a lane holds 16 entries (15 with a
// newline), the k-1 entries of context come from lane L-1's region by DPP, lane
// 0 takes the previous region's lane 63.
#ifndef KF_NT_STORES
#define KF_NT_STORES 1   // non-temporal count-row stores (k=7 -1.4 %; v10_lib_ab_k*_nt_stores)
#endif
constexpr int kXNt = 2;   // buffer-load cache policy bit: non-temporal

__device__ __forceinline__ XBlock xc_load(const uint8_t* bytes, uint64_t c0, uint32_t rel, uint32_t end_r, int lane) {
    // clamped to the genome end rounded up to 16 B (load_chunk): bytes past it read 0
    const uint32_t rec = end_r > rel ? min(end_r - rel, (uint32_t)kXChunk) : 0u;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + c0 + rel), (short)0, (int)rec, 0x00020000);
    XBlock b;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + kChunk * i, 0, kXNt);
        b.q[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    return b;
}

// dot4 weights of dword i of a 16-byte region in its newline test: byte b = 4i + t
// weighs 2 (32 - b), so V = 0 without a newline, 34 + 2e for one newline at entry
// e = 15 - b (<= 64), and >= 68 otherwise (every further nonzero z adds >= 34, a
// bad byte's z >= 2)
__device__ __forceinline__ constexpr uint32_t xc_nl_weights(int i) {
    return (uint32_t)(64 - 8 * i) | (uint32_t)(62 - 8 * i) << 8 | (uint32_t)(60 - 8 * i) << 16 |
           (uint32_t)(58 - 8 * i) << 24;
}
constexpr uint32_t kXcBad = 68u;   // V at or above: not the fast case

// One region's codes (entry 0 = byte 15) and newline / bad-byte sum: per dword,
// the v_perm table lookup and x_zmap above give z, one v_dot4 per dword packs
// the codes and another sums z weighted by position (xc_nl_weights).
struct XcCls {
    uint32_t C, V;
};
__device__ __forceinline__ XcCls xc_cls(const uint4 d) {
    const uint32_t w[4] = {d.x, d.y, d.z, d.w};
    const uint32_t cdf = 0xDFDFDFDFu;
    uint32_t pc[4], z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t x = w[i];
        const uint32_t e = __builtin_amdgcn_perm(kXTabHi, kXTabLo, x & 0x07070707u);
        z[i] = x_zmap(x, e, cdf);
        pc[i] = __builtin_amdgcn_udot4(x & 0x06060606u, 0x01041040u, (i & 1) ? pc[i - 1] << 8 : 0u, false);
    }
    XcCls r;
    r.C = (pc[1] << 15) | (pc[3] >> 1);
    r.V = __builtin_amdgcn_udot4(z[1], xc_nl_weights(1), __builtin_amdgcn_udot4(z[0], xc_nl_weights(0), 0u, false),
                                 false) +
          __builtin_amdgcn_udot4(z[3], xc_nl_weights(3), __builtin_amdgcn_udot4(z[2], xc_nl_weights(2), 0u, false),
                                 false);
    return r;
}

// A region's window register W after the newline entry is removed: the lane's
// 16 - nl entries c, lane L-1's entries pC above them (lane 0: lane 63 of the
// previous region, passed as `rot`, a register whose lane 0 holds it).  Returned
// as two views of X = W << 1: x0 = X bits 0..31, y0 = X bits 16..47 (pair and
// window addresses are plain shifts and masks of them), c (for the half masks,
// W bits 0..31 where they are read) and nl.
struct XcWin {
    uint32_t x0, y0, c, nl;
};
__device__ __forceinline__ XcWin xc_window(const XcCls& k, uint32_t rot) {
    uint32_t nl;   // min(V, 1), opaque: the compiler would turn its uses into selects (v_cndmask)
    asm("v_min_u32_e32 %0, 1, %1" : "=v"(nl) : "v"(k.V));
    const uint32_t q = min(k.V - 34u, 32u);   // 2e; no newline: wraps high, 32
    const uint32_t L = (uint32_t)(~0ull << q);
    const uint32_t c = bfi(L, k.C >> 2, k.C);
    const uint32_t pC = wave_shr1(rot, c);
    // W = c | pC << (32 - 2 nl) (64-bit), so X = W << 1 has
    // x0 = c << 1 | (nl ? pC << 31 : 0), y0 = c >> 15 | pC << (17 - 2 nl)
    XcWin x;
    x.x0 = (c << 1) | ((pC << 31) & (0u - nl));
    x.y0 = (c >> 15) | (pC << (17u - 2u * nl));
    x.c = c, x.nl = nl;
    return x;
}
// wave_ror:1 (lane 0 gets lane 63)
__device__ __forceinline__ uint32_t wave_ror1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x13C, 0xF, 0xF, false);
}

// k <= 7 adds of one region: pair j = windows 2j (newer) and 2j+1, the (k+1)-mer at
// bits [4j, 4j+2k+2) of W; with a newline window 14 is left alone and goes to S.
// Word addresses: P (k+1)-mer code x at (x >> 1) << 2 = (x << 1) & ~3, i.e. the
// bits [4j, 4j+2k+3) of X = W << 1 masked by PM; an S k-mer likewise with SM.
template <int K>
__device__ __forceinline__ void xc_pairs(const XcWin& x, uint32_t (&rt)[8]) {
    static_assert(K >= 2 && K <= 7, "pairs of k-mers: k <= 7");
    constexpr uint32_t PM = (1u << (2 * K + 3)) - 4u, SM = (1u << (2 * K + 1)) - 4u;
    const uint32_t one = 1u;
    const uint32_t x0 = x.x0, y0 = x.y0;
    const uint32_t H0 = (x.c << 4) & 0x10101010u, H1 = x.c & 0x10101010u;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        const uint32_t a = ((j < 4 ? x0 : y0) >> (4 * (j & 3))) & PM;
        const uint32_t H = (j & 1) ? H1 : H0;
        uint32_t dl;
        switch (j >> 1) {
        case 0: dl = shl1_byte<0>(H, one); break;
        case 1: dl = shl1_byte<1>(H, one); break;
        case 2: dl = shl1_byte<2>(H, one); break;
        default: dl = shl1_byte<3>(H, one); break;
        }
        rt[j] = lds_add_rtn(a, dl);
    }
    const uint32_t v = y0 >> 12;
    const uint32_t a7 = bfi(0u - x.nl, XL<K>::P | (v & SM), v & PM);
    rt[7] = lds_add_rtn(a7, shl1_byte<3>(H1, one));
}

// k = 8 adds of one region: window r = the 8-mer at bits [2r, 2r+16) of W, r < 16 - nl.
__device__ __forceinline__ void xc_wins8(const XcWin& x, uint32_t (&rt)[16]) {
    constexpr uint32_t PM = 0x1FFFCu;
    const uint32_t one = 1u;
    const uint32_t x0 = x.x0, y0 = x.y0, w0 = x.c;
    const uint32_t keep15 = x.nl - 1u;   // 0 with a newline: window 15 is lane L-1's window 0
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t a = ((r < 8 ? x0 : y0) >> (2 * (r & 7))) & PM;
        const int tb = r & 3;   // W bit 2r sits at bit 8m + 2tb of w0 (m = r >> 2): move it to 8m + 4
        const uint32_t H = (tb == 0 ? w0 << 4 : (tb == 1 ? w0 << 2 : (tb == 2 ? w0 : w0 >> 2))) & 0x10101010u;
        uint32_t dl;
        switch (r >> 2) {
        case 0: dl = shl1_byte<0>(H, one); break;
        case 1: dl = shl1_byte<1>(H, one); break;
        case 2: dl = shl1_byte<2>(H, one); break;
        default: dl = shl1_byte<3>(H, one); break;
        }
        if (r == 15) dl &= keep15;
        rt[r] = lds_add_rtn(a, dl);
    }
}

// ---------------------------------------------------------------- K9b, the window register
// A region's window register for k = 9 (as xc_window): W = c | pC << (32 - 2 nl)
// as a 64-bit value, window r = bits [2r, 2r + 18), r < 16 - nl.
struct K9Win {
    uint32_t c, nl, wlo, whi;
};
__device__ __forceinline__ K9Win k9_window(const XcCls& k, uint32_t rot) {
    uint32_t nl;
    asm("v_min_u32_e32 %0, 1, %1" : "=v"(nl) : "v"(k.V));
    const uint32_t q = min(k.V - 34u, 32u);
    const uint32_t L = (uint32_t)(~0ull << q);
    const uint32_t c = bfi(L, k.C >> 2, k.C);
    const uint32_t pC = wave_shr1(rot, c);
    K9Win x;
    x.c = c, x.nl = nl;
    x.wlo = c | ((pC << 30) & (0u - nl));   // (c's top entry is 0 after a newline)
    x.whi = pC >> (2u * nl);
    return x;
}

// ---------------------------------------------------------------- K9b (k = 9, the product)
// All 131,072 classes as u8 counters in LDS (class index i at byte i: word
// i >> 2, byte i & 3; 128 KiB), one pass, no staging.  A byte wraps every 256
// adds; the carry then runs into the bytes above it in the word.  Every add
// returns the word's old value and is atomic, so the lane whose add carries
// sees it exactly: a byte b at 0xFF before the add means class b wrapped (+256
// to its row column) and byte b+1 got a carry that is no count of its class
// (-1), which wraps in turn if it was at 0xFF (+256, carry on), up to byte 3
// (the carry out of the word is lost).  Those corrections go to the count row
// by global atomics (once per 256 adds of a class at most), the LDS bytes keep
// the counts mod 256, and the flush adds them.  Per window: the class, one LDS
// add, and a two-op check of its return (the byte's old value is 0xFF) folded
// into one max per region; only a region with a wrap walks its windows again.
// Class index (17 bits) of window r of the window register (wlo, whi), whose
// reverse complement is (rlo, rhi).
__device__ __forceinline__ uint32_t k9_index(uint32_t wlo, uint32_t whi, uint32_t rlo, uint32_t rhi, int r) {
    const uint32_t y = r < 8 ? wlo >> (2 * r) : __builtin_amdgcn_alignbit(whi, wlo, 2 * r);
    const uint32_t rc = r < 8 ? rhi >> (14 - 2 * r) : __builtin_amdgcn_alignbit(rhi, rlo, 46 - 2 * r);
    const uint32_t c = bfi((uint32_t)__builtin_amdgcn_sbfe((int)y, 9u, 1u), rc, y);
    return bfi(0x1FFu, c, c >> 1) & 0x1FFFFu;
}

// The exact carry corrections of one region (rare: out of line, so its
// registers do not weigh on the counting loop).  Returns 1 if any lane made one.
__device__ __noinline__ uint32_t k9b_carries(uint32_t wlo, uint32_t whi, const uint32_t* __restrict__ code2col,
                                             uint32_t* gcounts, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                             uint32_t w4, uint32_t w5, uint32_t w6, uint32_t w7, uint32_t w8,
                                             uint32_t w9, uint32_t w10, uint32_t w11, uint32_t w12, uint32_t w13,
                                             uint32_t w14, uint32_t w15) {
    const uint32_t rlo = revpairs(whi) ^ 0xAAAAAAAAu, rhi = revpairs(wlo) ^ 0xAAAAAAAAu;
    const uint32_t rt[16] = {w0, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11, w12, w13, w14, w15};
    uint32_t fixed = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t w = rt[r], ki = k9_index(wlo, whi, rlo, rhi, r), b = ki & 3u;
        if (((w >> (8 * b)) & 0xFFu) != 0xFFu) continue;   // (a window not counted has w = 0)
        const uint32_t base = ki & ~3u;
        fixed = 1;
        atomicAdd(gcounts + code2col[k9_code_of(base | b)], 256u);
        for (uint32_t j = b + 1; j < 4; ++j) {   // the carry into byte j
            const uint32_t col = code2col[k9_code_of(base | j)];
            const bool wraps = ((w >> (8 * j)) & 0xFFu) == 0xFFu;
            atomicAdd(gcounts + col, wraps ? 255u : 0xFFFFFFFFu);   // -1, +256 if it wrapped too
            if (!wraps) break;
        }
    }
    return __builtin_amdgcn_ballot_w64(fixed != 0) != 0 ? 1u : 0u;
}

template <bool DENSE>
__device__ __forceinline__ uint32_t k9b_region(uint32_t wlo, uint32_t whi, uint32_t R, const CountArgs& A,
                                               uint32_t* gcounts) {
    const uint32_t rlo = revpairs(whi) ^ 0xAAAAAAAAu, rhi = revpairs(wlo) ^ 0xAAAAAAAAu;
    uint32_t rt[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t ki = k9_index(wlo, whi, rlo, rhi, r);
        rt[r] = 0;   // (a window not counted: no byte of 0 is 0xFF)
        const bool v = (DENSE && r < 15) || ((R >> r) & 1u);
        if (v) rt[r] = lds_add_rtn(ki & 0x1FFFCu, 1u << ((ki << 3) & 24u));
    }
    // any byte of an old word at 0xFF (its add may have carried): ~(w + 0x01..)
    // & w has bit 7 of byte j set iff byte j of w is 0xFF (a borrow-free test);
    // another class's byte at 0xFF only sends the region down the exact path
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc |= ~(rt[r] + 0x01010101u) & rt[r];
    if (__builtin_amdgcn_ballot_w64((acc & 0x80808080u) != 0) == 0) return 0;
    return k9b_carries(wlo, whi, A.code2col, gcounts, rt[0], rt[1], rt[2], rt[3], rt[4], rt[5], rt[6], rt[7], rt[8],
                       rt[9], rt[10], rt[11], rt[12], rt[13], rt[14], rt[15]);
}

// Fast case of a coalesced 3 KiB iteration (uniform): every region of every lane
// is bases with at most one newline and the carry is complete; returns false
// (nothing counted) otherwise.  u16 exactness: every add's return is checked at
// the end of its iteration; after a half crosses HOT's threshold, every wave adds
// at most one more iteration to it before its own drain.  k = 7: at most 24 x 64
// adds per wave and iteration, so a half stays below 0x4000 + 16 x 1536 = 0xA000;
// k = 8: 48 x 64, below 0x2000 + 16 x 3072 = 0xE000.
template <int K>
__device__ __forceinline__ bool xc_fast(const XBlock& d, const CountArgs& A, int lane, uint32_t& carry,
                                        uint32_t* gcounts, uint32_t& lane_total, uint32_t& drained) {
    constexpr uint32_t HOT = x_hot<K>();
    constexpr uint32_t TM = (1u << (2 * (K - 1))) - 1u;
    const XcCls k0 = xc_cls(d.q[0]), k1 = xc_cls(d.q[1]), k2 = xc_cls(d.q[2]);
    carry = __builtin_amdgcn_readfirstlane(carry);
    if (t_n(carry) < (uint32_t)(K - 1) || __builtin_amdgcn_ballot_w64(max(max(k0.V, k1.V), k2.V) >= kXcBad) != 0)
        return false;
    if constexpr (K == 9) {
        // K9b: each region's window register, then its 16 windows (window 15 of
        // a region with a newline belongs to lane L-1's region: not counted); no
        // drains (byte carries are corrected as they happen)
        const K9Win x0 = k9_window(k0, t_codes(carry));
        uint32_t f = k9b_region<true>(x0.wlo, x0.whi, 0xFFFFu >> x0.nl, A, gcounts);
        const K9Win x1 = k9_window(k1, wave_ror1(x0.c));
        f |= k9b_region<true>(x1.wlo, x1.whi, 0xFFFFu >> x1.nl, A, gcounts);
        const K9Win x2 = k9_window(k2, wave_ror1(x1.c));
        f |= k9b_region<true>(x2.wlo, x2.whi, 0xFFFFu >> x2.nl, A, gcounts);
        lane_total -= x0.nl + x1.nl + x2.nl;
        carry = tail_pack((uint32_t)__builtin_amdgcn_readlane((int)x2.c, kWave - 1) & TM, 31u, 31u);
        drained |= f;   // (K9b: a carry was corrected in the row)
        return true;
    }
    uint32_t o = 0;
    const XcWin x0 = xc_window(k0, t_codes(carry));
    const XcWin x1 = xc_window(k1, wave_ror1(x0.c));
    const XcWin x2 = xc_window(k2, wave_ror1(x1.c));
    if constexpr (K <= 7) {
        const XcWin* xs[3] = {&x0, &x1, &x2};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            uint32_t r[8];
            xc_pairs<K>(*xs[i], r);
#pragma unroll
            for (int j = 0; j < 8; j += 4) o |= r[j] | r[j + 1] | r[j + 2] | r[j + 3];
        }
    } else {
        const XcWin* xs[3] = {&x0, &x1, &x2};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            uint32_t r[16];
            xc_wins8(*xs[i], r);
#pragma unroll
            for (int j = 0; j < 16; j += 4) o |= r[j] | r[j + 1] | r[j + 2] | r[j + 3];
        }
    }
    lane_total -= x0.nl + x1.nl + x2.nl;   // + 48 per fast iteration, added by the caller
    carry = tail_pack((uint32_t)__builtin_amdgcn_readlane((int)x2.c, kWave - 1) & TM, 31u, 31u);
    if (__builtin_amdgcn_ballot_w64((o & HOT) != 0) != 0) {
        x_scan_drain<K>(A.code2col, gcounts, lane);
        drained = 1;
    }
    return true;
}

// Irregular 1 KiB chunk (16-byte lane layout, the general front end): every
// counted window as a single by its forward code -- into S (k = 7) or P
// (k = 8) -- with its return checked at once.
template <int K, bool MASKED>
__device__ __forceinline__ uint32_t x_singles(const uint4 d, const CountArgs& A, uint64_t chunk, int lane,
                                              const ChunkMask& m, uint64_t iv0, uint32_t carry, uint32_t* gcounts,
                                              uint32_t& lane_total, uint32_t& drained) {
    constexpr uint32_t HOT = x_hot<K>();
    uint32_t C, V, EN, ne, own;
    front_end<K, MASKED, false>(d, A, chunk, lane, m, iv0, C, V, EN, ne, own);
    const Windows win = windows<K, MASKED>(C, V, EN, ne, carry, lane);
    const uint32_t wlo = win.wlo, whi = win.whi, R = win.R;
    if constexpr (K == 9) {   // K9b: every counted window through the k = 9 region step
        drained |= k9b_region<false>(wlo, whi, R, A, gcounts);
        lane_total += (uint32_t)__builtin_popcount(R);
        return win.next;
    }
    const uint32_t wv[4] = {wlo, __builtin_amdgcn_alignbit(whi, wlo, 8), __builtin_amdgcn_alignbit(whi, wlo, 16),
                            __builtin_amdgcn_alignbit(whi, wlo, 24)};
    uint32_t o = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int fo = (2 * r) & ~7;
        const uint32_t y = __builtin_amdgcn_ubfe(wv[fo >> 3], 2 * r - fo, 2 * K);
        o |= lds_add_rtn((K == 8 ? 0u : XL<K>::P) + ((y >> 1) << 2), ((R >> r) & 1u) * half_one(y));
    }
    if (__builtin_amdgcn_ballot_w64((o & HOT) != 0) != 0) {
        x_scan_drain<K>(A.code2col, gcounts, lane);
        drained = 1;
    }
    lane_total += (uint32_t)__builtin_popcount(R);
    return win.next;
}

// The wave range [lo, hi) of genome [glo, ghi) in 3 KiB iterations (K1x).
// `drained` is set if a u16 half of this range was moved to the count row (the
// flush then adds with atomics).
template <int K>
__device__ __forceinline__ uint32_t x_range(const CountArgs& A, int32_t g, uint64_t glo, uint64_t ghi, uint64_t lo,
                                            uint64_t hi, int lane, uint32_t& drained) {
    if (lo >= hi) return 0;
    uint32_t* gcounts = A.counts + (uint64_t)g * A.nbins;
    Range rg;
    rg.init(glo, ghi, lo, hi);
    auto load = [&](uint32_t r) {
        return xc_load(A.bytes, rg.c0, r, rg.end_r, lane);
    };
    // k <= 8: the ring as an array the compiler unrolls into registers; k = 9's
    // step is too large for that unroll, so its ring is two named blocks (an
    // array it cannot unroll would be indexed in scratch memory)
    static_assert(kXRing == 2, "two-deep register ring");
    XBlock buf[K == 9 ? 1 : kXRing];
    XBlock b0, b1;
    if constexpr (K == 9) {
        b0 = load(0);
        b1 = load(kXChunk);
    } else {
#pragma unroll
        for (int j = 0; j < kXRing; ++j) buf[j] = load(j * kXChunk);
    }
    const uint32_t nx = (rg.nch + 2) / 3;   // 3 KiB iterations
    rg.warm16<K>(A, lane);
    __builtin_amdgcn_s_setprio(0);   // (the setup ran at top priority, see k1x_kernel)
    uint32_t carry = rg.carry;
    uint32_t rel = 0;
    const ChunkMask m = rg.mask();
    uint32_t lane_total = 0;
    uint32_t nfast = 0;   // fast iterations (wave-uniform): 48 windows per lane each, less its newlines
    auto step = [&](const XBlock& bf) {
        // one test for the whole 3 KiB (range edges, excluded intervals)
        bool fast = !rg.masked_span(A, rel, kXChunk);
        if (fast)
            fast = xc_fast<K>(bf, A, lane, carry, gcounts, lane_total, drained);
        nfast += fast ? 1u : 0u;
        if (!fast) {
            // interval cursor before each 1 KiB third (a later test may advance it)
            const bool m0 = rg.masked(A, rel);
            const uint64_t iv0 = rg.iv;
            const bool m1 = rg.masked(A, rel + kChunk);
            const uint64_t iv1 = rg.iv;
            const bool m2 = rg.masked(A, rel + 2 * kChunk);
            // irregular: the three 1 KiB thirds in 16-byte lane layout, singles
#pragma unroll
            for (int h = 0; h < 3; ++h) {
                const uint32_t r = rel + h * kChunk;
                if (h > 0 && r >= rg.nch * kChunk) break;
                const bool mh = h == 0 ? m0 : (h == 1 ? m1 : m2);
                const uint64_t ivh = h == 0 ? iv0 : (h == 1 ? iv1 : rg.iv);
                // the coalesced block already holds this third in the 16-byte lane layout
                const uint4 hb = bf.q[h];
                if (mh)
                    carry = x_singles<K, true>(hb, A, rg.c0 + r, lane, m, ivh, carry, gcounts, lane_total, drained);
                else
                    carry = x_singles<K, false>(hb, A, rg.c0 + r, lane, m, ivh, carry, gcounts, lane_total, drained);
            }
        }
        rel += kXChunk;
    };
    if constexpr (K == 9) {
        for (uint32_t i = 0; i + 2 <= nx; i += 2) {
            step(b0);
            b0 = load(rel + kXChunk);
            step(b1);
            b1 = load(rel + kXChunk);
        }
        if (nx & 1u) step(b0);
    } else {
        for (uint32_t i = 0; i + kXRing <= nx; i += kXRing) {
#pragma unroll
            for (int j = 0; j < kXRing; ++j) {
                step(buf[j]);
                buf[j] = load(rel + (kXRing - 1) * kXChunk);
            }
        }
        const uint32_t rem = nx % kXRing;
#pragma unroll
        for (int j = 0; j < kXRing - 1; ++j)
            if (rem > (uint32_t)j) step(buf[j]);
    }
    return lane_total + 48u * nfast;
}

// F(y) word in the k = 7 flush: bits 1-4 XOR bits 8-11.  A wave reads F at 64
// representatives y that differ in their low bases and at their reverse
// complements, which then differ only in bits 8-13: unswizzled, every rc read
// of a wave would hit one bank.  Bit 0 is kept, so F(2m), F(2m+1) stay a pair.
__device__ __forceinline__ uint32_t f_swz(uint32_t y) { return y ^ (((y >> 8) & 15u) << 1); }
__device__ __forceinline__ uint32_t u16sum2(uint32_t w) { return (w & 0xFFFFu) + (w >> 16); }

// k = 7 flush step 1 (1024 threads): per forward 7-mer y, F(y) = sum_a P[4y + a]
// (y as the older window of a pair) + sum_a P[a 4^7 + y] (as the newer one);
// thread t owns y = 2048 i + 2t + {0, 1}, i = 0..7 (lane-consecutive reads).
__device__ __forceinline__ void pair_f_sums(const uint32_t* hist, int tid, uint32_t (&F)[16]) {
    const uint4* h4 = (const uint4*)hist;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint4 w = h4[i * 1024 + tid];   // words 2y .. 2y+3 of y = 2048 i + 2 tid
        F[2 * i] = u16sum2(w.x) + u16sum2(w.y);
        F[2 * i + 1] = u16sum2(w.z) + u16sum2(w.w);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const uint32_t v = hist[a * 8192 + i * 1024 + tid];   // halves a 4^7 + y, a 4^7 + y + 1
            F[2 * i] += v & 0xFFFFu;
            F[2 * i + 1] += v >> 16;
        }
    }
}

// k <= 6 flush (1024 threads): F(y) for the 4^k forward k-mers, thread t owning
// y = t + 1024 m: sum_a P[4y + a] (two words) + sum_a P[a 4^k + y] + S[y].
template <int K>
__device__ __forceinline__ void pair_f_sums_small(const uint32_t* hist, int tid,
                                                  uint32_t (&F)[((1u << (2 * K)) + kBlock - 1) / kBlock]) {
    constexpr uint32_t NY = 1u << (2 * K), NM = (NY + kBlock - 1) / kBlock;
#pragma unroll
    for (uint32_t m = 0; m < NM; ++m) {
        const uint32_t y = (uint32_t)tid + kBlock * m;
        F[m] = 0;
        if (y < NY) {
            const uint32_t sh = (y & 1u) << 4;
            uint32_t f = u16sum2(hist[2 * y]) + u16sum2(hist[2 * y + 1]);   // y older: P[4y .. 4y + 3]
#pragma unroll
            for (uint32_t a = 0; a < 4; ++a) f += (hist[a * (NY / 2) + (y >> 1)] >> sh) & 0xFFFFu;   // y newer
            f += (hist[XL<K>::P / 4 + (y >> 1)] >> sh) & 0xFFFFu;                                    // single
            F[m] = f;
        }
    }
}

template <int K>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4, 4))) k1x_kernel(CountArgs A) {
    static_assert(K >= 2 && K <= 9, "K1x serves k = 2 .. 9 (k = 9: K9b byte counters)");
    // P and S (the whole dynamic LDS, at address 0: see lds_add); no LDS is left
    // for reduction slots, so totals go straight to global atomics
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    {
        uint4* h4 = (uint4*)hist;
        for (uint32_t i = tid; i < XL<K>::bytes / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
    if ((uint32_t)(uintptr_t)(lds_u32*)hist != 0u) __builtin_trap();   // lds_add assumes base 0
    uint64_t span_lo, span_hi;
    wg_span(A, span_lo, span_hi);
    if (span_lo >= span_hi) return;
    int32_t g = (int32_t)wave_upper_bound((uint64_t)A.n_genomes, span_lo, lane,
                                          [&](uint64_t i) { return A.goff[i + 1]; });
    const uint32_t fr_lo = wave_frac((uint32_t)wave, kWaveWeights), fr_hi = wave_frac((uint32_t)wave + 1, kWaveWeights);
    for (; g < A.n_genomes; ++g) {
        // a piece's setup (bounds, interval search, warm-up: dependent loads) at
        // top priority, so the youngest wave slots do not start late
        __builtin_amdgcn_s_setprio(3);
        const uint64_t glo = A.goff[g], ghi = A.goff[g + 1];
        if (glo >= span_hi) break;
        const uint64_t plo = max(glo, span_lo), phi = min(ghi, span_hi);
        if (phi <= plo) continue;
        const uint64_t lo = split_at_frac(plo, phi, fr_lo), hi = split_at_frac(plo, phi, fr_hi);
        uint32_t drained = 0;   // plain row stores unless a half was drained
        unsigned long long s = x_range<K>(A, g, glo, ghi, lo, hi, lane, drained);
        uint32_t* gc = A.counts + (uint64_t)g * A.nbins;
        // A whole genome in this span (the common case) with no drained half: no
        // other workgroup and nothing else touches row g, which the caller
        // zeroed, so it is written with plain stores; otherwise atomics.
        const bool whole = plo == glo && phi == ghi && !(A.flags & KF_ACCUMULATE);
        if constexpr (K == 9) {
            // every column in order (coalesced row writes): its class's byte;
            // rows with carry corrections (already added to them) take atomics
            lds_barrier();   // every add of this piece is done
            if (lane == 0) hist[XL<K>::P / 4 + wave] = drained;
            lds_barrier();
            const uint4* fl = (const uint4*)(hist + XL<K>::P / 4);
            const uint4 f0 = fl[0], f1 = fl[1], f2 = fl[2], f3 = fl[3];
            const bool any_fix = (f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w | f2.x | f2.y | f2.z |
                                  f2.w | f3.x | f3.y | f3.z | f3.w) != 0;
            const uint8_t* hb = (const uint8_t*)hist;
            for (uint32_t c0 = (uint32_t)tid; c0 < (1u << 17); c0 += 4 * kBlock) {
                uint32_t rep[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) rep[j] = A.col2rep[c0 + j * kBlock];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t c = (rep[j] & 0x200u) ? kf_revcomp<9>(rep[j]) : rep[j];
                    const uint32_t v = hb[((c >> 1) & 0x1FE00u) | (c & 0x1FFu)];
                    if (whole && !any_fix)
                        __builtin_nontemporal_store(v, gc + c0 + j * kBlock);
                    else if (v)
                        __hip_atomic_fetch_add(gc + c0 + j * kBlock, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            lds_barrier();   // bytes read
            uint4* h4 = (uint4*)hist;
            for (uint32_t i = tid; i < XL<K>::bytes / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
        } else if constexpr (K == 8) {
            // canonical 8-mer column = P[rep] + P[rc rep] (a palindrome once);
            // drain flags in the (unused) S area
            lds_barrier();   // every add of this piece is done
            if (lane == 0) hist[XL<K>::P / 4 + wave] = drained;
            lds_barrier();
            const uint4* fl = (const uint4*)(hist + XL<K>::P / 4);
            const uint4 f0 = fl[0], f1 = fl[1], f2 = fl[2], f3 = fl[3];
            const bool any_drain = (f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w | f2.x | f2.y | f2.z |
                                    f2.w | f3.x | f3.y | f3.z | f3.w) != 0;
            for (uint32_t col = tid; col < A.nbins; col += kBlock) {
                const uint32_t y = A.col2rep[col], rc = kf_revcomp<8>(y);
                uint32_t v = (hist[y >> 1] >> ((y & 1u) << 4)) & 0xFFFFu;
                if (rc != y) v += (hist[rc >> 1] >> ((rc & 1u) << 4)) & 0xFFFFu;
                if (whole && !any_drain)
                    gc[col] = v;
                else if (v)
                    __hip_atomic_fetch_add(gc + col, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            lds_barrier();   // columns read
            uint4* h4 = (uint4*)hist;
            for (uint32_t i = tid; i < XL<K>::bytes / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
        } else if constexpr (K <= 6) {
            // canonical column = F(rep) + F(rc rep) (a palindrome once, even k);
            // F = pair and single sums (pair_f_sums_small), back in LDS words
            // [0, 4^k) (swizzled as f_swz), the drain flags after them
            constexpr uint32_t NY = 1u << (2 * K), NM = (NY + kBlock - 1) / kBlock;
            constexpr uint32_t NCOL = (NY + (K % 2 == 0 ? (1u << K) : 0u)) / 2, NC = (NCOL + kBlock - 1) / kBlock;
            uint32_t rep[NC];
#pragma unroll
            for (uint32_t c = 0; c < NC; ++c) {
                const uint32_t col = (uint32_t)tid + c * kBlock;
                rep[c] = col < NCOL ? A.col2rep[col] : 0u;
            }
            lds_barrier();   // every add of this piece is done
            uint32_t F[NM];
            pair_f_sums_small<K>(hist, tid, F);
            lds_barrier();   // P and S read
#pragma unroll
            for (uint32_t m = 0; m < NM; ++m) {
                const uint32_t y = (uint32_t)tid + kBlock * m;
                if (y < NY) hist[f_swz(y)] = F[m];
            }
            if (lane == 0) hist[NY + wave] = drained;   // (P holds 2 x 4^k words: past F is free)
            lds_barrier();   // F in LDS words [0, 4^k), drain flags after it
            const uint4* fl = (const uint4*)(hist + NY);
            const uint4 f0 = fl[0], f1 = fl[1], f2 = fl[2], f3 = fl[3];
            const bool any_drain = (f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w | f2.x | f2.y | f2.z | f2.w |
                                    f3.x | f3.y | f3.z | f3.w) != 0;
            uint32_t cv[NC];
#pragma unroll
            for (uint32_t c = 0; c < NC; ++c) {
                const uint32_t y = rep[c], rc = kf_revcomp<K>(y);
                cv[c] = hist[f_swz(y)] + (rc != y ? hist[f_swz(rc)] : 0u);
            }
            lds_barrier();   // columns read
            uint4* h4 = (uint4*)hist;
            for (uint32_t i = tid; i < XL<K>::bytes / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (uint32_t c = 0; c < NC; ++c) {
                const uint32_t col = (uint32_t)tid + c * kBlock;
                if (col >= NCOL) continue;
                if (whole && !any_drain)
                    __builtin_nontemporal_store(cv[c], gc + col);
                else if (cv[c])
                    __hip_atomic_fetch_add(gc + col, cv[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            // the columns' forward representatives, loaded before the barrier so
            // their latency overlaps it.  A whole genome takes four consecutive
            // columns per lane and 16-byte row stores (the flush is bound by the
            // CU's store issue); other pieces one column per lane and atomics.
            uint32_t rep[8];
            if (whole) {
                const uint4 r0 = *(const uint4*)(A.col2rep + 4 * tid), r1 = *(const uint4*)(A.col2rep + 4096 + 4 * tid);
                rep[0] = r0.x, rep[1] = r0.y, rep[2] = r0.z, rep[3] = r0.w;
                rep[4] = r1.x, rep[5] = r1.y, rep[6] = r1.z, rep[7] = r1.w;
            } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) rep[c] = A.col2rep[tid + c * kBlock];
            }
            lds_barrier();   // every add of this piece is done
            uint32_t F[16];
            pair_f_sums(hist, tid, F);
#pragma unroll
            for (int i = 0; i < 8; ++i) {   // singles of y = 2048 i + 2 tid + {0, 1}
                const uint32_t v = hist[XL<K>::P / 4 + i * 1024 + tid];
                F[2 * i] += v & 0xFFFFu;
                F[2 * i + 1] += v >> 16;
            }
            lds_barrier();   // P and S read
#pragma unroll
            for (int i = 0; i < 8; ++i) *(uint2*)(hist + f_swz(i * 2048 + 2 * tid)) = make_uint2(F[2 * i], F[2 * i + 1]);
            if (lane == 0) hist[16384 + wave] = drained;   // (words past F are free now)
            lds_barrier();   // F in LDS words [0, 16384), drain flags after it
            const uint4* fl = (const uint4*)(hist + 16384);
            const uint4 f0 = fl[0], f1 = fl[1], f2 = fl[2], f3 = fl[3];
            const bool any_drain = (f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w | f2.x | f2.y | f2.z | f2.w |
                                    f3.x | f3.y | f3.z | f3.w) != 0;
            uint32_t cv[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t y = rep[c], rc = kf_revcomp<7>(y);
                cv[c] = hist[f_swz(y)] + hist[f_swz(rc)];
            }
            lds_barrier();   // columns read
            uint4* h4 = (uint4*)hist;
            for (uint32_t i = tid; i < XL<K>::bytes / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
            // the row writes last: their issue overlaps the zeroing, the barrier
            // and the next piece's setup
            if (whole && !any_drain) {
#if KF_NT_STORES
                typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(v4u_t{cv[0], cv[1], cv[2], cv[3]}, (v4u_t*)(gc + 4 * tid));
                __builtin_nontemporal_store(v4u_t{cv[4], cv[5], cv[6], cv[7]}, (v4u_t*)(gc + 4096 + 4 * tid));
#else
                *(uint4*)(gc + 4 * tid) = make_uint4(cv[0], cv[1], cv[2], cv[3]);
                *(uint4*)(gc + 4096 + 4 * tid) = make_uint4(cv[4], cv[5], cv[6], cv[7]);
#endif
            } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const uint32_t col = whole ? (c >> 2) * 4096 + 4 * tid + (c & 3) : tid + c * kBlock;
                    if (cv[c]) __hip_atomic_fetch_add(gc + col, cv[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        s = wave_sum(s);
        if (lane == 0 && s) atomicAdd(A.totals + g, s);
        lds_barrier();    // P and S zero before the next piece's adds
    }
}

// ---------------------------------------------------------------- synthetic input
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ bool in_nrun(uint64_t key, uint64_t i, uint64_t n_period) {
    if (!n_period) return false;
    uint64_t b = i >> 12;
    for (int d = 0; d < 2; ++d) {
        if (d == 1) {
            if (b == 0) break;
            b -= 1;
        }
        const uint64_t h = splitmix64((key ^ 0xA5A5A5A5A5A5A5A5ull) + b);
        if (h % n_period) continue;
        const uint64_t st = (b << 12) + ((h >> 16) % 4096), ln = 1 + ((h >> 32) % 100);
        if (i >= st && i < st + ln) return true;
    }
    return false;
}

// Genome gi of the launch (id g0 + gi * gstride) at [goff[gi], goff[gi+1]):
// ">syn_<g>\n", bases in lines of `width`, '\n' padding (oracle_synth_genome).
__global__ void __launch_bounds__(256) synth_kernel(uint8_t* bytes, const uint64_t* goff, int64_t g0, int64_t gstride,
                                                     uint64_t seed0, uint64_t seq_len, int width, uint64_t n_period) {
    const int32_t gi = blockIdx.y;
    const uint64_t lo = goff[gi], hi = goff[gi + 1];
    const int64_t g = g0 + gi * gstride;
    char digits[24];
    int nd = 0;
    {
        uint64_t v = (uint64_t)(g < 0 ? -g : g);
        do { digits[nd++] = (char)('0' + v % 10); v /= 10; } while (v);
    }
    const uint64_t hlen = 5 + (uint64_t)nd + (g < 0 ? 1 : 0) + 1;
    const uint64_t key = splitmix64(seed0 + (uint64_t)g);
    const uint64_t W1 = (uint64_t)width + 1;
    for (uint64_t p0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; lo + p0 < hi;
         p0 += (uint64_t)gridDim.x * blockDim.x * 16) {
        uint32_t out[4] = {0, 0, 0, 0};
        for (int j = 0; j < 16; ++j) {
            const uint64_t p = p0 + j;
            uint32_t ch;
            if (p < hlen) {
                if (p == 0) ch = '>';
                else if (p < 5) ch = "syn_"[p - 1];
                else if (g < 0 && p == 5) ch = '-';
                else if (p == hlen - 1) ch = '\n';
                else ch = (uint32_t)digits[nd - 1 - (int)(p - 5 - (g < 0 ? 1 : 0))];
            } else {
                const uint64_t q = p - hlen, line = q / W1, col = q % W1;
                const uint64_t i = line * (uint64_t)width + col;
                if (col == (uint64_t)width || i >= seq_len) {
                    ch = '\n';
                } else {
                    const uint64_t h = splitmix64(key + (i >> 5));
                    ch = (uint32_t)"ACGT"[(h >> (2 * (i & 31))) & 3];
                    if (in_nrun(key, i, n_period)) ch = 'N';
                }
            }
            out[j >> 2] |= ch << (8 * (j & 3));
        }
        if (lo + p0 + 16 <= hi) {
            *(uint4*)(bytes + lo + p0) = make_uint4(out[0], out[1], out[2], out[3]);
        } else {
            for (int j = 0; lo + p0 + j < hi; ++j) bytes[lo + p0 + j] = (uint8_t)(out[j >> 2] >> (8 * (j & 3)));
        }
    }
}

// ---------------------------------------------------------------- stream probe
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) v ^= (uint32_t)__shfl_xor((int)v, d, kWave);
    return v;
}

// Practical HBM read ceiling for bench.py (measured_ceiling): the fastest read
// pattern measured on this chip (tools/unaligned_rate.hip mode 5, 6.1 TB/s):
// 3 KiB blocks dealt grid-stride over the waves, lane L reading bytes 16 L +
// 1024 q (q = 0..2, coalesced), four blocks in flight per wave; every byte once.
__global__ void __launch_bounds__(1024) stream_probe_kernel(const uint8_t* bytes, uint64_t n, uint32_t* out) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / kWave);
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x >> 6);
    constexpr uint32_t kB = 3 * kChunk;
    const uint64_t nblk = (n + kB - 1) / kB;
    uint32_t acc = 0;
    for (uint64_t b = w; b < nblk; b += 4 * nw) {
        uint4 v[4][3];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t bb = b + (uint64_t)k * nw;
            const uint64_t base = bb < nblk ? bb * kB : 0;
            const int rec = bb < nblk ? (int)min((uint64_t)kB, n - base) : 0;   // past the end: zeros
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + base), (short)0, rec, 0x00020000);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane + 1024 * q, 0, 0);
                v[k][q] = make_uint4(t[0], t[1], t[2], t[3]);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int q = 0; q < 3; ++q) acc ^= v[k][q].x ^ v[k][q].y ^ v[k][q].z ^ v[k][q].w;
    }
    // XOR of every dword (test_stream_probe_xor_fold: each byte read exactly once)
    acc = wave_xor(acc);
    if (lane == 0 && acc) atomicXor(out, acc);
}

}  // namespace kf

// ====================================================================== C-ABI
using namespace kf;

namespace {

void* kernel_for(int k) {
    switch (k) {
    case 2: return (void*)&k1x_kernel<2>;
    case 3: return (void*)&k1x_kernel<3>;
    case 4: return (void*)&k1x_kernel<4>;
    case 5: return (void*)&k1x_kernel<5>;
    case 6: return (void*)&k1x_kernel<6>;
    case 7: return (void*)&k1x_kernel<7>;
    case 8: return (void*)&k1x_kernel<8>;
    case 9: return (void*)&k1x_kernel<9>;
    default: return nullptr;
    }
}

// K1: histogram (4^k u32) + one u64 reduction slot per wave; K1x: P + S
int lds_bytes_for(int k) {
    switch (k) {
    case 2: return (int)XL<2>::bytes;
    case 3: return (int)XL<3>::bytes;
    case 4: return (int)XL<4>::bytes;
    case 5: return (int)XL<5>::bytes;
    case 6: return (int)XL<6>::bytes;
    case 7: return (int)XL<7>::bytes;
    case 8: return (int)XL<8>::bytes;
    default: return (int)XL<9>::bytes;
    }
}


// grid per (k, device): workgroups per CU from the occupancy API x CUs
int g_grid[KF_MAX_K + 1][64];
std::mutex g_grid_mu;

int launch_info(int k, int* grid, int* block, int* lds) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kf_fail(KF_EHIP, "hipGetDevice failed");
    if (dev < 0 || dev >= 64) return kf_fail(KF_EINVAL, "device index out of range");
    const int l = lds_bytes_for(k);
    std::lock_guard<std::mutex> lk(g_grid_mu);
    int& gr = g_grid[k][dev];
    if (!gr) {
        void* fn = kernel_for(k);
        if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, l) != hipSuccess)
            return kf_fail(KF_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, l) != hipSuccess)
            return kf_fail(KF_EHIP, "hipOccupancyMaxActiveBlocksPerMultiprocessor failed");
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return kf_fail(KF_EHIP, "hipDeviceGetAttribute(MultiprocessorCount) failed");
        gr = (per_cu < 1 ? 1 : per_cu) * (cus > 0 ? cus : 1);
    }
    *grid = gr;
    *block = kBlock;
    *lds = l;
    return KF_OK;
}
}  // namespace

extern "C" int kf_count_launch_info(int k, int* grid, int* block, int* lds_bytes) {
    if (k < KF_MIN_K || k > KF_MAX_K) return kf_fail(KF_EINVAL, "k out of range [2, 12]");
    if (!grid || !block || !lds_bytes) return kf_fail(KF_EINVAL, "null output pointer");
    if (k >= 10) return bucket_launch_info(k, grid, block, lds_bytes);
    return launch_info(k, grid, block, lds_bytes);
}

extern "C" int kf_workspace_reserve(int k, int32_t max_genomes) {
    if (k < KF_MIN_K || k > KF_MAX_K) return kf_fail(KF_EINVAL, "k out of range [2, 12]");
    if (max_genomes < 0) return kf_fail(KF_EINVAL, "max_genomes < 0");
    if (k >= 10) return bucket_reserve(k, max_genomes);
    int grid = 0, block = 0, lds = 0;   // the kernel attribute and grid of k
    return launch_info(k, &grid, &block, &lds);
}

extern "C" int kf_count_batch(const uint8_t* d_bytes, const uint64_t* d_goff, int32_t n_genomes,
                              const uint64_t* d_excl, uint64_t n_excl, const uint32_t* d_code2col,
                              const uint32_t* d_col2rep, int k, uint32_t* d_counts, uint64_t* d_totals,
                              uint32_t flags, void* stream) {
    if (k < KF_MIN_K || k > KF_MAX_K) return kf_fail(KF_EINVAL, "k out of range [2, 12]");
    if (n_genomes < 0) return kf_fail(KF_EINVAL, "n_genomes < 0");
    if (n_genomes == 0) return KF_OK;
    if (!d_bytes || !d_goff || !d_counts || !d_totals || !d_code2col || !d_col2rep)
        return kf_fail(KF_EINVAL, "null device pointer");
    if (n_excl && !d_excl) return kf_fail(KF_EINVAL, "d_excl is null but n_excl > 0");
    if (((uintptr_t)d_bytes) & 15) return kf_fail(KF_EINVAL, "d_bytes must be 16-byte aligned");
    const uint64_t nb = kf_num_bins(k);
    hipStream_t s = (hipStream_t)stream;
#ifdef KF_PROFILE_BUILD
    // profiling builds: KF_K9_BUCKET=1 counts k = 9 with bucket_kernel<9> (the
    // rounds 1-5 path), for A/B against K9b
    const bool bucket = k >= 10 || (k == 9 && getenv("KF_K9_BUCKET") && atoi(getenv("KF_K9_BUCKET")));
#else
    const bool bucket = k >= 10;
#endif
    if (!(flags & KF_ACCUMULATE)) {
        // k >= 9: the bucket kernels write every row themselves
        if ((!bucket && hipMemsetAsync(d_counts, 0, (size_t)n_genomes * nb * sizeof(uint32_t), s) != hipSuccess) ||
            hipMemsetAsync(d_totals, 0, (size_t)n_genomes * sizeof(uint64_t), s) != hipSuccess)
            return kf_fail(KF_EHIP, "hipMemsetAsync failed");
    }
    CountArgs A;
    A.bytes = d_bytes;
    A.goff = d_goff;
    A.excl = d_excl;
    A.n_excl = n_excl;
    A.code2col = d_code2col;
    A.col2rep = d_col2rep;
    A.counts = d_counts;
    A.totals = (unsigned long long*)d_totals;
    A.nbins = (uint32_t)nb;
    A.n_genomes = n_genomes;
    A.flags = flags;
    if (bucket) return bucket_launch(A, k, flags, s);
    int grid = 0, block = 0, lds = 0;
    const int rc = launch_info(k, &grid, &block, &lds);
    if (rc) return rc;

    void* args[] = {&A};
    if (hipLaunchKernel(kernel_for(k), dim3(grid), dim3(block), args, (size_t)lds, s) != hipSuccess)
        return kf_fail(KF_EHIP, "count kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
    return KF_OK;
}

extern "C" int kf_stream_probe(const uint8_t* d_bytes, uint64_t n, uint32_t* d_out, void* stream) {
    if (!d_bytes || !d_out) return kf_fail(KF_EINVAL, "null device pointer");
    if (((uintptr_t)d_bytes) & 15) return kf_fail(KF_EINVAL, "d_bytes must be 16-byte aligned");
    if (n == 0) return KF_OK;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return kf_fail(KF_EHIP, "device query failed");
    hipLaunchKernelGGL(stream_probe_kernel, dim3(2 * (cus > 0 ? cus : 1)), dim3(1024), 0, (hipStream_t)stream, d_bytes,
                       n, d_out);
    if (hipGetLastError() != hipSuccess) return kf_fail(KF_EHIP, "stream probe launch failed");
    return KF_OK;
}

extern "C" int kf_synth_fasta(uint8_t* d_bytes, const uint64_t* d_goff, int32_t n_genomes, int64_t g0,
                              int64_t g_stride, uint64_t seed0, uint64_t seq_len, int width, uint64_t n_period,
                              void* stream) {
    if (n_genomes <= 0) return n_genomes == 0 ? KF_OK : kf_fail(KF_EINVAL, "n_genomes < 0");
    if (!d_bytes || !d_goff) return kf_fail(KF_EINVAL, "null device pointer");
    if (width < 1) return kf_fail(KF_EINVAL, "width < 1");
    if (n_genomes > 65535) return kf_fail(KF_EINVAL, "at most 65535 genomes per synth call");
    dim3 grid(512, (unsigned)n_genomes);
    hipLaunchKernelGGL(synth_kernel, grid, dim3(256), 0, (hipStream_t)stream, d_bytes, d_goff, g0, g_stride, seed0,
                       seq_len, width, n_period);
    if (hipGetLastError() != hipSuccess) return kf_fail(KF_EHIP, "synth kernel launch failed");
    return KF_OK;
}
