// kf_count.hip -- canonical k-mer counting kernels for MI355X (gfx950, CDNA4).
//
// Replaces the Jellyfish shell-out of kf2vec's get_frequencies
// (reference kf2vec/main.py:309-323: `jellyfish count -C` + `jellyfish dump -c`
// + the pandas read of the dump).  Semantics restated in oracle/kmer_oracle.c.
//
// Work decomposition (DESIGN.md "Kernel K1"):
//   * the batch [goff[0], goff[n)) is split into `gridDim.x` equal byte spans, one
//     per workgroup (512 threads = 8 waves); a span may cross genome boundaries;
//   * each genome piece of a span is split into 8 contiguous wave ranges; a wave
//     walks its range in 1 KiB chunks, lane L owning bytes [16L, 16L+16) of the
//     chunk (one coalesced dwordx4 per lane, 3 chunks prefetched);
//   * per lane: SWAR classification of the 16 bytes (v_perm + v_dot4, no table
//     loads), newline compaction, then the k-1 bases of context arrive from
//     lane L-1 through one DPP `wave_shr:1` (lane 0 from the previous chunk's
//     lane 63); the 16 k-mer windows are cut from a 64-bit register window by
//     v_bfe, canonicalised by min(fwd, revcomp) and counted with one LDS
//     `ds_add_u32` each into the workgroup's 4^k-entry histogram (k <= 7);
//   * at the end of a genome piece the histogram is flushed with coalesced u32
//     global atomics in column order (col2rep gather) and re-zeroed;
//   * k >= 8: the same front end, counting straight into global memory.
// Records: FASTA header / FASTQ non-sequence lines arrive as an interval list
// (kf_index_records) and are treated as invalid bytes (k-mer reset).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <cstdio>
#include <map>
#include <utility>

#include "kf_front_zoo.h"
#include "kf_internal.h"

namespace kf {

// Workgroup shapes ("variants"): one 4^k-entry LDS histogram is shared by all
// waves of a workgroup, so a bigger workgroup raises occupancy at equal LDS.
//   variant 0: 512 threads (8 waves), 2 workgroups/CU at k=7
//   variant 1: 1024 threads (16 waves), 8 waves/SIMD register budget
//   variant 2: as 1 with a 6-deep chunk prefetch ring (5 chunks in flight)
//   variants 5..7: k = 7 pair counting (pair_kernel below), one 1024-thread
//             workgroup per CU (144 KiB of LDS), 4 waves/SIMD, prefetch ring 6 / 4 / 8;
//             for every other k they run as variant 1
//   variants 8, 9: k <= 7 dynamic-chunk forward histogram (dyn_kernel below), as
//             variant 1 with chunks from an LDS counter, prefetch ring 4 / 6;
//             for k = 8 they run as variant 1
//   variants 10, 11: k = 7 pair counting on count_kernel's static wave ranges
//             (count_chunk_pair), one 1024-thread workgroup per CU, ring 6 / 8;
//             for every other k they run as variant 1
//   variants 12, 13: k = 7 pair counting with 32-byte lanes (K1w, wide_fast),
//             static wave ranges, one 1024-thread workgroup per CU, ring of
//             2 / 3 iterations of 2 KiB; for every other k they run as variant 1
//   variant 22: K1x variant 19 whose waves split only the first part of each
//             genome piece statically and claim the rest in small units from a
//             per-workgroup ticket (KF_DYN_FRAC, KF_DYN_UNIT), so they finish a
//             piece together
//   variant 23: K1x variant 19 whose waves claim their own range's 3 KiB
//             iterations one by one from the front (with the loads, two ahead)
//             while waves that are done take the back half of the range with
//             the most left (compare-and-swap on the range's word)
//   variant 24: k = 8 on the K1x front end (48-byte lanes): every window an
//             8-mer in 65,536 u16 LDS counters, one pass (instead of K2's two);
//             for every other k it runs as variant 1
constexpr int kNumVariants = 25;
constexpr int kDefaultVariant = 19;   // K1x (every add's return checked, ring 2) at k = 7; variant 1 (K1) for every other k
// (variant 20, returns checked every other iteration, is not exact on inputs built so that
// a counter only grows in unchecked iterations: test_k7_unchecked_iterations_adversarial)
constexpr int kDefaultVariantK8 = 24;   // k = 8: single pass on the K1x front end (K2, variant 1, takes two)
constexpr int kFirstPairVariant = 5;
// K1x default shares by wave age slot (KF_WAVE_WEIGHTS overrides)
constexpr uint32_t kWaveW0 = 20, kWaveW1 = 17, kWaveW2 = 11, kWaveW3 = 6;
#ifndef KF_PAIR_ABL
#define KF_PAIR_ABL 0
#endif
// pair variants: 4 waves/SIMD (one workgroup per CU); the half-table ablation runs two
constexpr int kPairWpe = KF_PAIR_ABL == 4 ? 8 : 4;
template <int V> struct Shape;
template <> struct Shape<0> { static constexpr int block = 512, wpe = 0, abl = 0, ring = 4; };
template <> struct Shape<1> { static constexpr int block = 1024, wpe = 8, abl = 0, ring = 4; };
template <> struct Shape<2> { static constexpr int block = 1024, wpe = 8, abl = 0, ring = 6; };
template <> struct Shape<5> { static constexpr int block = 1024, wpe = kPairWpe, abl = 0, ring = 6; };
template <> struct Shape<6> { static constexpr int block = 1024, wpe = kPairWpe, abl = 0, ring = 4; };
template <> struct Shape<7> { static constexpr int block = 1024, wpe = kPairWpe, abl = 0, ring = 8; };
template <> struct Shape<8> { static constexpr int block = 1024, wpe = 8, abl = 0, ring = 4; };
template <> struct Shape<9> { static constexpr int block = 1024, wpe = 8, abl = 0, ring = 6; };
template <> struct Shape<10> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 6; };
template <> struct Shape<11> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 8; };
template <> struct Shape<12> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 2; };   // ring in 2 KiB
template <> struct Shape<13> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 3; };
// K1w knobs: aux = cache policy of the byte-stream loads (2 = nt), late = returns
// checked one iteration later (two register sets by ring-slot parity)
template <> struct Shape<14> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 3, aux = 2, late = 0; };
template <> struct Shape<15> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 4, aux = 0, late = 0; };
template <> struct Shape<16> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 4, aux = 0, late = 1; };
template <> struct Shape<17> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 4, aux = 2, late = 1; };
template <int V> constexpr bool kWide = V >= 12 && V <= 17;
template <int V> struct WideKnobs { static constexpr int aux = 0, late = 0; };
template <> struct WideKnobs<14> { static constexpr int aux = Shape<14>::aux, late = Shape<14>::late; };
template <> struct WideKnobs<15> { static constexpr int aux = Shape<15>::aux, late = Shape<15>::late; };
template <> struct WideKnobs<16> { static constexpr int aux = Shape<16>::aux, late = Shape<16>::late; };
template <> struct WideKnobs<17> { static constexpr int aux = Shape<17>::aux, late = Shape<17>::late; };
// K1x: 48-byte lanes (3 KiB per wave iteration), table classification (x_fast)
template <> struct Shape<18> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 3; };
template <> struct Shape<19> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 2; };
template <> struct Shape<20> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 2; };   // + alternating checks
template <> struct Shape<21> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 2; };   // + paired iterations
template <> struct Shape<22> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 2; };   // 19 + claimed tail units
template <> struct Shape<23> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 2; };   // 19 + stealing
template <> struct Shape<24> { static constexpr int block = 1024, wpe = 4, abl = 0, ring = 2; };   // k = 8 on K1x
template <int V> constexpr bool kX = V >= 18 && V <= 24;
template <int V> constexpr bool kStaticPair = V == 10 || V == 11 || kWide<V> || kX<V>;
#ifdef KF_ABLATION
// profiling-only builds (python -m kf2vecfsw_amd.build --ablation): wrong counts by design
template <> struct Shape<3> { static constexpr int block = 1024, wpe = 8, abl = 1, ring = 4; };   // no LDS adds
template <> struct Shape<4> { static constexpr int block = 1024, wpe = 8, abl = 3, ring = 4; };   // stream only
#endif
// Counting modes by k:
//   k <= 7 : one LDS histogram of all 4^k forward codes (64 KiB at k=7)
//   k = 8  : multi-pass LDS: the forward-code space is cut into 32768-code
//            ranges (128 KiB of LDS); pass p counts codes with code >> 15 == p
//            and its flush merges into the canonical columns (2 passes)
//   k >= 9 : bucket kernels (kf_bucket.hip), see there.  The count kernels
//            below still cover k 9..12 (multi-pass at 9, global atomics at
//            code2col[min(fwd, revcomp)] above) for A/B runs via KF_BUCKET_MIN_K.
constexpr int kLdsMaxK = 7;
constexpr int kMultiMaxK = 9;
constexpr int kMultiBits = 15;
constexpr int kDefaultBucketMinK = 9;
enum { kModeLds = 0, kModeMulti = 1, kModeGlobal = 2 };
template <int K>
struct ModeOf {
    static constexpr int mode = K <= kLdsMaxK ? kModeLds : (K <= kMultiMaxK ? kModeMulti : kModeGlobal);
    static constexpr int passes = mode == kModeMulti ? (1 << (2 * K - kMultiBits)) : 1;
    static constexpr uint32_t lds_codes = mode == kModeLds ? (1u << (2 * K))
                                        : (mode == kModeMulti ? (1u << kMultiBits) : 0u);
};


// Count one chunk.  GLOBAL = count straight into d_counts (k > kLdsMaxK).
template <int K, bool MASKED, bool GLOBAL, int ABL>
__device__ __forceinline__ uint32_t count_chunk(const uint4 d, const CountArgs& A, uint64_t chunk, int lane,
                                                const ChunkMask& m, uint64_t iv0, uint32_t carry,
                                                uint32_t* __restrict__ hist, uint32_t* __restrict__ gcounts,
                                                uint32_t& lane_total, uint32_t pass) {
    constexpr uint32_t TM = (K > 1) ? ((1u << (2 * (K - 1))) - 1u) : 0u;
    constexpr int W2 = 2 * K;
    if constexpr (ModeOf<K>::mode == kModeLds && !MASKED && ABL == 0) {
        // Fast case (uniform, the common one): every lane's 16 bytes are bases
        // except at most one newline, and the carry is complete.  Then every
        // lane's 15-16 entries are valid, so is lane L-1's tail, windows
        // 0..ne-1 are valid and the context is just lane L-1's raw codes: no
        // validity masks, no tails, no run mask, no inc extraction.
        uint32_t Cf, NNL, bad;
        classify16_fast(d, Cf, NNL, bad);
        const uint32_t nef = (uint32_t)__builtin_popcount(NNL);
        const bool self_ok = bad == 0 && nef >= 15u;
        if (t_n(carry) >= (uint32_t)(K - 1) && __builtin_amdgcn_ballot_w64(!self_ok) == 0) {
            // drop the newline entry (none: r = 16, identity)
            const uint32_t r = (uint32_t)__builtin_ctz((NNL ^ 0xFFFFu) | 0x10000u);
            const uint32_t lo1 = (1u << r) - 1u, lo2 = lo1 | (lo1 << r);
            const uint32_t C = bfi(lo2, Cf, Cf >> 2);
            const uint32_t pC = wave_shr1(t_codes(carry), C);
            // X = (pC:C) << 2 over ne entries of C; ne in {15, 16} and C is zero
            // above entry ne-1, so the high word is pC << (2ne+2 mod 32) | C >> 30.
            // Byte address of window r = bits [2r, 2r+2K+2) of X, masked: 8
            // views at bit offsets 0,2,..,14 serve r = 0..7 from their low 16
            // bits and r = 8..15 from their high 16 bits (a word select).
            constexpr uint32_t M4 = ((1u << W2) - 1u) << 2;
            const uint32_t xlo = C << 2, xhi = (pC << ((2u * nef + 2u) & 31u)) | (C >> 30);
            uint32_t xv[8];
#pragma unroll
            for (int o = 0; o < 8; ++o) xv[o] = o ? __builtin_amdgcn_alignbit(xhi, xlo, 2 * o) : xlo;
            auto addr = [&](int w) -> uint32_t { return (w < 8 ? xv[w] : (xv[w - 8] >> 16)) & M4; };
            const uint32_t inc15 = nef >> 4;   // window 15 exists iff no newline
#ifdef KF_K1_NOADD   // profiling only (tools/build_abl.sh): the fast path without its LDS adds
#pragma unroll
            for (int w = 0; w < 16; ++w) lane_total += addr(w);
#else
#pragma unroll
            for (int w = 0; w < 15; ++w) lds_add(addr(w), 1u);
            lds_add(addr(15), inc15);
#endif
            lane_total += 15u + inc15;
            // lane 63's block is all valid bases: its tail is complete
            const uint32_t c63 = (uint32_t)__builtin_amdgcn_readlane((int)C, kWave - 1);
            return tail_pack(c63 & TM, 31u, 31u);
        }
    }
    uint32_t C, V, EN, ne, own;
    front_end<K, MASKED, false>(d, A, chunk, lane, m, iv0, C, V, EN, ne, own);
    const Windows win = windows<K, MASKED>(C, V, EN, ne, carry, lane);
    const uint32_t wlo = win.wlo, whi = win.whi, R = win.R;
    const uint32_t wv[4] = {wlo, __builtin_amdgcn_alignbit(whi, wlo, 8), __builtin_amdgcn_alignbit(whi, wlo, 16),
                            __builtin_amdgcn_alignbit(whi, wlo, 24)};
    // forward window ending at entry r: bits [2r, 2r+2K) of W (first base highest)
    auto fwd = [&](int r) -> uint32_t {
        const int fo = (2 * r) & ~7;
        return __builtin_amdgcn_ubfe(wv[fo >> 3], 2 * r - fo, W2);
    };
    if (ModeOf<K>::mode == kModeMulti) {
        // multi-pass LDS: this pass counts forward codes in [pass << 15, (pass+1) << 15)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t f = fwd(r);
            if (((R >> r) & 1u) && (f >> kMultiBits) == pass) lds_add((f & ((1u << kMultiBits) - 1u)) << 2, 1u);
        }
    } else if (!GLOBAL) {
        // LDS path: count FORWARD k-mers only into the 4^k histogram; a k-mer and
        // its reverse complement are merged into one canonical bin at flush time.
        // Byte address of window r = 4*fwd(r) = bits [2r, 2r+2K+2) of X = W << 2,
        // masked: 8 views at bit offsets 0,2,..,14 serve r = 0..7 from their low
        // 16 bits and r = 8..15 from their high 16 bits (a word select).
        constexpr uint32_t M4 = ((1u << W2) - 1u) << 2;
        const uint32_t xlo = wlo << 2, xhi = __builtin_amdgcn_alignbit(whi, wlo, 30);
        uint32_t xv[8];
#pragma unroll
        for (int o = 0; o < 8; ++o) xv[o] = o ? __builtin_amdgcn_alignbit(xhi, xlo, 2 * o) : xlo;
        auto addr = [&](int r) -> uint32_t { return (r < 8 ? xv[r] : (xv[r - 8] >> 16)) & M4; };
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t inc = (R >> r) & 1u;
            if (ABL == 0)
                lds_add(addr(r), inc);
            else   // profiling only (no LDS traffic)
                lane_total += addr(r) ^ inc;
        }
    } else {
        // global path: canonical = min(fwd, revcomp) in kf code, then column via code2col
        const uint32_t rhi = revpairs(wlo) ^ 0xAAAAAAAAu;   // revcomp of the 64-bit window
        const uint32_t rlo = revpairs(whi) ^ 0xAAAAAAAAu;
        constexpr int RS = 2 * (17 - K);
        const uint32_t rplo = __builtin_amdgcn_alignbit(rhi, rlo, RS);
        const uint32_t rphi = rhi >> RS;
        const uint32_t rv[4] = {rplo, __builtin_amdgcn_alignbit(rphi, rplo, 8),
                                __builtin_amdgcn_alignbit(rphi, rplo, 16), __builtin_amdgcn_alignbit(rphi, rplo, 24)};
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t f = fwd(r);
            const int rr = 2 * (15 - r), ro = rr & ~7;
            const uint32_t c = __builtin_amdgcn_ubfe(rv[ro >> 3], rr - ro, W2);
            if ((R >> r) & 1u) {
                const uint32_t col = A.code2col[min(f, c)];
                __hip_atomic_fetch_add(gcounts + col, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    lane_total += (uint32_t)__builtin_popcount(R);
    return win.next;
}

// ---------------------------------------------------------------- k = 7 pair counting
// Two consecutive 7-mer windows are one 8-mer: its first seven bases are the
// older window, its last seven the newer one.  The fast path counts the windows
// of a chunk in pairs, one LDS atomic per pair instead of one per window, into
// P = 4^8 u16 counters (128 KiB: 8-mer x in half x & 1 of word x >> 1).  Windows
// left unpaired (an odd chunk total, and every window of an irregular chunk) go
// to S, 8192 u16 counters (16 KiB) indexed by the 7-mer folded to the orientation
// whose middle base is A or C (s_fold): one slot per canonical 7-mer.  At flush a
// canonical column with forward representative y gets
//   F(y) + F(rc y) + S[fold y],  F(y) = sum_a P[4y + a] + sum_a P[a 4^7 + y]
// (y as the older window of a pair, then as the newer one).
// u16 halves: every add returns the old word; a half that has reached 0x4000 is
// moved to the genome's count row (pair_drain).  At most two chunks of adds per
// wave (16 waves x 2 x 1024) can land on a half between its crossing and the
// first drain, so it stays below 0x4000 + 0x8000: the counts are exact.
#if KF_PAIR_ABL == 4   // profiling only: P folded to 64 KiB and S to 8 KiB (wrong counts), 2 workgroups/CU
constexpr uint32_t kPairSBase = 1u << 16;
constexpr uint32_t kPairCtl = kPairSBase + (1u << 13);
#else
constexpr uint32_t kPairSBase = 1u << 17;                    // byte offset of S
constexpr uint32_t kPairCtl = kPairSBase + (1u << 14);       // two chunk counters (pair_kernel)
#endif
constexpr uint32_t kPairLdsBytes = kPairCtl + 16;
constexpr uint32_t kU16Hot = 0xC000C000u;                    // a half >= 0x4000
// (address masks: no-ops for the real layout, keep the ablation inside its LDS)
constexpr uint32_t kPairPMask = kPairSBase - 4u;
constexpr uint32_t kPairSMask = kPairCtl - kPairSBase - 4u;
// K1s (count_chunk_pair): its singles by forward 7-mer, 16384 u16 after P (32 KiB),
// so P + S fill the 160 KiB of a CU and a single costs no revcomp/fold
constexpr uint32_t kFwdSEnd = kPairSBase + (1u << 15);

__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t a, uint32_t v) {
    return __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Workgroup barrier ordering LDS only: waits for this wave's LDS operations, not
// for its vector-memory ones (__syncthreads waits for vmcnt(0) too, i.e. for the
// ring's last prefetches and the flush's row stores, a full memory latency under
// load; nothing here reads global memory another wave of the workgroup wrote).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 7-mer (kf code, A0 C1 T2 G3, complement = ^2) -> S slot: the orientation whose
// middle base (bits 6-7) has bit 7 clear, with that bit dropped.
__device__ __forceinline__ uint32_t s_fold(uint32_t y, uint32_t rc) {
    const uint32_t z = (y & 0x80u) ? rc : y;
    return ((z >> 8) << 7) | (z & 0x7Fu);
}
__device__ __forceinline__ uint32_t s_unfold(uint32_t i) { return ((i >> 7) << 8) | (i & 0x7Fu); }
__device__ __forceinline__ uint32_t s_addr(uint32_t i) { return kPairSBase + (((i >> 1) << 2) & kPairSMask); }
__device__ __forceinline__ uint32_t half_one(uint32_t i) { return 1u << ((i & 1u) << 4); }

// Rare path: move 0x4000 out of each half of the LDS word at byte address a that
// has reached it, into the count row (compare-and-swap: each move happens once).
template <bool FWD_S = false>   // S indexed by forward 7-mer (K1s) instead of s_fold
__device__ __noinline__ void pair_drain(uint32_t a, const uint32_t* __restrict__ code2col, uint32_t* gcounts) {
    lds_u32* p = (lds_u32*)(uintptr_t)a;
    uint32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (cur & kU16Hot) {
        const uint32_t sub = ((cur & 0xC0000000u) ? 0x40000000u : 0u) | ((cur & 0xC000u) ? 0x4000u : 0u);
        uint32_t seen = cur;
        if (__hip_atomic_compare_exchange_strong(p, &seen, cur - sub, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
            const bool single = a >= kPairSBase;
            const uint32_t w = (single ? a - kPairSBase : a) >> 2;
            for (uint32_t h = 0; h < 2; ++h) {
                if (!((sub >> (16 * h)) & 0x4000u)) continue;
                const uint32_t bin = 2 * w + h;   // 8-mer (P) or S slot
                if (single) {
                    atomicAdd(gcounts + code2col[FWD_S ? bin : s_unfold(bin)], 0x4000u);
                } else {
                    atomicAdd(gcounts + code2col[bin >> 2], 0x4000u);
                    atomicAdd(gcounts + code2col[bin & 0x3FFFu], 0x4000u);
                }
            }
            cur -= sub;
        } else {
            cur = seen;
        }
    }
}

// Exclusive count of set bits of m below this lane.
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// 1 << byte b of h (the byte is 0 or 16): one SDWA shift.
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

// A pair-kernel chunk is self-contained: lane 0 loads the 16 bytes before the
// chunk's own 1008 (63 lanes x 16 B), which give lane 1 its k-1 bases of context,
// and counts nothing itself.  So chunks need no carry from their predecessor and
// the waves of a workgroup can take them in any order (pair_kernel hands them out
// from an LDS counter).  Chunk c of a piece owns [c0 + 1008 c, c0 + 1008 (c+1)).
constexpr uint32_t kOwn = kChunk - 16;

// Chunk bookkeeping is 32-bit relative to c0 (a piece is far below 4 GiB) so it
// stays on the SALU: gfx9 has no 64-bit ordered scalar compare.
struct PPiece {
    uint64_t glo, plo, phi, c0;
    const uint8_t* pb16;   // bytes + c0 - 16: lane 0's block of chunk 0
    uint32_t nch;          // chunks
    uint32_t end_r;        // align16(ghi) - c0: readable bytes
    uint32_t fast_lo;      // chunks whose own bytes start at >= fast_lo ...
    uint32_t fast_hi;      // ... and end at <= fast_hi can take the fast path
    uint32_t skip0;        // chunk 0's lane-0 block would start before the genome
};
__device__ __forceinline__ PPiece make_piece(const uint8_t* bytes, uint64_t glo, uint64_t ghi, uint64_t plo,
                                             uint64_t phi) {
    PPiece P;
    P.glo = glo, P.plo = plo, P.phi = phi;
    P.c0 = plo & ~(uint64_t)15;
    P.pb16 = bytes + P.c0 - 16;
    const uint64_t gal = glo & ~(uint64_t)15;
    P.skip0 = P.c0 < gal + 16 ? 16u : 0u;
    P.end_r = (uint32_t)(((ghi + 15) & ~(uint64_t)15) - P.c0);
    P.nch = phi > plo ? (uint32_t)((phi - P.c0 + kOwn - 1) / kOwn) : 0u;
    P.fast_lo = (uint32_t)(max(glo + 16, plo) - P.c0);
    P.fast_hi = (uint32_t)(phi - P.c0);
    return P;
}
// Lane block of chunk c (zeros for c >= nch, without touching memory).  Lane 0
// of a chunk whose context would start before the genome's aligned start reads
// zeros (its offset wraps past num_records), never bytes before the buffer.
__device__ __forceinline__ uint4 pload(const PPiece& P, uint32_t c, int lane) {
    const uint32_t adj = c == 0 ? P.skip0 : 0u;
    const uint32_t b16 = kOwn * c + adj;   // descriptor base - (c0 - 16)
    const uint32_t avail = P.end_r + 16u > b16 ? P.end_r + 16u - b16 : 0u;
    // (readfirstlane: keeps the descriptor in SGPRs; the compiler turns the clamp
    // above into a VALU saturating subtract and would waterfall the load)
    const uint32_t rec = __builtin_amdgcn_readfirstlane(c < P.nch ? min(avail, (uint32_t)kChunk) : 0u);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(P.pb16 + b16), (short)0, (int)rec, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(16 * lane) - adj, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// Excluded-interval cursor of a wave (its chunks come in increasing order);
// s_r / e_r: the current interval relative to the piece's c0 - 16, clamped.
struct IvCursor {
    uint64_t iv;
    uint32_t s_r, e_r;
    __device__ __forceinline__ void init(const CountArgs& A, uint64_t pos, int lane) {
        iv = wave_upper_bound(A.n_excl, pos, lane, [&](uint64_t i) { return A.excl[2 * i + 1]; });
    }
    // (signed: c0 - 16 is negative for a piece in the buffer's first 16 bytes)
    __device__ __forceinline__ static uint32_t rel(uint64_t x, int64_t o) {
        const int64_t d = (int64_t)x - o;
        return d <= 0 ? 0u : (d >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)d);
    }
    __device__ __forceinline__ void load(const CountArgs& A, const PPiece& P) {
        s_r = e_r = 0xFFFFFFFFu;
        if (iv < A.n_excl) {
            s_r = rel(uload64(A.excl + 2 * iv), (int64_t)P.c0 - 16);
            e_r = rel(uload64(A.excl + 2 * iv + 1), (int64_t)P.c0 - 16);
        }
    }
    // true if an interval overlaps [a, b) (relative to c0 - 16); first moves past
    // intervals ending <= a
    __device__ __forceinline__ bool hits(const CountArgs& A, const PPiece& P, uint32_t a, uint32_t b) {
        if (e_r <= a) {   // rare
            const int64_t aa = (int64_t)P.c0 - 16 + (int64_t)a;
            do { ++iv; } while (iv < A.n_excl && (int64_t)uload64(A.excl + 2 * iv + 1) <= aa);
            load(A, P);
        }
        return s_r < b;
    }
};

// Rare path: drain every hot word of P and S (one wave, CAS-exact as pair_drain).
template <bool FWD_S = false>
__device__ __noinline__ void pair_scan_drain(const uint32_t* __restrict__ code2col, uint32_t* gcounts, int lane) {
    for (uint32_t w = (uint32_t)lane; w < (FWD_S ? kFwdSEnd : kPairCtl) / 4; w += kWave) {
        const uint32_t v = __hip_atomic_load((lds_u32*)(uintptr_t)(4 * w), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        if (v & kU16Hot) pair_drain<FWD_S>(4 * w, code2col, gcounts);
    }
}

__device__ __forceinline__ uint32_t u16sum2(uint32_t w) { return (w & 0xFFFFu) + (w >> 16); }

// Flush step 1 (1024 threads): per forward 7-mer y, F(y) = sum_a P[4y + a] +
// sum_a P[a 4^7 + y]; thread t owns y = 2048 i + 2t + {0, 1}, i = 0..7
// (lane-consecutive reads).
// LDS word of F(y) in the flush: bits 1-4 XOR bits 8-11.  A wave reads F at 64
// representatives y that differ in their low bases and at their reverse
// complements, which then differ only in bits 8-13: unswizzled, every rc read
// of a wave would hit one bank.  Bit 0 is kept, so F(2m), F(2m+1) stay a pair.
__device__ __forceinline__ uint32_t f_swz(uint32_t y) { return y ^ (((y >> 8) & 15u) << 1); }

__device__ __forceinline__ void pair_f_sums(const uint32_t* hist, int tid, uint32_t (&F)[16]) {
    const uint4* h4 = (const uint4*)hist;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint4 w = h4[(i * 1024 + tid) & (kPairSBase / 16 - 1)];   // words 2y .. 2y+3 of y = 2048 i + 2 tid
        F[2 * i] = u16sum2(w.x) + u16sum2(w.y);
        F[2 * i + 1] = u16sum2(w.z) + u16sum2(w.w);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const uint32_t v = hist[(a * 8192 + i * 1024 + tid) & (kPairSBase / 4 - 1)];   // halves a 4^7 + y, a 4^7 + y + 1
            F[2 * i] += v & 0xFFFFu;
            F[2 * i + 1] += v >> 16;
        }
    }
}

// Every counted window of an irregular chunk as a single 7-mer into S; with
// these returns the pending ones of the last fast chunk are checked too.
__device__ __forceinline__ void pair_singles(const Windows& win, const CountArgs& A, uint32_t* gcounts, int lane,
                                             uint32_t& lane_total, uint32_t (&pend)[9]) {
    constexpr int K = 7;
    const uint32_t wlo = win.wlo, whi = win.whi, R = win.R;
    const uint32_t wv[4] = {wlo, __builtin_amdgcn_alignbit(whi, wlo, 8), __builtin_amdgcn_alignbit(whi, wlo, 16),
                            __builtin_amdgcn_alignbit(whi, wlo, 24)};
    auto fwd = [&](int r) -> uint32_t {
        const int fo = (2 * r) & ~7;
        return __builtin_amdgcn_ubfe(wv[fo >> 3], 2 * r - fo, 2 * K);
    };
    // reverse complement of the 64-bit window: revcomp of window r = bits [2(15-r), +2K) of RP
    const uint32_t rhi = revpairs(wlo) ^ 0xAAAAAAAAu, rlo = revpairs(whi) ^ 0xAAAAAAAAu;
    constexpr int RS = 2 * (17 - K);
    const uint32_t rplo = __builtin_amdgcn_alignbit(rhi, rlo, RS), rphi = rhi >> RS;
    const uint32_t rv[4] = {rplo, __builtin_amdgcn_alignbit(rphi, rplo, 8), __builtin_amdgcn_alignbit(rphi, rplo, 16),
                            __builtin_amdgcn_alignbit(rphi, rplo, 24)};
    auto rcw = [&](int r) -> uint32_t {
        const int rr = 2 * (15 - r), ro = rr & ~7;
        return __builtin_amdgcn_ubfe(rv[ro >> 3], rr - ro, 2 * K);
    };
    uint32_t o = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t i = s_fold(fwd(r), rcw(r));
        o |= lds_add_rtn(s_addr(i), ((R >> r) & 1u) * half_one(i));
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        o |= pend[j];
        pend[j] = 0;
    }
    if (__builtin_amdgcn_ballot_w64((o & kU16Hot) != 0) != 0) pair_scan_drain(A.code2col, gcounts, lane);
    lane_total += (uint32_t)__builtin_popcount(R);
}

// The fast path checks the returned words of the PREVIOUS fast chunk (pend), after
// issuing its own adds, so a wave never waits for its own LDS returns; a hot word
// then costs one scan of P and S.  With that one chunk of delay at most three
// chunks of adds per wave (16 x 3 x 520) land on a half between its crossing of
// 0x4000 and the drain, still below 0x10000.
template <bool MASKED>
__device__ __forceinline__ void count_chunk_ind(const uint4 d, const CountArgs& A, const PPiece& P, uint32_t c,
                                                int lane, uint64_t iv0, uint32_t* gcounts, uint32_t& lane_total,
                                                uint32_t (&pend)[9]) {
    constexpr int K = 7;
    const uint64_t own = P.c0 + (uint64_t)kOwn * c;
    if constexpr (!MASKED) {
        uint32_t Cf, NNL, bad;
        classify16_fast(d, Cf, NNL, bad);
        const uint32_t nef = (uint32_t)__builtin_popcount(NNL);
        const bool self_ok = bad == 0 && nef >= 15u;
        if (__builtin_amdgcn_ballot_w64(!self_ok) == 0) {
            // every block is bases with at most one newline: lane 0's 15-16 bases are
            // lane 1's context; drop the newline entry, context from lane L-1
            const uint32_t r = (uint32_t)__builtin_ctz((NNL ^ 0xFFFFu) | 0x10000u);
            const uint32_t lo1 = (1u << r) - 1u, lo2 = lo1 | (lo1 << r);
            const uint32_t C = bfi(lo2, Cf, Cf >> 2);
            const uint32_t pC = wave_shr1(0u, C);
            // The windows of lanes 1..63 in stream order are paired (0,1), (2,3), ...;
            // a lane owns the pairs whose newer window is its own.  p = parity of the
            // windows in lanes 1..L-1 (lanes with 15 entries are the odd ones); pairs
            // then end at entries q, q+2, ... (entry 0 = newest).
            const uint32_t p = lanes_below(__builtin_amdgcn_ballot_w64(nef == 15u) & ~1ull) & 1u;
            const uint32_t q = (nef + p) & 1u;
            const uint64_t W = (((uint64_t)pC << (2u * nef)) | (uint64_t)C) >> (2u * q);
            const uint32_t lo = (uint32_t)W, hi = (uint32_t)(W >> 32);
            // pair j = 8-mer at bits [4j, 4j+16) of W: word (x >> 1) at byte address
            // bits [4j+1, 4j+16) << 2, half = bit 4j (as 16 x that bit, one per byte)
            const uint32_t H0 = (lo << 4) & 0x10101010u, H1 = lo & 0x10101010u;
            const uint32_t one = 1u;
            const bool has7 = !(nef == 15u && p == 0u);   // pair 7 would end at entry 15
            auto paddr = [&](int j) -> uint32_t {
                return (j == 0 ? (lo << 1) : __builtin_amdgcn_alignbit(hi, lo, 4 * j - 1)) & kPairPMask;
            };
            uint32_t rt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            const bool single = lane == kWave - 1 && q;   // odd total: the newest window is unpaired
            if (lane != 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    uint32_t dl;
                    switch (j) {
                    case 0: dl = shl1_byte<0>(H0, one); break;
                    case 1: dl = shl1_byte<0>(H1, one); break;
                    case 2: dl = shl1_byte<1>(H0, one); break;
                    case 3: dl = shl1_byte<1>(H1, one); break;
                    case 4: dl = shl1_byte<2>(H0, one); break;
                    case 5: dl = shl1_byte<2>(H1, one); break;
                    case 6: dl = shl1_byte<3>(H0, one); break;
                    default: dl = has7 ? shl1_byte<3>(H1, one) : 0u; break;
                    }
#if KF_PAIR_ABL == 1 || KF_PAIR_ABL == 4   // profiling only: no returns, no overflow check (wrong on low complexity)
                    lds_add(paddr(j), dl);
#elif KF_PAIR_ABL == 2   // profiling only: no pair adds at all
                    lane_total += paddr(j) ^ dl;
#else
                    rt[j] = lds_add_rtn(paddr(j), dl);
#endif
                }
                lane_total += nef;
                if (single) {
                    const uint32_t y = C & 0x3FFFu;
                    const uint32_t i = s_fold(y, kf_revcomp<K>(y));
                    rt[8] = lds_add_rtn(s_addr(i), half_one(i));
                }
            }
            uint32_t po = 0;
#pragma unroll
            for (int j = 0; j < 9; ++j) po |= pend[j];
            if (__builtin_amdgcn_ballot_w64((po & kU16Hot) != 0) != 0) pair_scan_drain(A.code2col, gcounts, lane);
#pragma unroll
            for (int j = 0; j < 9; ++j) pend[j] = rt[j];
            return;
        }
    }
    // irregular chunk: every counted window as a single 7-mer into S
    const uint64_t B = own - 16;   // lane 0's block (may lie before the genome: invalid)
    const ChunkMask m{P.glo, max(own, P.plo), min(own + kOwn, P.phi)};
    uint32_t C, V, EN, ne, own_t;
    front_end<K, true>(d, A, B, lane, m, iv0, C, V, EN, ne, own_t);
    // lane 1 needs exact context: lane 0's block if its tail is complete, else walk back
    uint32_t carry = tail_pack(0, 0, 0);
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)own_t, 0);
    if (!tail_complete<K>(t0)) {   // rare: fewer than k-1 bases and no reset in 16 bytes
        for (int64_t p = (int64_t)B; p > (int64_t)P.glo && !tail_complete<K>(carry);) {
            p -= kChunk;
            carry = tail_combine<K>(chunk_tail<K>(A.bytes, A.excl, A.n_excl, p, P.glo, lane), carry);
        }
    }
    const Windows win = windows<K, true>(C, V, EN, ne, carry, lane);
    pair_singles(win, A, gcounts, lane, lane_total, pend);
}

// Pair counting on count_kernel's static wave ranges (variants 10, 11): a chunk
// continues its wave's stream (lane 0's context is the carry), so every lane of
// the fast case holds 16 windows (8 pairs) or, with a newline in its block, 15
// (7 pairs and its oldest window as a single).  Irregular chunks go to S whole.
// Here S is indexed by the forward 7-mer (16384 u16 after P, kFwdSEnd): a single
// costs no revcomp/fold, and the flush adds S[y] into F(y).  Returns are checked one chunk late as in count_chunk_ind: this chunk's land in
// pout, the previous chunk's are checked from pin.  The caller alternates two
// register sets by ring-slot parity, so no returned word is ever copied (a copy
// would wait for the returns before this chunk's adds go out).
template <bool MASKED>
__device__ __forceinline__ uint32_t count_chunk_pair(const uint4 d, const CountArgs& A, uint64_t chunk, int lane,
                                                     const ChunkMask& m, uint64_t iv0, uint32_t carry,
                                                     uint32_t* gcounts, uint32_t& lane_total, uint32_t (&pin)[9],
                                                     uint32_t (&pout)[9]) {
    constexpr int K = 7;
    constexpr uint32_t TM = (1u << (2 * (K - 1))) - 1u;
    if constexpr (!MASKED) {
        uint32_t Cf, NNL, bad;
        classify16_fast(d, Cf, NNL, bad);
        const uint32_t nef = (uint32_t)__builtin_popcount(NNL);
        const bool self_ok = bad == 0 && nef >= 15u;
        if (t_n(carry) >= (uint32_t)(K - 1) && __builtin_amdgcn_ballot_w64(!self_ok) == 0) {
            const uint32_t r = (uint32_t)__builtin_ctz((NNL ^ 0xFFFFu) | 0x10000u);
            const uint32_t lo1 = (1u << r) - 1u, lo2 = lo1 | (lo1 << r);
            const uint32_t C = bfi(lo2, Cf, Cf >> 2);
            const uint32_t pC = wave_shr1(t_codes(carry), C);
            // X = W << 2, W = (pC : C) over nef entries (as count_chunk).  Pair j =
            // windows 2j (newer) and 2j+1 = the 8-mer at bits [4j, 4j+16) of W: LDS
            // word bits [4j+1, 4j+16) of W, i.e. bits [4j+3, 4j+18) of X, times 4;
            // half = bit 4j of W.
            const uint32_t xlo = C << 2, xhi = (pC << ((2u * nef + 2u) & 31u)) | (C >> 30);
            const uint32_t wl = __builtin_amdgcn_alignbit(xhi, xlo, 2);   // W's low word
            const uint32_t H0 = (wl << 4) & 0x10101010u, H1 = wl & 0x10101010u;
            const uint32_t one = 1u;
            const bool has7 = nef == 16u;
            uint32_t (&rt)[9] = pout;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint32_t dl;
                switch (j) {
                case 0: dl = shl1_byte<0>(H0, one); break;
                case 1: dl = shl1_byte<0>(H1, one); break;
                case 2: dl = shl1_byte<1>(H0, one); break;
                case 3: dl = shl1_byte<1>(H1, one); break;
                case 4: dl = shl1_byte<2>(H0, one); break;
                case 5: dl = shl1_byte<2>(H1, one); break;
                case 6: dl = shl1_byte<3>(H0, one); break;
                default: dl = has7 ? shl1_byte<3>(H1, one) : 0u; break;
                }
                const uint32_t a = (j == 0 ? (wl << 1) : __builtin_amdgcn_alignbit(xhi, xlo, 4 * j + 1)) & kPairPMask;
#if KF_PAIR_ABL == 1   // profiling only: no returns, no overflow check (wrong on low complexity)
                lds_add(a, dl);
                rt[j] = 0;
#elif KF_PAIR_ABL == 2   // profiling only: no pair adds at all
                lane_total += a ^ dl;
                rt[j] = 0;
#else
                rt[j] = lds_add_rtn(a, dl);
#endif
            }
            rt[8] = 0;
            if (!has7) {   // window 14 (bits [28, 42) of W) alone, by forward code
                const uint32_t y = __builtin_amdgcn_alignbit(xhi, xlo, 30) & 0x3FFFu;
                rt[8] = lds_add_rtn(kPairSBase + ((y >> 1) << 2), half_one(y));
            }
            lane_total += nef;
            uint32_t po = 0;
#pragma unroll
            for (int j = 0; j < 9; ++j) po |= pin[j];
            if (__builtin_amdgcn_ballot_w64((po & kU16Hot) != 0) != 0) pair_scan_drain<true>(A.code2col, gcounts, lane);
            const uint32_t c63 = (uint32_t)__builtin_amdgcn_readlane((int)C, kWave - 1);
            return tail_pack(c63 & TM, 31u, 31u);
        }
    }
    uint32_t C, V, EN, ne, own;
    front_end<K, MASKED, false>(d, A, chunk, lane, m, iv0, C, V, EN, ne, own);
    const Windows win = windows<K, MASKED>(C, V, EN, ne, carry, lane);
    // irregular chunk: every counted window as a single, by forward code
    const uint32_t wlo = win.wlo, whi = win.whi, R = win.R;
    const uint32_t wv[4] = {wlo, __builtin_amdgcn_alignbit(whi, wlo, 8), __builtin_amdgcn_alignbit(whi, wlo, 16),
                            __builtin_amdgcn_alignbit(whi, wlo, 24)};
    uint32_t o = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int fo = (2 * r) & ~7;
        const uint32_t y = __builtin_amdgcn_ubfe(wv[fo >> 3], 2 * r - fo, 2 * K);
        o |= lds_add_rtn(kPairSBase + ((y >> 1) << 2), ((R >> r) & 1u) * half_one(y));
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        o |= pin[j];
        pout[j] = 0;
    }
    if (__builtin_amdgcn_ballot_w64((o & kU16Hot) != 0) != 0) pair_scan_drain<true>(A.code2col, gcounts, lane);
    lane_total += (uint32_t)__builtin_popcount(R);
    return win.next;
}

// ---------------------------------------------------------------- K1w: wide-lane pairs
// K1s with 32 bytes per lane: a wave iteration covers 2 KiB, lane L owning bytes
// [32L, 32L+32) (two dwordx4 loads).  The per-lane work that does not scale with
// the bytes -- newline removal, the context from lane L-1, the carry test, the
// return check, the chunk bookkeeping -- is paid once per 32 bytes instead of once
// per 16.  With at most one newline in a lane's 32 bytes (any FASTA of >= 32
// columns) a lane holds 32 windows (16 pairs into P) or 31 (15 pairs + window 30
// as a single into S); P and S are K1s's (forward 8-mer u16 halves, forward
// 7-mer u16 singles), so is the flush.
// u16 exactness: every add returns the old word and a wave checks its returns at
// the end of the same iteration; a half seen at >= 0x4000 is drained (the whole
// table is scanned, CAS-exact).  After a half crosses 0x4000 every wave that adds
// to it adds at most one more iteration (<= 1024 adds to one half) before its own
// drain, so a half stays below 0x4000 + 16 x 1024 = 0x8000.
constexpr int kWChunk = 2 * kChunk;
#ifndef KF_K1W_ABL
// profiling-only builds (tools/build_abl.sh, wrong counts by design): 1 = no LDS
// adds, 2 = adds without returns or checks, 3 = no classification (raw bits as
// codes, every lane fast without a newline), 4 = stream only, 5 = K1x compute
// only (the loads re-read the range's first chunks, cache-resident)
#define KF_K1W_ABL 0
#endif
constexpr uint32_t kWideHot = 0xC000C000u;    // a half >= 0x4000
constexpr uint32_t kWideStep = 0x4000u;

// Move STEP out of each hot half (>= STEP, HOT = the halves' bits at or above it)
// of the LDS word at byte address a into the count row until both halves are
// below STEP (compare-and-swap: exact under concurrent adds).  P word: 8-mers 2w,
// 2w+1; S word (a >= kPairSBase): forward 7-mers 2w, 2w+1.  K1w: STEP 0x4000;
// K1x: 0x2000 (it checks returns every other iteration, see x_fast).
// K = 8 (variant 24): a P half is one 8-mer, whose column is code2col[bin].
template <uint32_t HOT = kWideHot, uint32_t STEP = kWideStep, int K = 7>
__device__ __noinline__ void wide_drain(uint32_t a, const uint32_t* __restrict__ code2col, uint32_t* gcounts) {
    lds_u32* p = (lds_u32*)(uintptr_t)a;
    uint32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (cur & HOT) {
        const uint32_t sub = ((cur & (HOT & 0xFFFF0000u)) ? (STEP << 16) : 0u) | ((cur & (HOT & 0xFFFFu)) ? STEP : 0u);
        uint32_t seen = cur;
        if (__hip_atomic_compare_exchange_strong(p, &seen, cur - sub, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
            const bool single = a >= kPairSBase;
            const uint32_t w = (single ? a - kPairSBase : a) >> 2;
            for (uint32_t h = 0; h < 2; ++h) {
                if (!((sub >> (16 * h)) & 0xFFFFu)) continue;
                const uint32_t bin = 2 * w + h;
                if (K == 8) {
                    atomicAdd(gcounts + code2col[bin], STEP);
                } else if (single) {
                    atomicAdd(gcounts + code2col[bin], STEP);
                } else {
                    atomicAdd(gcounts + code2col[bin >> 2], STEP);       // older 7-mer
                    atomicAdd(gcounts + code2col[bin & 0x3FFFu], STEP);  // newer 7-mer
                }
            }
            cur -= sub;
        } else {
            cur = seen;
        }
    }
}
template <uint32_t HOT = kWideHot, uint32_t STEP = kWideStep, int K = 7>
__device__ __noinline__ void wide_scan_drain(const uint32_t* __restrict__ code2col, uint32_t* gcounts, int lane) {
    for (uint32_t w = (uint32_t)lane; w < (K == 8 ? kPairSBase : kFwdSEnd) / 4; w += kWave) {
        const uint32_t v = __hip_atomic_load((lds_u32*)(uintptr_t)(4 * w), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        if (v & HOT) wide_drain<HOT, STEP, K>(4 * w, code2col, gcounts);
    }
}
constexpr uint32_t kXHot = 0xE000E000u;   // K1x: a half >= 0x2000
constexpr uint32_t kXStep = 0x2000u;

struct WideBlock {
    uint4 a, b;   // lane L: bytes [32L, 32L + 16) and [32L + 16, 32L + 32) of the 2 KiB chunk
};
// Lane blocks of the 2 KiB chunk at c0 + rel, clamped to align16(ghi) like load_chunk.
template <int AUX = 0>
__device__ __forceinline__ WideBlock wide_load(const uint8_t* bytes, uint64_t c0, uint32_t rel, uint32_t end_r,
                                               int lane) {
    const uint32_t rec = end_r > rel ? min(end_r - rel, (uint32_t)kWChunk) : 0u;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + c0 + rel), (short)0, (int)rec, 0x00020000);
    const auto v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 32, 0, AUX);
    const auto v1 = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 32 + 16, 0, AUX);
    WideBlock w;
    w.a = make_uint4(v0[0], v0[1], v0[2], v0[3]);
    w.b = make_uint4(v1[0], v1[1], v1[2], v1[3]);
    return w;
}

// Fast case of a 2 KiB iteration (uniform): every lane's 32 bytes are bases
// with at most one newline, and the carry is complete.  Returns false (nothing
// counted) otherwise.
// LATE: this iteration's returns go to pout and the previous fast iteration's
// (pin) are checked before this iteration's adds go out, so no wave waits for
// its own returns; a half then stays below 0x4000 + 16 x 2 x 1024 = 0xC000.
template <bool LATE = false>
__device__ __forceinline__ bool wide_fast(const WideBlock& d, const CountArgs& A, int lane, uint32_t& carry,
                                          uint32_t* gcounts, uint32_t& lane_total, const uint32_t (&pin)[16],
                                          uint32_t (&pout)[16]) {
    constexpr uint32_t TM = (1u << 12) - 1u;
    uint32_t Ca, Na, ba, Cb, Nb, bb;
#if KF_K1W_ABL == 3
    Ca = d.a.x ^ d.a.y ^ d.a.z ^ d.a.w, Cb = d.b.x ^ d.b.y ^ d.b.z ^ d.b.w;
    Na = Nb = 0xFFFFu, ba = bb = 0;
#else
    classify16_fast(d.a, Ca, Na, ba);   // bytes 0..15: entries 31..16
    classify16_fast(d.b, Cb, Nb, bb);   // bytes 16..31: entries 15..0 (entry 0 = newest)
#endif
    // not-newline mask, bit r = entry r; inv has one bit per newline
    const uint32_t inv = ~((Na << 16) | Nb);
    const uint32_t M1 = inv - 1u;       // entries below the newline (all if none)
    const bool self_ok = (ba | bb) == 0 && (inv & M1) == 0;
    carry = __builtin_amdgcn_readfirstlane(carry);   // wave-uniform: its tests run on the SALU
    if (t_n(carry) < 6u || __builtin_amdgcn_ballot_w64(!self_ok) != 0) return false;
    // 2-bit entry mask of M1 (a prefix mask per half: m | m << popcount(m))
    const uint32_t m1l = M1 & 0xFFFFu, m1h = M1 >> 16;
    const uint32_t Ml = m1l | (m1l << __builtin_popcount(m1l));
    const uint32_t Mh = m1h | (m1h << __builtin_popcount(m1h));
    // drop the newline entry: every entry above it moves down one
    const uint32_t Cl = bfi(Ml, Cb, __builtin_amdgcn_alignbit(Ca, Cb, 2));
    const uint32_t Ch = bfi(Mh, Ca, Ca >> 2);
    // context: lane L-1's newest entries (lane 0: the carry), placed above this
    // lane's nef = 31 or 32 entries: W = pC << 2 nef | (Ch : Cl)
    const uint32_t pC = wave_shr1(t_codes(carry), Cl);
    const uint32_t nl = 1u - (M1 >> 31);                 // 1 iff this lane has a newline
    const uint64_t t = (uint64_t)pC << (32u - 2u * nl);
    const uint32_t w0 = Cl, w1 = Ch | (uint32_t)t, w2 = (uint32_t)(t >> 32);
    // pair j = windows 2j (newer) and 2j+1 = the 8-mer at bits [4j, 4j+16) of W:
    // P word (8-mer >> 1) at byte address bits [4j+1, 4j+16) << 2 = (X >> 4j) &
    // 0x1FFFC with X = W << 1; half = bit 4j of W
    const uint32_t x0 = w0 << 1, x1 = __builtin_amdgcn_alignbit(w1, w0, 31), x2 = __builtin_amdgcn_alignbit(w2, w1, 31);
    // X >> 16 views: pairs 4..7 and 12..15 then need a plain shift (a 2-cycle
    // VOP2 op) instead of an alignbit each (VOP3, 4 cycles; profiles/r02/valu_rate.txt)
    const uint32_t y0 = __builtin_amdgcn_alignbit(x1, x0, 16), y1 = __builtin_amdgcn_alignbit(x2, x1, 16);
    constexpr uint32_t PM = 0x1FFFCu;
    const uint32_t H0 = (w0 << 4) & 0x10101010u, H1 = w0 & 0x10101010u;
    const uint32_t H2 = (w1 << 4) & 0x10101010u, H3 = w1 & 0x10101010u;
    const uint32_t one = 1u;
    if constexpr (LATE) {
        const uint32_t po = ((pin[0] | pin[1]) | (pin[2] | pin[3])) | ((pin[4] | pin[5]) | (pin[6] | pin[7])) |
                            ((pin[8] | pin[9]) | (pin[10] | pin[11])) | ((pin[12] | pin[13]) | (pin[14] | pin[15]));
        if (__builtin_amdgcn_ballot_w64((po & kWideHot) != 0) != 0) wide_scan_drain(A.code2col, gcounts, lane);
    }
    uint32_t rtl[16];
    uint32_t (&rt)[16] = LATE ? pout : rtl;   // returned words
#pragma unroll
    for (int j = 0; j < 15; ++j) {
        uint32_t a;
        if (j < 4) a = (x0 >> (4 * j)) & PM;
        else if (j < 8) a = (y0 >> (4 * (j - 4))) & PM;
        else if (j < 12) a = (x1 >> (4 * (j - 8))) & PM;
        else a = (y1 >> (4 * (j - 12))) & PM;
        uint32_t dl;
        const int jj = j & 7;
        const uint32_t He = j < 8 ? H0 : H2, Ho = j < 8 ? H1 : H3;
        switch (jj) {
        case 0: dl = shl1_byte<0>(He, one); break;
        case 1: dl = shl1_byte<0>(Ho, one); break;
        case 2: dl = shl1_byte<1>(He, one); break;
        case 3: dl = shl1_byte<1>(Ho, one); break;
        case 4: dl = shl1_byte<2>(He, one); break;
        case 5: dl = shl1_byte<2>(Ho, one); break;
        case 6: dl = shl1_byte<3>(He, one); break;
        default: dl = shl1_byte<3>(Ho, one); break;
        }
#if KF_PAIR_ABL == 1 || KF_K1W_ABL == 2   // profiling only: no returns (wrong on low complexity)
        lds_add(a, dl);
        rt[j] = 0;
#elif KF_K1W_ABL == 1
        lane_total += a ^ dl;
        rt[j] = 0;
#else
        rt[j] = lds_add_rtn(a, dl);
#endif
    }
    {
        // pair 15 (windows 30, 31) without a newline; with one, window 30 alone
        // (bits [60, 74) of W) into S by its forward code
        const uint32_t ap = (y1 >> 12) & PM;
        const uint32_t dp = shl1_byte<3>(H3, one);
        const uint32_t y = __builtin_amdgcn_alignbit(w2, w1, 28) & 0x3FFFu;
        const uint32_t as = kPairSBase + ((y >> 1) << 2), ds = half_one(y);
        const uint32_t sel = 0u - nl;
#if KF_K1W_ABL == 1
        lane_total += bfi(sel, as, ap) ^ bfi(sel, ds, dp);
        rt[15] = 0;
#elif KF_K1W_ABL == 2
        lds_add(bfi(sel, as, ap), bfi(sel, ds, dp));
        rt[15] = 0;
#else
        rt[15] = lds_add_rtn(bfi(sel, as, ap), bfi(sel, ds, dp));
#endif
    }
    lane_total += 32u - nl;
    if constexpr (!LATE) {
        const uint32_t o = ((rt[0] | rt[1]) | (rt[2] | rt[3])) | ((rt[4] | rt[5]) | (rt[6] | rt[7])) |
                           ((rt[8] | rt[9]) | (rt[10] | rt[11])) | ((rt[12] | rt[13]) | (rt[14] | rt[15]));
        if (__builtin_amdgcn_ballot_w64((o & kWideHot) != 0) != 0) wide_scan_drain(A.code2col, gcounts, lane);
    }
    carry = tail_pack((uint32_t)__builtin_amdgcn_readlane((int)Cl, kWave - 1) & TM, 31u, 31u);
    return true;
}

// Irregular 1 KiB chunk (16-byte lane layout, count_chunk's general path): every
// counted window as a single into S by its forward code; returns checked at once.
// K = 8 (variant 24): every window is an 8-mer counted in P (u16 half of word y >> 1).
template <bool MASKED, uint32_t HOT = kWideHot, uint32_t STEP = kWideStep, int K = 7>
__device__ __forceinline__ uint32_t wide_singles(const uint4 d, const CountArgs& A, uint64_t chunk, int lane,
                                                 const ChunkMask& m, uint64_t iv0, uint32_t carry, uint32_t* gcounts,
                                                 uint32_t& lane_total, uint32_t& drained) {
    uint32_t C, V, EN, ne, own;
    front_end<K, MASKED, false>(d, A, chunk, lane, m, iv0, C, V, EN, ne, own);
    const Windows win = windows<K, MASKED>(C, V, EN, ne, carry, lane);
    const uint32_t wlo = win.wlo, whi = win.whi, R = win.R;
    const uint32_t wv[4] = {wlo, __builtin_amdgcn_alignbit(whi, wlo, 8), __builtin_amdgcn_alignbit(whi, wlo, 16),
                            __builtin_amdgcn_alignbit(whi, wlo, 24)};
    uint32_t o = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int fo = (2 * r) & ~7;
        const uint32_t y = __builtin_amdgcn_ubfe(wv[fo >> 3], 2 * r - fo, 2 * K);
        o |= lds_add_rtn((K == 8 ? 0u : kPairSBase) + ((y >> 1) << 2), ((R >> r) & 1u) * half_one(y));
    }
    if (__builtin_amdgcn_ballot_w64((o & HOT) != 0) != 0) {
        wide_scan_drain<HOT, STEP, K>(A.code2col, gcounts, lane);
        drained = 1;
    }
    lane_total += (uint32_t)__builtin_popcount(R);
    return win.next;
}

// The wave range [lo, hi) of genome [glo, ghi) in 2 KiB iterations (K1w).
template <int RING, int AUX = 0, bool LATE = false>
__device__ __forceinline__ uint64_t process_range_wide(const CountArgs& A, int32_t g, uint64_t glo, uint64_t ghi,
                                                       uint64_t lo, uint64_t hi, int lane) {
    static_assert(!LATE || RING % 2 == 0, "late return sets alternate by ring slot");
    if (lo >= hi) return 0;
    uint32_t* gcounts = A.counts + (uint64_t)g * A.nbins;
    Range rg;
    rg.init(glo, ghi, lo, hi);
    WideBlock buf[RING];
#pragma unroll
    for (int j = 0; j < RING; ++j) buf[j] = wide_load<AUX>(A.bytes, rg.c0, j * kWChunk, rg.end_r, lane);
    rg.warm<7>(A, lane);
    uint32_t carry = rg.carry;
    uint32_t rel = 0;
    const ChunkMask m = rg.mask();
    uint32_t lane_total = 0;
    uint32_t drained = 0;   // (K1w flushes with atomics whatever its drains)
    uint32_t pend0[16], pend1[16];   // LATE: returns of the last fast iteration, by slot parity
#pragma unroll
    for (int j = 0; j < 16; ++j) pend0[j] = pend1[j] = 0;
    auto step = [&](const WideBlock& bf, int slot) {
#if KF_K1W_ABL == 4
        lane_total += bf.a.x ^ bf.a.y ^ bf.a.z ^ bf.a.w ^ bf.b.x ^ bf.b.y ^ bf.b.z ^ bf.b.w;
        rel += kWChunk;
        return;
#endif
        uint32_t(&pin)[16] = (slot & 1) ? pend0 : pend1;
        uint32_t(&pout)[16] = (slot & 1) ? pend1 : pend0;
        const bool m0 = rg.masked(A, rel);
        const uint64_t iv0 = rg.iv;   // first half's interval cursor (m1's test may advance it)
        const bool m1 = rg.masked(A, rel + kChunk);
        if (m0 || m1 || !wide_fast<LATE>(bf, A, lane, carry, gcounts, lane_total, pin, pout)) {
            if constexpr (LATE) {   // the previous iteration's returns, then nothing pending
                uint32_t po = 0;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    po |= pin[j];
                    pout[j] = 0;
                }
                if (__builtin_amdgcn_ballot_w64((po & kWideHot) != 0) != 0) wide_scan_drain(A.code2col, gcounts, lane);
            }
            // irregular: the two 1 KiB halves in 16-byte lane layout, singles into S
            const uint4 h0 = rg.load(A.bytes, rel, lane);
            if (m0)
                carry = wide_singles<true>(h0, A, rg.c0 + rel, lane, m, iv0, carry, gcounts, lane_total, drained);
            else
                carry = wide_singles<false>(h0, A, rg.c0 + rel, lane, m, iv0, carry, gcounts, lane_total, drained);
            if (rel + kChunk < rg.nch * kChunk) {
                const uint4 h1 = rg.load(A.bytes, rel + kChunk, lane);
                if (m1)
                    carry = wide_singles<true>(h1, A, rg.c0 + rel + kChunk, lane, m, rg.iv, carry, gcounts,
                                               lane_total, drained);
                else
                    carry = wide_singles<false>(h1, A, rg.c0 + rel + kChunk, lane, m, rg.iv, carry, gcounts,
                                                lane_total, drained);
            }
        }
        rel += kWChunk;
    };
    const uint32_t nw = (rg.nch + 1) / 2;   // 2 KiB iterations
    for (uint32_t i = 0; i + RING <= nw; i += RING) {
#pragma unroll
        for (int j = 0; j < RING; ++j) {
            step(buf[j], j);
            buf[j] = wide_load<AUX>(A.bytes, rg.c0, rel + (RING - 1) * kWChunk, rg.end_r, lane);
        }
    }
    const uint32_t rem = nw % RING;
#pragma unroll
    for (int j = 0; j < RING - 1; ++j)
        if (rem > (uint32_t)j) step(buf[j], j);
    return lane_total;
}

// ---------------------------------------------------------------- K1x: 48-byte lanes
// K1w with 48 bytes per lane: a wave iteration covers 3 KiB, lane L owning bytes
// [48L, 48L+48) (three dwordx4 loads), so the per-lane work that does not scale
// with the bytes (newline removal, context, carry, return check, bookkeeping) is
// paid once per 48 bytes; FASTA of >= 48 columns still has at most one newline
// per lane.  A lane holds 48 windows (24 pairs into P) or 47 (23 pairs + window
// 46 as a single into S); P, S, the drains and the flush are K1w's.
// Classification per dword x (4 bytes), no per-byte newline compare:
//   s  = x & 7 per byte: A/a 1, C/c 3, T/t 4, G/g 7, '\n' 2 (distinct)
//   e  = kXTab[s] (one v_perm): the lowercase base, 0x0B for '\n', and values
//        whose low three bits differ from s elsewhere
//   z  = bitop3(x, e, 0xDF..): bits other than 5 as x ^ e, bit 5 as x & ~e, so a
//        base of either case gives 0 (e has bit 5 set: case ignored), '\n' gives
//        exactly 1 ('*', which folds onto '\n', gives 0x21), and every other
//        byte gives a value outside {0, 1}
//   so z | ... & 0xFE.. != 0 flags a bad byte and the low bit of z is the
//   newline flag, packed 8 bytes at a time by two chained v_dot4
//   codes: (x & 6) = 2 x code (A0 C1 T2 G3), packed by v_dot4 with the weights
//   of the 16-byte path (2x the packed byte; the shifts that merge four of them
//   drop the factor).
constexpr int kXChunk = 3 * kChunk;
constexpr uint32_t kXTabLo = 0x630B6102u;   // e0..e3 = 0x02, 'a', 0x0B, 'c'
constexpr uint32_t kXTabHi = 0x67000074u;   // e4..e7 = 't', 0x00, 0x00, 'g'

struct XBlock {
    uint4 q[3];   // lane L: bytes [48L + 16 i, 48L + 16 i + 16) of the 3 KiB chunk
};
template <int AUX = 0>
__device__ __forceinline__ XBlock x_load(const uint8_t* bytes, uint64_t c0, uint32_t rel, uint32_t end_r, int lane) {
    const uint32_t rec = end_r > rel ? min(end_r - rel, (uint32_t)kXChunk) : 0u;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(bytes + c0 + rel), (short)0, (int)rec, 0x00020000);
    XBlock b;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 48 + 16 * i, 0, AUX);
        b.q[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    return b;
}

// dot4 weights of word i's bytes t = 0..3 in the newline test: 2 (96 - (4i + t))
__device__ __forceinline__ constexpr uint32_t x_nl_weights(int i) {
    return (uint32_t)(192 - 8 * i) | (uint32_t)(190 - 8 * i) << 8 | (uint32_t)(188 - 8 * i) << 16 |
           (uint32_t)(186 - 8 * i) << 24;
}

// z = bits other than 5 (c = 1): x ^ e; bit 5 (c = 0): x & ~e  (one v_bitop3)
__device__ __forceinline__ uint32_t x_zmap(uint32_t x, uint32_t e, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x38" : "=v"(r) : "v"(x), "v"(e), "v"(c));
    return r;
}

// Fast case of a 3 KiB iteration (uniform): every lane's 48 bytes are bases with
// at most one newline, and the carry is complete.  Returns false (nothing
// counted) otherwise.  Returns are checked at the end of the iteration: after a
// half crosses 0x4000 every wave adds at most one more iteration to it (<= 24 x 64
// adds) before its own drain, so a half stays below 0x4000 + 16 x 1536 = 0xA000.
// CHECK = false (K1x with alternating checks, variant 20): adds without returns;
// the caller checks every other iteration with the 0x2000 threshold, so a half
// stays below 0x2000 + 16 x 2 x 1536 = 0xE000.
// Classification of a 3 KiB block: the packed codes of each lane's 48 bytes
// (newline entry not yet removed) and the newline / bad-byte sum V.
struct XCls {
    uint32_t C[3], V;
};
__device__ __forceinline__ XCls x_cls(const XBlock& d) {
    const uint32_t w[12] = {d.q[0].x, d.q[0].y, d.q[0].z, d.q[0].w, d.q[1].x, d.q[1].y,
                            d.q[1].z, d.q[1].w, d.q[2].x, d.q[2].y, d.q[2].z, d.q[2].w};
    const uint32_t cdf = 0xDFDFDFDFu;
    uint32_t pc[12], z[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const uint32_t x = w[i];
        const uint32_t e = __builtin_amdgcn_perm(kXTabHi, kXTabLo, x & 0x07070707u);
        z[i] = x_zmap(x, e, cdf);
        // 2 x packed codes; odd words accumulate onto the even word's, shifted up one byte
        pc[i] = __builtin_amdgcn_udot4(x & 0x06060606u, 0x01041040u, (i & 1) ? pc[i - 1] << 8 : 0u, false);
    }
    // codes: C2 = entries 32..47 (bytes 0..15), C1 = 16..31, C0 = 0..15 (entry 0 = byte 47)
    // (pc[b + 1] = pc[b] << 8 + dot4 of word b + 1 is twice the 16-bit code of 8 bases)
    uint32_t C[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int b = 4 * (2 - i);
        C[i] = (pc[b + 1] << 15) | (pc[b + 3] >> 1);
    }
    // Newline and bad-byte test in one dot4 chain: byte b (entry 47 - b) weighs
    // 2 (96 - b), so V = sum z_b 2 (96 - b) is 0 without a newline, 98 + 2e for
    // one newline at entry e, and >= 196 otherwise (every nonzero z adds >= 98:
    // two newlines, or one bad byte's z >= 2).
    uint32_t va[4] = {0u, 0u, 0u, 0u};   // four chains of three: a short dependent path
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) va[c] = __builtin_amdgcn_udot4(z[3 * c + i], x_nl_weights(3 * c + i), va[c], false);
    const uint32_t V = (va[0] + va[1]) + (va[2] + va[3]);
    XCls r;
    r.C[0] = C[0], r.C[1] = C[1], r.C[2] = C[2], r.V = V;
    return r;
}

// Counting half of a fast iteration (the caller has tested V < 196 in every lane
// and a complete carry): newline removal, context, the 24 pair adds.  Returns the
// OR of the adds' returns (CHECK) for the caller's u16 test; updates the carry.
template <bool CHECK>
__device__ __forceinline__ uint32_t x_body(const XCls& k, uint32_t& carry, uint32_t& lane_total) {
    constexpr uint32_t TM = (1u << 12) - 1u;
    const uint32_t V = k.V;
    const uint32_t C[3] = {k.C[0], k.C[1], k.C[2]};
    uint32_t nl;   // min(V, 1), opaque: the compiler would turn its uses into selects (v_cndmask)
    asm("v_min_u32_e32 %0, 1, %1" : "=v"(nl) : "v"(V));
    // drop the newline entry: entries below it stay, every entry above moves down
    // one.  Region r (entries 16r..16r+15) keeps its low q_r = clamp(2e - 32r, 0, 32)
    // bits; without a newline V - 98 wraps high and every region keeps all.
    const uint32_t e2 = V - 98u;
    const uint32_t q0 = min(e2, 32u), q1 = min(max(e2, 32u), 64u) - 32u, q2 = min(max(e2, 64u) - 64u, 32u);
    const uint32_t L0 = (uint32_t)(~0ull << q0), L1 = (uint32_t)(~0ull << q1), L2 = (uint32_t)(~0ull << q2);
    const uint32_t c0 = bfi(L0, __builtin_amdgcn_alignbit(C[1], C[0], 2), C[0]);
    const uint32_t c1 = bfi(L1, __builtin_amdgcn_alignbit(C[2], C[1], 2), C[1]);
    const uint32_t c2 = bfi(L2, C[2] >> 2, C[2]);
    // context: lane L-1's newest entries (lane 0: the carry) above this lane's
    // n = 48 - nl entries: W = pC << 2n | (c2 : c1 : c0)
    const uint32_t pC = wave_shr1(t_codes(carry), c0);
    const uint64_t t = (uint64_t)pC << (32u - 2u * nl);
    const uint32_t w0 = c0, w1 = c1, w2 = c2 | (uint32_t)t, w3 = (uint32_t)(t >> 32);
    // pair j = windows 2j (newer) and 2j+1 = the 8-mer at bits [4j, 4j+16) of W:
    // P word address = (X >> 4j) & 0x1FFFC with X = W << 1; half = bit 4j of W.
    // Views: X dwords and X >> 16 (Y), so every pair is a plain shift and an and.
    const uint32_t x0 = w0 << 1, x1 = __builtin_amdgcn_alignbit(w1, w0, 31), x2 = __builtin_amdgcn_alignbit(w2, w1, 31),
                   x3 = __builtin_amdgcn_alignbit(w3, w2, 31);
    const uint32_t X[3] = {x0, x1, x2};
    const uint32_t Y[3] = {__builtin_amdgcn_alignbit(x1, x0, 16), __builtin_amdgcn_alignbit(x2, x1, 16),
                           __builtin_amdgcn_alignbit(x3, x2, 16)};
    const uint32_t Wd[3] = {w0, w1, w2};
    constexpr uint32_t PM = 0x1FFFCu;
    const uint32_t one = 1u;
    uint32_t rt[24];
#pragma unroll
    for (int j = 0; j < 23; ++j) {
        const int i = j >> 3, tt = j & 7;
        const uint32_t a = ((tt < 4 ? X[i] : Y[i]) >> (4 * (tt & 3))) & PM;
        const uint32_t H = (tt & 1) ? (Wd[i] & 0x10101010u) : ((Wd[i] << 4) & 0x10101010u);
        uint32_t dl;
        switch (tt >> 1) {
        case 0: dl = shl1_byte<0>(H, one); break;
        case 1: dl = shl1_byte<1>(H, one); break;
        case 2: dl = shl1_byte<2>(H, one); break;
        default: dl = shl1_byte<3>(H, one); break;
        }
#if KF_K1W_ABL == 2
        lds_add(a, dl);
        rt[j] = 0;
#elif KF_K1W_ABL == 1
        lane_total += a ^ dl;
        rt[j] = 0;
#else
        if constexpr (CHECK) {
            rt[j] = lds_add_rtn(a, dl);
        } else {
            lds_add(a, dl);
            rt[j] = 0;
        }
#endif
    }
    {
        // pair 23 (windows 46, 47) without a newline; with one, window 46 alone
        // into S by its forward code y = bits [92, 106) of W.  Both addresses come
        // from one view: v = X >> 92, P address v & 0x1FFFC, S address
        // kPairSBase | (v & 0x7FFC) (= (y >> 1) << 2); both halves are bit 92 of W.
        const uint32_t v = Y[2] >> 12;
        const uint32_t sel = 0u - nl;
        const uint32_t a23 = bfi(sel, kPairSBase | (v & 0x7FFCu), v & PM);
        const uint32_t d23 = shl1_byte<3>(w2 & 0x10101010u, one);
#if KF_K1W_ABL == 1
        lane_total += a23 ^ d23;
        rt[23] = 0;
#elif KF_K1W_ABL == 2
        lds_add(a23, d23);
        rt[23] = 0;
#else
        if constexpr (CHECK) {
            rt[23] = lds_add_rtn(a23, d23);
        } else {
            lds_add(a23, d23);
            rt[23] = 0;
        }
#endif
    }
    lane_total -= nl;   // + 48 per fast iteration, added by the caller
    uint32_t o = 0;
    if constexpr (CHECK) {
#pragma unroll
        for (int j = 0; j < 24; j += 3) o |= rt[j] | rt[j + 1] | rt[j + 2];
    }
    carry = tail_pack((uint32_t)__builtin_amdgcn_readlane((int)c0, kWave - 1) & TM, 31u, 31u);
    return o;
}

// k = 8 (variant 24): the counting half of a fast iteration with every window
// an 8-mer in P (65,536 u16 counters, half y & 1 of word y >> 1): window r =
// bits [2r, 2r + 16) of W, address (X >> 2r) & 0x1FFFC with X = W << 1, half =
// W bit 2r.  48 adds per lane (47 with a newline: window 47 then adds 0).
// Every return is checked (HOT = 0x2000 per half: a half stays below 0x2000 +
// 16 x 48 x 64 = 0xE000).
template <bool CHECK>
__device__ __forceinline__ uint32_t x_body8(const XCls& k, uint32_t& carry, uint32_t& lane_total) {
    constexpr uint32_t TM = (1u << 14) - 1u;   // 7 context entries
    const uint32_t V = k.V;
    const uint32_t C[3] = {k.C[0], k.C[1], k.C[2]};
    uint32_t nl;
    asm("v_min_u32_e32 %0, 1, %1" : "=v"(nl) : "v"(V));
    const uint32_t e2 = V - 98u;
    const uint32_t q0 = min(e2, 32u), q1 = min(max(e2, 32u), 64u) - 32u, q2 = min(max(e2, 64u) - 64u, 32u);
    const uint32_t L0 = (uint32_t)(~0ull << q0), L1 = (uint32_t)(~0ull << q1), L2 = (uint32_t)(~0ull << q2);
    const uint32_t c0 = bfi(L0, __builtin_amdgcn_alignbit(C[1], C[0], 2), C[0]);
    const uint32_t c1 = bfi(L1, __builtin_amdgcn_alignbit(C[2], C[1], 2), C[1]);
    const uint32_t c2 = bfi(L2, C[2] >> 2, C[2]);
    const uint32_t pC = wave_shr1(t_codes(carry), c0);
    const uint64_t t = (uint64_t)pC << (32u - 2u * nl);
    const uint32_t w0 = c0, w1 = c1, w2 = c2 | (uint32_t)t, w3 = (uint32_t)(t >> 32);
    const uint32_t x0 = w0 << 1, x1 = __builtin_amdgcn_alignbit(w1, w0, 31), x2 = __builtin_amdgcn_alignbit(w2, w1, 31),
                   x3 = __builtin_amdgcn_alignbit(w3, w2, 31);
    const uint32_t X[3] = {x0, x1, x2};
    const uint32_t Y[3] = {__builtin_amdgcn_alignbit(x1, x0, 16), __builtin_amdgcn_alignbit(x2, x1, 16),
                           __builtin_amdgcn_alignbit(x3, x2, 16)};
    const uint32_t Wd[3] = {w0, w1, w2};
    constexpr uint32_t PM = 0x1FFFCu;
    const uint32_t one = 1u;
    const uint32_t keep47 = nl - 1u;   // 0 with a newline: window 47 is lane L-1's window 0
    uint32_t o = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t rt[24];
#pragma unroll
        for (int q = 0; q < 24; ++q) {
            const int r = 24 * h + q, i = r >> 4, tt = r & 15;
            const uint32_t a = ((tt < 8 ? X[i] : Y[i]) >> (2 * (tt & 7))) & PM;
            const int tb = tt & 3;   // W bit 2r sits at bit 8m + 2tb of Wd[i] (m = tt >> 2): move it to 8m + 4
            const uint32_t H = (tb == 0 ? Wd[i] << 4 : (tb == 1 ? Wd[i] << 2 : (tb == 2 ? Wd[i] : Wd[i] >> 2))) & 0x10101010u;
            uint32_t dl;
            switch (tt >> 2) {
            case 0: dl = shl1_byte<0>(H, one); break;
            case 1: dl = shl1_byte<1>(H, one); break;
            case 2: dl = shl1_byte<2>(H, one); break;
            default: dl = shl1_byte<3>(H, one); break;
            }
            if (r == 47) dl &= keep47;
            if constexpr (CHECK) {
                rt[q] = lds_add_rtn(a, dl);
            } else {
                lds_add(a, dl);
                rt[q] = 0;
            }
        }
        if constexpr (CHECK) {
#pragma unroll
            for (int q = 0; q < 24; q += 3) o |= rt[q] | rt[q + 1] | rt[q + 2];
        }
    }
    lane_total -= nl;
    carry = tail_pack((uint32_t)__builtin_amdgcn_readlane((int)c0, kWave - 1) & TM, 31u, 31u);
    return o;
}

template <bool CHECK = true, uint32_t HOT = kWideHot, uint32_t STEP = kWideStep, int K = 7>
__device__ __forceinline__ bool x_fast(const XBlock& d, const CountArgs& A, int lane, uint32_t& carry,
                                       uint32_t* gcounts, uint32_t& lane_total, uint32_t& drained) {
    const XCls k = x_cls(d);
    carry = __builtin_amdgcn_readfirstlane(carry);   // wave-uniform: its tests run on the SALU
    if (t_n(carry) < (uint32_t)(K - 1) || __builtin_amdgcn_ballot_w64(k.V >= 196u) != 0) return false;
    uint32_t o;
    if constexpr (K == 8)
        o = x_body8<CHECK>(k, carry, lane_total);
    else
        o = x_body<CHECK>(k, carry, lane_total);
#ifdef KF_K1X_PAD   // profiling only: N extra VALU ops of one kind (1 = v_xor VOP2, 2 = v_perm VOP3)
    {
        const uint32_t w[12] = {d.q[0].x, d.q[0].y, d.q[0].z, d.q[0].w, d.q[1].x, d.q[1].y,
                                d.q[1].z, d.q[1].w, d.q[2].x, d.q[2].y, d.q[2].z, d.q[2].w};
        uint32_t pad[4] = {w[0], w[1], w[2], w[3]};   // four independent chains
#pragma unroll
        for (int i = 0; i < KF_K1X_PAD_N; ++i) {
#if KF_K1X_PAD == 1
            asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(pad[i & 3]) : "v"(w[i % 12]));
#else
            asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(pad[i & 3]) : "v"(w[i % 12]), "v"(w[(i + 5) % 12]));
#endif
        }
        lane_total += (pad[0] ^ pad[1] ^ pad[2] ^ pad[3]) & 1u;
    }
#endif
    if (CHECK && __builtin_amdgcn_ballot_w64((o & HOT) != 0) != 0) {
        wide_scan_drain<HOT, STEP, K>(A.code2col, gcounts, lane);
        drained = 1;
    }
    return true;
}

// The wave range [lo, hi) of genome [glo, ghi) in 3 KiB iterations (K1x).
// `drained` is set if a u16 half of this range was moved to the count row (the
// flush then adds with atomics).
// ALT (variant 20, RING = 2): returns checked in ring slot 0 only, with the
// 0x2000 threshold (every irregular iteration checks too).
// PAIRED (variant 21, RING = 2): two fast iterations at a time when both pass
// (classification of both first, then both refills, then both bodies, with one
// u16 test of all 48 returns, threshold 0x2000), else one at a time.  Every add's
// return is tested, at most two iterations after the add, so a half stays below
// 0x2000 + 16 x 2 x 1536 = 0xE000.
template <int RING, bool ALT = false, bool PAIRED = false, int K = 7>
__device__ __forceinline__ uint64_t process_range_x(const CountArgs& A, int32_t g, uint64_t glo, uint64_t ghi,
                                                    uint64_t lo, uint64_t hi, int lane, uint32_t& drained,
                                                    uint32_t piece = 0, IvHint* hint = nullptr,
                                                    unsigned long long* own = nullptr, uint32_t tag = 0) {
    static_assert(!ALT || RING == 2, "alternating checks need a 2-slot ring");
    static_assert(!PAIRED || (RING == 2 && !ALT), "paired iterations need a 2-slot ring");
    static_assert(K == 7 || (K == 8 && !ALT && !PAIRED), "k = 8 checks every return");
    constexpr uint32_t HOT = (ALT || PAIRED || K == 8) ? kXHot : kWideHot;
    constexpr uint32_t STEP = (ALT || PAIRED || K == 8) ? kXStep : kWideStep;
    if (lo >= hi) return 0;
    uint32_t* gcounts = A.counts + (uint64_t)g * A.nbins;
    const uint64_t t_begin = A.prof ? __builtin_amdgcn_s_memtime() : 0;
    Range rg;
    rg.init(glo, ghi, lo, hi);
    XBlock buf[RING];
#pragma unroll
    for (int j = 0; j < RING; ++j) buf[j] = x_load(A.bytes, rg.c0, j * kXChunk, rg.end_r, lane);
    const uint32_t nx = (rg.nch + 2) / 3;   // 3 KiB iterations
    // variant 23: the range's iterations are claimed one by one from its word
    // (tag << 48 | back << 24 | front), RING iterations ahead with the loads, so
    // other waves can take iterations from the back (claim_steal)
    unsigned long long cl[RING];
    if (own) {
        if (lane == 0) {
            __hip_atomic_store(own, ((unsigned long long)tag << 48) | ((unsigned long long)nx << 24), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int j = 0; j < RING; ++j)
                cl[j] = __hip_atomic_fetch_add(own, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // iteration `it` is this wave's if the claim made for it saw back > it
    auto owned = [&](int j, uint32_t it) -> bool {
        const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(cl[j] >> 32));
        const uint32_t l = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)cl[j]);
        return it < (((h & 0xFFFFu) << 8) | (l >> 24));
    };
    rg.warm16<K>(A, lane, hint);
    // the cursor as it stands at the range start (the loop's tests of a last
    // iteration's thirds may advance it past intervals beyond the range end)
    if (hint) *hint = rg.hint();
    __builtin_amdgcn_s_setprio(0);   // (the setup ran at top priority, see count_kernel)
    uint64_t t_loop = 0;
    if (A.prof) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        t_loop = __builtin_amdgcn_s_memtime();
    }
    uint32_t carry = rg.carry;
    uint32_t rel = 0;
    const ChunkMask m = rg.mask();
    uint32_t lane_total = 0;
    uint32_t nfast = 0;   // fast iterations (wave-uniform): 48 windows per lane each, less its newlines
#ifdef KF_K1X_PRIO   // experiment: rotate the wave priority every iteration (equal issue share by age slot)
    uint32_t prio = (uint32_t)(threadIdx.x >> 8);
#endif
    auto step = [&](const XBlock& bf, int slot) {
#ifdef KF_K1X_PRIO
        prio = (prio + 1) & 3u;
        switch (prio) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
        }
#endif
#if KF_K1W_ABL == 4
        lane_total += bf.q[0].x ^ bf.q[0].w ^ bf.q[1].y ^ bf.q[1].z ^ bf.q[2].x ^ bf.q[2].w;
        rel += kXChunk;
        return;
#endif
        // one test for the whole 3 KiB (range edges, excluded intervals)
        bool fast = !rg.masked_span(A, rel, kXChunk);
        if (fast) {
#ifdef KF_K1X_NOCHECK   // profiling only (unsafe on low-complexity input): no u16 return checks
            if (false)
#else
            if (!ALT || slot == 0)
#endif
                fast = x_fast<true, HOT, STEP, K>(bf, A, lane, carry, gcounts, lane_total, drained);
            else
                fast = x_fast<false, HOT, STEP, K>(bf, A, lane, carry, gcounts, lane_total, drained);
        }
        nfast += fast ? 1u : 0u;
        if (!fast) {
            // interval cursor before each 1 KiB third (a later test may advance it)
            const bool m0 = rg.masked(A, rel);
            const uint64_t iv0 = rg.iv;
            const bool m1 = rg.masked(A, rel + kChunk);
            const uint64_t iv1 = rg.iv;
            const bool m2 = rg.masked(A, rel + 2 * kChunk);
            // irregular: the three 1 KiB thirds in 16-byte lane layout, singles into S
#pragma unroll
            for (int h = 0; h < 3; ++h) {
                const uint32_t r = rel + h * kChunk;
                if (h > 0 && r >= rg.nch * kChunk) break;
                const bool mh = h == 0 ? m0 : (h == 1 ? m1 : m2);
                const uint64_t ivh = h == 0 ? iv0 : (h == 1 ? iv1 : rg.iv);
                const uint4 hb = rg.load(A.bytes, r, lane);
                if (mh)
                    carry = wide_singles<true, HOT, STEP, K>(hb, A, rg.c0 + r, lane, m, ivh, carry, gcounts, lane_total,
                                                             drained);
                else
                    carry = wide_singles<false, HOT, STEP, K>(hb, A, rg.c0 + r, lane, m, ivh, carry, gcounts, lane_total,
                                                              drained);
            }
        }
        rel += kXChunk;
    };
    bool stop = false;
    for (uint32_t i = 0; i + RING <= nx; i += RING) {
        if constexpr (PAIRED) {
            if (!rg.masked_span(A, rel, 2 * kXChunk)) {
                const XCls k0 = x_cls(buf[0]), k1 = x_cls(buf[1]);
                carry = __builtin_amdgcn_readfirstlane(carry);
                if (t_n(carry) >= 6u && __builtin_amdgcn_ballot_w64(max(k0.V, k1.V) >= 196u) == 0) {
                    // both raw blocks are consumed: refill the ring before the bodies
                    buf[0] = x_load(A.bytes, rg.c0, rel + 2 * kXChunk, rg.end_r, lane);
                    buf[1] = x_load(A.bytes, rg.c0, rel + 3 * kXChunk, rg.end_r, lane);
                    const uint32_t o = x_body<true>(k0, carry, lane_total) | x_body<true>(k1, carry, lane_total);
                    if (__builtin_amdgcn_ballot_w64((o & HOT) != 0) != 0) {
                        wide_scan_drain<HOT, STEP>(A.code2col, gcounts, lane);
                        drained = 1;
                    }
                    nfast += 2;
                    rel += 2 * kXChunk;
                    continue;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < RING; ++j) {
            if (own && !owned(j, i + j)) {
                stop = true;
                break;
            }
            step(buf[j], j);
#if KF_K1W_ABL == 5   // profiling only: every iteration re-reads the range's first chunks (cache hits)
            buf[j] = x_load(A.bytes, rg.c0, (uint32_t)j * kXChunk, rg.end_r, lane);
#else
            buf[j] = x_load(A.bytes, rg.c0, rel + (RING - 1) * kXChunk, rg.end_r, lane);
#endif
            if (own && lane == 0) cl[j] = __hip_atomic_fetch_add(own, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (stop) break;
    }
    const uint32_t rem = nx % RING;
#pragma unroll
    for (int j = 0; j < RING - 1; ++j)
        if (!stop && rem > (uint32_t)j) {
            if (own && !owned(j, nx - rem + j)) break;
            step(buf[j], j);
        }
    if (A.prof && lane == 0) {   // KF_COUNT_PROFILE=1: per-wave-slot loop cycles per 1 KiB chunk
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const uint64_t t_end = __builtin_amdgcn_s_memtime();
        const int w = (int)(threadIdx.x >> 6);
        atomicAdd(A.prof + 0, (unsigned long long)(t_loop - t_begin));
        atomicAdd(A.prof + 96 + w, (unsigned long long)(t_loop - t_begin));
        atomicAdd(A.prof + 1, (unsigned long long)(t_end - t_loop));
        atomicAdd(A.prof + 2, 1ull);
        atomicAdd(A.prof + 8 + w, (unsigned long long)(t_end - t_loop));
        atomicAdd(A.prof + 24 + w, (unsigned long long)rg.nch);
        if (blockIdx.x == 0 && piece < 8) {   // timeline of workgroup 0: setup start, loop start, loop end
            unsigned long long* tr = A.prof + 112 + (piece * 16 + w) * 16;
            tr[1] = t_begin;
            tr[2] = t_loop;
            tr[3] = t_end;
        }
    }
    return lane_total + 48u * nfast;
}

// Process the wave range [lo, hi) of genome [glo, ghi).
template <int K, bool GLOBAL, int ABL, int RING, bool PAIR = false>
__device__ __forceinline__ uint64_t process_range(const CountArgs& A, int32_t g, uint64_t glo, uint64_t ghi,
                                                  uint64_t lo, uint64_t hi, int lane,
                                                  uint32_t* __restrict__ hist, uint32_t pass) {
    if (lo >= hi) return 0;
    uint32_t* gcounts = (GLOBAL || PAIR) ? A.counts + (uint64_t)g * A.nbins : nullptr;
    // PAIR: returns of the last fast chunk, in set (ring slot parity)
    uint32_t pend0[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, pend1[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t t_begin = A.prof ? __builtin_amdgcn_s_memtime() : 0;
    Range rg;
    rg.init(glo, ghi, lo, hi);
    // RING-deep register ring, RING-1 chunks in flight while one is counted; a
    // buffer is refilled only after it has been consumed, so no register
    // rotation waits on a load.  The first loads go out before the warm-up.
    uint4 buf[RING];
#pragma unroll
    for (int j = 0; j < RING; ++j) buf[j] = rg.load(A.bytes, j * kChunk, lane);
    rg.warm<K>(A, lane);
    uint64_t t_loop = 0;
    if (A.prof) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        t_loop = __builtin_amdgcn_s_memtime();
    }
    uint32_t carry = rg.carry;
    uint32_t rel = 0;
    const ChunkMask m = rg.mask();
    uint32_t lane_total = 0;
    auto count = [&](const uint4 bf, int slot) {
        const uint64_t cc = rg.c0 + rel;
        const bool msk = rg.masked(A, rel);
        if constexpr (PAIR) {
            static_assert(RING % 2 == 0, "pair sets alternate by ring slot");
            uint32_t(&pin)[9] = (slot & 1) ? pend0 : pend1;
            uint32_t(&pout)[9] = (slot & 1) ? pend1 : pend0;
            if (msk)
                carry = count_chunk_pair<true>(bf, A, cc, lane, m, rg.iv, carry, gcounts, lane_total, pin, pout);
            else
                carry = count_chunk_pair<false>(bf, A, cc, lane, m, rg.iv, carry, gcounts, lane_total, pin, pout);
        } else if (ABL == 3) {   // profiling only: stream the bytes, no counting
            lane_total += bf.x ^ bf.y ^ bf.z ^ bf.w;
        } else if (msk)
            carry = count_chunk<K, true, GLOBAL, ABL>(bf, A, cc, lane, m, rg.iv, carry, hist, gcounts, lane_total, pass);
        else
            carry = count_chunk<K, false, GLOBAL, ABL>(bf, A, cc, lane, m, rg.iv, carry, hist, gcounts, lane_total, pass);
        rel += kChunk;
    };
    // steady state: groups of RING chunks with no exit in between (keeps the
    // compiler's vmcnt bookkeeping exact: wait for the oldest load only)
    const uint32_t nch = rg.nch;
    for (uint32_t i = 0; i + RING <= nch; i += RING) {
#pragma unroll
        for (int j = 0; j < RING; ++j) {
            count(buf[j], j);
            buf[j] = rg.load(A.bytes, rel + (RING - 1) * kChunk, lane);
        }
    }
    const uint32_t rem = nch % RING;
#pragma unroll
    for (int j = 0; j < RING - 1; ++j)
        if (rem > (uint32_t)j) count(buf[j], j);
    if (A.prof && lane == 0) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const uint64_t t_end = __builtin_amdgcn_s_memtime();
        const int w = (int)(threadIdx.x >> 6);
        atomicAdd(A.prof + 0, (unsigned long long)(t_loop - t_begin));
        atomicAdd(A.prof + 1, (unsigned long long)(t_end - t_loop));
        atomicAdd(A.prof + 2, 1ull);
        atomicAdd(A.prof + 8 + w, (unsigned long long)(t_end - t_loop));
        atomicAdd(A.prof + 24 + w, (unsigned long long)nch);
    }
    return lane_total;
}


template <int K, int V>
__global__ void __launch_bounds__(Shape<V>::block)
    __attribute__((amdgpu_waves_per_eu(Shape<V>::wpe ? Shape<V>::wpe : 1, Shape<V>::wpe ? Shape<V>::wpe : 8)))
    count_kernel(CountArgs A) {
    constexpr int kBlock = Shape<V>::block;
    constexpr int kWaves = kBlock / kWave;
    constexpr bool GLOBAL = ModeOf<K>::mode == kModeGlobal;
    constexpr bool MULTI = ModeOf<K>::mode == kModeMulti;
    constexpr bool PAIR = kStaticPair<V>;
    static_assert(!PAIR || ((K == 7 || (K == 8 && V == 24)) && kBlock == 1024),
                  "static pair counting is k = 7 (k = 8: variant 24), 1024 threads");
    // dynamic LDS: the histogram (PAIR: P and S) at offset 0 (so bin addresses need
    // no base add), then kWaves u64 reduction slots; no static __shared__ (it would
    // precede it)
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr uint32_t NCODES = PAIR ? kFwdSEnd / 4 : (GLOBAL ? 4u : ModeOf<K>::lds_codes);
    // variant 22: this workgroup's claim ticket as the previous launch left it
    // (read by every wave before the barrier below, which precedes every claim)
    uint32_t claim_base = 0;
    if constexpr (V == 22)
        claim_base = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(A.claim + blockIdx.x * kClaimStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (!GLOBAL) {
        for (uint32_t i = tid; i < NCODES; i += kBlock) hist[i] = 0;
        __syncthreads();
    }
    unsigned long long* red = (unsigned long long*)(hist + NCODES);
    if (!GLOBAL && (uint32_t)(uintptr_t)(lds_u32*)hist != 0u) __builtin_trap();   // lds_add assumes base 0

    const uint64_t base = A.goff[0];
    const uint64_t total = A.goff[A.n_genomes] - base;
    const uint64_t G = gridDim.x, b = blockIdx.x;
    const uint64_t span_lo = base + ((total / G * b + (total % G) * b / G) & ~(uint64_t)15);
    const uint64_t span_hi = (b + 1 == G) ? base + total
                                          : base + ((total / G * (b + 1) + (total % G) * (b + 1) / G) & ~(uint64_t)15);
    if (span_lo >= span_hi) return;
    const uint64_t tk0 = A.prof ? __builtin_amdgcn_s_memtime() : 0;        // shader clock
    const uint64_t rt0 = A.prof ? __builtin_amdgcn_s_memrealtime() : 0;    // 100 MHz
    // first genome whose end is beyond span_lo
    int32_t g = (int32_t)wave_upper_bound((uint64_t)A.n_genomes, span_lo, lane,
                                          [&](uint64_t i) { return A.goff[i + 1]; });
    uint32_t npiece = 0;   // (KF_COUNT_PROFILE timeline)
    const uint32_t fr_lo = kX<V> ? wave_frac((uint32_t)wave, A.wave_w) : 0u;
    const uint32_t fr_hi = kX<V> ? wave_frac((uint32_t)wave + 1, A.wave_w) : 0u;
    for (; g < A.n_genomes; ++g) {
        const uint64_t t_top = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        // K1x: a piece's setup (bounds, interval search, warm-up: dependent loads)
        // at top priority, so the youngest wave slots do not start late
        if constexpr (kX<V>) __builtin_amdgcn_s_setprio(3);
        const uint64_t glo = A.goff[g], ghi = A.goff[g + 1];
        if (glo >= span_hi) break;
        const uint64_t plo = max(glo, span_lo), phi = min(ghi, span_hi);
        if (phi <= plo) continue;
        // wave w owns [split(w), split(w+1)): 16-byte aligned, monotone, covering [plo, phi)
        uint64_t lo_c, hi_c;
        // variant 22: [plo, dlo) is split by wave slot, [dlo, phi) claimed in units
        const uint64_t dlo = V == 22 ? split_at_frac(plo, phi, A.dyn_frac) : phi;
        if constexpr (kX<V>) {   // K1x: parts weighted by wave slot (KF_WAVE_WEIGHTS)
            lo_c = split_at_frac(plo, dlo, fr_lo);
            hi_c = split_at_frac(plo, dlo, fr_hi);
        } else {
            lo_c = split_at(plo, phi, wave, kWaves);
            hi_c = split_at(plo, phi, wave + 1, kWaves);
        }
        if (GLOBAL) {
            const uint64_t lt = process_range<K, GLOBAL, Shape<V>::abl, Shape<V>::ring>(A, g, glo, ghi, lo_c, hi_c, lane, hist, 0);
            const unsigned long long s = wave_sum(lt);
            if (lane == 0 && s) atomicAdd(A.totals + g, s);
            continue;
        }
        unsigned long long s = 0;
        uint32_t* gc = A.counts + (uint64_t)g * A.nbins;
        if constexpr (PAIR) {
            uint32_t drained = kX<V> ? 0u : 1u;   // K1x: plain row stores unless a half was drained
            if constexpr (kX<V>) {
                // variant 22: after its static part each wave claims units of
                // [dlo, phi) by ticket until it draws one past the last unit, so
                // every piece takes exactly nunits + kWaves tickets and the next
                // piece's base is known to all waves (one call site of the loop)
                const uint32_t U = A.dyn_unit;
                const uint32_t nunits = V == 22 ? (uint32_t)((phi - dlo + U - 1) / U) : 0u;
                // In the claimed phase the next ticket is drawn before the current
                // unit is counted (its return latency hides under the unit), and
                // the interval cursor passes from range to range (no search).
                uint64_t rlo = lo_c, rhi = hi_c;
                uint32_t* const tk = A.claim + blockIdx.x * kClaimStride;
                IvHint hint{0, 0, 0, false};
                bool claimed = false;
                uint32_t t_next = 0;
                s = 0;
                for (;;) {
                    if (V == 22 && claimed && lane == 0)
                        t_next = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s += process_range_x<Shape<V>::ring, V == 20, V == 21, (V == 24 ? 8 : 7)>(
                        A, g, glo, ghi, rlo, rhi, lane, drained, npiece, V == 22 ? &hint : nullptr,
                        V == 23 && !claimed ? (unsigned long long*)tk + wave : nullptr, (npiece + 1u) & 0xFFFFu);
                    if constexpr (V != 22 && V != 23) break;
                    if constexpr (V == 23) {
                        // variant 23: take the back half of the range with the most
                        // iterations left (its owner claims from the front)
                        claimed = true;
                        const uint32_t tag = (npiece + 1u) & 0xFFFFu;
                        unsigned long long* const words = (unsigned long long*)tk;
                        unsigned long long w = 0;
                        if (lane < kWaves) w = __hip_atomic_load(words + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t f = (uint32_t)w & 0xFFFFFFu, bk = (uint32_t)(w >> 24) & 0xFFFFFFu;
                        const uint32_t left = ((uint32_t)(w >> 48) == tag && bk > f) ? bk - f : 0u;
                        uint32_t key = lane < kWaves ? (min(left, 0x3FFFFFu) << 5) | (uint32_t)lane : 0u;
#pragma unroll
                        for (int d = 1; d < kWaves; d <<= 1) key = max(key, (uint32_t)__shfl_xor((int)key, d, kWave));
                        key = (uint32_t)__builtin_amdgcn_readfirstlane((int)key);
                        if ((key >> 5) < 2u) break;
                        const uint32_t v = key & 31u;
                        uint32_t a = 0, b = 0;
                        if (lane == 0) {
                            unsigned long long cur = __hip_atomic_load(words + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            for (;;) {
                                const uint32_t cf = (uint32_t)cur & 0xFFFFFFu, cb = (uint32_t)(cur >> 24) & 0xFFFFFFu;
                                if ((uint32_t)(cur >> 48) != tag || cb < cf + 2u) break;
                                const uint32_t kk = (cb - cf) / 2u;
                                if (__hip_atomic_compare_exchange_strong(words + v, &cur, cur - ((unsigned long long)kk << 24),
                                                                         __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT)) {
                                    a = cb - kk, b = cb;
                                    break;
                                }
                            }
                        }
                        a = (uint32_t)__builtin_amdgcn_readfirstlane((int)a);
                        b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
                        if (a < b) {   // the victim's range, iterations [a, b)
                            const uint64_t vlo = split_at_frac(plo, dlo, wave_frac(v, A.wave_w));
                            const uint64_t vhi = split_at_frac(plo, dlo, wave_frac(v + 1, A.wave_w));
                            const uint64_t vc0 = vlo & ~(uint64_t)15;
                            rlo = max(vlo, vc0 + (uint64_t)a * kXChunk);
                            rhi = min(vhi, vc0 + (uint64_t)b * kXChunk);
                        } else {
                            rlo = rhi = 0;   // lost the race: look again
                        }
                        __builtin_amdgcn_s_setprio(3);
                        continue;
                    }
                    if (!claimed && lane == 0)
                        t_next = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    claimed = true;
                    const uint32_t u = (uint32_t)__builtin_amdgcn_readfirstlane((int)t_next) - claim_base;
                    if (u >= nunits) break;
                    rlo = dlo + (uint64_t)u * U;
                    rhi = min(rlo + U, phi);
                    __builtin_amdgcn_s_setprio(3);
                }
                if constexpr (V == 22) claim_base += nunits + (uint32_t)kWaves;
            }
            if constexpr (kWide<V>)
                s = process_range_wide<Shape<V>::ring, WideKnobs<V>::aux, WideKnobs<V>::late != 0>(
                    A, g, glo, ghi, lo_c, hi_c, lane);
            if constexpr (!kX<V> && !kWide<V>)
                s = process_range<K, false, 0, Shape<V>::ring, true>(A, g, glo, ghi, lo_c, hi_c, lane, hist, 0);
            const uint64_t t_p0 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            if constexpr (K == 8) {
                // variant 24 flush: canonical 8-mer column = P[rep] + P[rc rep]
                // (a palindrome once); drain flags in the unused S area
                (void)t_p0;
                lds_barrier();   // every add of this piece is done
                if (lane == 0) hist[kPairSBase / 4 + wave] = drained;
                lds_barrier();
                const uint4* fl = (const uint4*)(hist + kPairSBase / 4);
                const uint4 f0 = fl[0], f1 = fl[1], f2 = fl[2], f3 = fl[3];
                const bool any_drain = (f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w | f2.x | f2.y | f2.z |
                                        f2.w | f3.x | f3.y | f3.z | f3.w) != 0;
                const bool whole = plo == glo && phi == ghi && !(A.flags & KF_ACCUMULATE);
                for (uint32_t col = tid; col < A.nbins; col += kBlock) {
                    const uint32_t y = A.col2rep[col], rc = kf_revcomp<8>(y);
                    uint32_t v = (hist[y >> 1] >> ((y & 1u) << 4)) & 0xFFFFu;
                    if (rc != y) v += (hist[rc >> 1] >> ((rc & 1u) << 4)) & 0xFFFFu;
                    if (whole && !any_drain)
                        gc[col] = v;   // this workgroup owns row g (zeroed by the caller)
                    else if (v)
                        __hip_atomic_fetch_add(gc + col, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                lds_barrier();   // columns read
                uint4* h4 = (uint4*)hist;
                for (uint32_t i = tid; i < kFwdSEnd / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
                ++npiece;
            } else {
            // the columns' forward representatives, loaded before the barrier so
            // their latency overlaps it.  A whole genome (the common case) takes
            // four consecutive columns per lane and 16-byte row stores (the flush
            // is bound by the CU's store issue); other pieces one column per lane
            // and coalesced atomics.
            const bool whole = plo == glo && phi == ghi && !(A.flags & KF_ACCUMULATE);
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
            const uint64_t t_p1 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            uint32_t F[16];
            pair_f_sums(hist, tid, F);
#pragma unroll
            for (int i = 0; i < 8; ++i) {   // singles of y = 2048 i + 2 tid + {0, 1}
                const uint32_t v = hist[kPairSBase / 4 + i * 1024 + tid];
                F[2 * i] += v & 0xFFFFu;
                F[2 * i + 1] += v >> 16;
            }
            const uint64_t t_q0 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            lds_barrier();   // P and S read
            const uint64_t t_q1 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) *(uint2*)(hist + f_swz(i * 2048 + 2 * tid)) = make_uint2(F[2 * i], F[2 * i + 1]);
            if (lane == 0) hist[16384 + wave] = drained;   // (words past F are free now)
            lds_barrier();   // F in LDS words [0, 16384), drain flags after it
            const uint64_t t_q2 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            // A whole genome in this span with no drained half: no other workgroup
            // and nothing else touches row g, which the caller zeroed, so it is
            // written with plain stores; otherwise coalesced atomics.
            const uint4* fl = (const uint4*)(hist + 16384);
            const uint4 f0 = fl[0], f1 = fl[1], f2 = fl[2], f3 = fl[3];
            const bool any_drain = (f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w | f2.x | f2.y | f2.z | f2.w |
                                    f3.x | f3.y | f3.z | f3.w) != 0;
            uint32_t cv[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t y = rep[c], rc = kf_revcomp<K>(y);
                cv[c] = hist[f_swz(y)] + hist[f_swz(rc)];
            }
            const uint64_t t_q3 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            lds_barrier();   // columns read
            const uint64_t t_q4 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            uint4* h4 = (uint4*)hist;
            for (uint32_t i = tid; i < kFwdSEnd / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
            // the row writes last: their issue overlaps the zeroing, the barrier
            // and the next piece's setup
            if (whole && !any_drain) {
                *(uint4*)(gc + 4 * tid) = make_uint4(cv[0], cv[1], cv[2], cv[3]);
                *(uint4*)(gc + 4096 + 4 * tid) = make_uint4(cv[4], cv[5], cv[6], cv[7]);
            } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const uint32_t col = whole ? (c >> 2) * 4096 + 4 * tid + (c & 3) : tid + c * kBlock;
                    if (cv[c]) __hip_atomic_fetch_add(gc + col, cv[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (A.prof && lane == 0) atomicAdd(A.prof + 80 + wave, (unsigned long long)(t_p1 - t_p0));   // per wave
            if (A.prof && lane == 0 && blockIdx.x == 0 && npiece < 8) {
                unsigned long long* tr = A.prof + 112 + (npiece * 16 + wave) * 16;
                tr[0] = t_top;
                tr[4] = t_p0;
                tr[5] = t_p1;
                tr[6] = t_q0;
                tr[7] = t_q1;
                tr[8] = t_q2;
                tr[9] = t_q3;
                tr[10] = t_q4;
                tr[11] = __builtin_amdgcn_s_memtime();
            }
            ++npiece;
            if (A.prof && tid == 0) {   // barrier wait of wave 0 and the flush, per piece
                atomicAdd(A.prof + 3, (unsigned long long)(t_p1 - t_p0));
                atomicAdd(A.prof + 4, 1ull);
                atomicAdd(A.prof + 5, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_p1));
            }
            }   // (K == 7)
        }
        for (uint32_t pass = 0; pass < (PAIR ? 0u : (uint32_t)ModeOf<K>::passes); ++pass) {
            const uint64_t lt = process_range<K, GLOBAL, Shape<V>::abl, Shape<V>::ring>(A, g, glo, ghi, lo_c, hi_c, lane, hist, pass);
            if (Shape<V>::abl) asm volatile("" ::"v"((uint32_t)lt));   // keep ablated work alive
            const uint64_t t_f0 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            __syncthreads();
            const uint64_t t_f1 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            // canonical bin = forward count of the k-mer + forward count of its
            // revcomp; coalesced u32 atomics in column order
            for (uint32_t col = tid; col < A.nbins; col += kBlock) {
                const uint32_t rep = A.col2rep[col];
                const uint32_t rc = kf_revcomp<K>(rep);
                uint32_t v;
                if (!MULTI) {
                    v = hist[rep] + (rc != rep ? hist[rc] : 0u);
                    if (v) {
                        hist[rep] = 0;
                        hist[rc] = 0;
                    }
                } else {
                    constexpr uint32_t M = (1u << kMultiBits) - 1u;
                    v = 0;
                    if ((rep >> kMultiBits) == pass) {
                        v += hist[rep & M];
                        hist[rep & M] = 0;
                    }
                    if (rc != rep && (rc >> kMultiBits) == pass) {
                        v += hist[rc & M];
                        hist[rc & M] = 0;
                    }
                }
                if (v) {
                    __hip_atomic_fetch_add(gc + col, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s += v;
                }
            }
            const uint64_t t_f2 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
            __syncthreads();
            if (A.prof && tid == 0) {
                const uint64_t t_f3 = __builtin_amdgcn_s_memtime();
                atomicAdd(A.prof + 3, (unsigned long long)(t_f1 - t_f0));
                atomicAdd(A.prof + 4, 1ull);
                atomicAdd(A.prof + 5, (unsigned long long)(t_f2 - t_f1));
                atomicAdd(A.prof + 6, (unsigned long long)(t_f3 - t_f2));
            }
        }
        s = wave_sum(s);
        if constexpr (PAIR) {   // (no LDS left for reduction slots)
            if (lane == 0 && s) atomicAdd(A.totals + g, s);
            lds_barrier();    // P and S zero before the next piece's adds
        } else {
            if (lane == 0) red[wave] = s;
            __syncthreads();
            if (tid == 0) {
                unsigned long long t = 0;
                for (int w = 0; w < kWaves; ++w) t += red[w];
                if (t) atomicAdd(A.totals + g, t);
            }
        }
    }
    if (A.prof && tid == 0) {
        const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
        atomicAdd(A.prof + 40, (unsigned long long)(__builtin_amdgcn_s_memtime() - tk0));
        atomicAdd(A.prof + 41, (unsigned long long)(rt1 - rt0));
        atomicMin(A.prof + 42, (unsigned long long)rt0);
        atomicMax(A.prof + 43, (unsigned long long)rt1);
        atomicMax(A.prof + 44, (unsigned long long)(rt1 - rt0));
        atomicMax(A.prof + 45, (unsigned long long)rt0);
        const int hb = blockIdx.x * 2 >= gridDim.x;
        atomicAdd(A.prof + 46 + hb, (unsigned long long)(rt1 - rt0));
        atomicMax(A.prof + 48 + hb, (unsigned long long)(rt1 - rt0));
        const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7u;   // HW_REG_XCC_ID[2:0]
        atomicAdd(A.prof + 56 + xcc, (unsigned long long)(rt1 - rt0));
        atomicMax(A.prof + 64 + xcc, (unsigned long long)(rt1 - rt0));
        atomicAdd(A.prof + 72 + xcc, 1ull);
    }
}

// k = 7 pair counting kernel: same spans as count_kernel, one workgroup per CU
// holding P and S (144 KiB), so nothing else on the CU hides a stall; the kernel
// keeps the byte stream busy instead:
// * the 16 waves take self-contained chunks (count_chunk_ind) of the current
//   genome piece from an LDS counter, RING chunks ahead, so they finish a piece
//   together although a SIMD issues oldest-first (its 4th wave gets about half
//   the issue slots of its 1st);
// * at the end of a piece each wave takes and loads the next piece's first RING
//   chunks before the flush, so the flush runs under those loads;
// * flush: every 8-mer counter is read once, with lane-consecutive addresses,
//   into per-7-mer sums F (y as the older window + y as the newer window), which
//   go back to LDS; a column then needs F[rep] + F[rc rep] + S.

// Next genome piece of this workgroup at or after genome g (g = n: none).
__device__ __forceinline__ int32_t pair_next_piece(const CountArgs& A, int32_t g, uint64_t span_lo, uint64_t span_hi,
                                                   PPiece& P) {
    for (; g < A.n_genomes; ++g) {
        const uint64_t glo = A.goff[g], ghi = A.goff[g + 1];
        if (glo >= span_hi) break;
        const uint64_t plo = max(glo, span_lo), phi = min(ghi, span_hi);
        if (phi > plo) {
            P = make_piece(A.bytes, glo, ghi, plo, phi);
            return g;
        }
    }
    P = make_piece(A.bytes, 0, 0, 0, 0);
    return A.n_genomes;
}

__device__ __forceinline__ uint32_t pair_grab(uint32_t ctr, int lane) {
    uint32_t t = 0;
    if (lane == 0) t = lds_add_rtn(ctr, 1u);
    return t;
}

template <int V>
__global__ void __launch_bounds__(Shape<V>::block) __attribute__((amdgpu_waves_per_eu(Shape<V>::wpe, Shape<V>::wpe)))
    pair_kernel(CountArgs A) {
    constexpr int K = 7;
    constexpr int kBlock = Shape<V>::block;
    constexpr int RING = Shape<V>::ring;
    static_assert(kBlock == 1024, "pair_kernel flush assumes 1024 threads");
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint4* h4 = (uint4*)hist;
    for (uint32_t i = tid; i < kPairLdsBytes / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    if ((uint32_t)(uintptr_t)(lds_u32*)hist != 0u) __builtin_trap();   // addresses assume LDS base 0

    const uint64_t base = A.goff[0];
    const uint64_t total = A.goff[A.n_genomes] - base;
    const uint64_t G = gridDim.x, b = blockIdx.x;
    const uint64_t span_lo = base + ((total / G * b + (total % G) * b / G) & ~(uint64_t)15);
    const uint64_t span_hi = (b + 1 == G) ? base + total
                                          : base + ((total / G * (b + 1) + (total % G) * (b + 1) / G) & ~(uint64_t)15);
    if (span_lo >= span_hi) return;
    const uint64_t tk0 = A.prof ? __builtin_amdgcn_s_memtime() : 0;        // shader clock
    const uint64_t rt0 = A.prof ? __builtin_amdgcn_s_memrealtime() : 0;    // 100 MHz
    int32_t g = (int32_t)wave_upper_bound((uint64_t)A.n_genomes, span_lo, lane,
                                          [&](uint64_t i) { return A.goff[i + 1]; });
    PPiece P;
    g = pair_next_piece(A, g, span_lo, span_hi, P);
    if (g >= A.n_genomes) return;
    IvCursor cur;
    cur.init(A, P.c0 >= 16 ? P.c0 - 16 : 0, lane);
    cur.load(A, P);
    uint32_t par = 0;   // counter of the current piece: kPairCtl + 4 par
    uint32_t idx[RING];
    uint4 buf[RING];
#pragma unroll
    for (int j = 0; j < RING; ++j) {
        idx[j] = __builtin_amdgcn_readfirstlane(pair_grab(kPairCtl, lane));
        buf[j] = pload(P, idx[j], lane);
    }
    for (;;) {
        const uint64_t t0 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        const uint32_t ctr = kPairCtl + 4 * par;
        uint32_t* gc = A.counts + (uint64_t)g * A.nbins;
        uint32_t lt = 0, nproc = 0;
        uint32_t pend[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // returns of the last fast chunk
        for (;;) {
#pragma unroll
            for (int j = 0; j < RING; ++j) {
                const uint32_t tok = pair_grab(ctr, lane);   // refill of this slot, used below
                const uint32_t c = idx[j];
                if (c < P.nch) {
                    const uint32_t own_r = kOwn * c;   // own bytes start at c0 + own_r
                    const bool msk = own_r < P.fast_lo || own_r + kOwn > P.fast_hi ||
                                     cur.hits(A, P, own_r, own_r + kChunk);
#if KF_PAIR_ABL == 3   // profiling only: stream the bytes, no counting
                    lt += buf[j].x ^ buf[j].y ^ buf[j].z ^ buf[j].w;
                    (void)msk;
#else
                    if (msk)
                        count_chunk_ind<true>(buf[j], A, P, c, lane, cur.iv, gc, lt, pend);
                    else
                        count_chunk_ind<false>(buf[j], A, P, c, lane, cur.iv, gc, lt, pend);
#endif
                    ++nproc;
                }
                idx[j] = __builtin_amdgcn_readfirstlane(tok);
                buf[j] = pload(P, idx[j], lane);
            }
            uint32_t mn = idx[0];
#pragma unroll
            for (int j = 1; j < RING; ++j) mn = min(mn, idx[j]);
            if (mn >= P.nch) break;
        }
        const unsigned long long s = wave_sum(lt);
        if (lane == 0 && s) atomicAdd(A.totals + g, s);
        const uint64_t t1 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        if (A.prof && lane == 0) {
            atomicAdd(A.prof + 1, (unsigned long long)(t1 - t0));
            atomicAdd(A.prof + 2, 1ull);
            atomicAdd(A.prof + 8 + wave, (unsigned long long)(t1 - t0));
            atomicAdd(A.prof + 24 + wave, (unsigned long long)nproc);
        }
        __syncthreads();   // (A) every add of this piece is done
        const uint64_t t_f1 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        const int32_t gcur = g;
        // the columns' forward representatives: loaded before the next piece's byte
        // stream, so their wait does not queue behind it (loads return in order)
        uint32_t rep[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) rep[c] = A.col2rep[tid + c * kBlock];
        PPiece Pn;
        g = pair_next_piece(A, g + 1, span_lo, span_hi, Pn);
        // flush (1): per forward 7-mer y, F(y) = sum_a P[4y + a] + sum_a P[a 4^7 + y];
        // thread t owns y = 2048 i + 2t + {0, 1}, i = 0..7 (lane-consecutive reads)
        uint32_t F[16];
        pair_f_sums(hist, tid, F);
        __syncthreads();   // (B) P read
#pragma unroll
        for (int i = 0; i < 8; ++i) *(uint2*)(hist + i * 2048 + 2 * tid) = make_uint2(F[2 * i], F[2 * i + 1]);
        // next piece: its first chunks taken and in flight under the rest of the flush
        // (not earlier: the ring and F together would not fit in 128 VGPRs)
        const uint32_t ctr_next = kPairCtl + 4 * (par ^ 1u);
#pragma unroll
        for (int j = 0; j < RING; ++j) {
            idx[j] = __builtin_amdgcn_readfirstlane(pair_grab(ctr_next, lane));
            buf[j] = pload(Pn, idx[j], lane);
        }
        __syncthreads();   // (C) F in LDS words [0, 16384)
        const uint16_t* S = (const uint16_t*)((const uint8_t*)hist + kPairSBase);
        uint32_t* gcf = A.counts + (uint64_t)gcur * A.nbins;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t y = rep[c], rc = kf_revcomp<K>(y);
            const uint32_t v = hist[y] + hist[rc] + S[s_fold(y, rc) & ((kPairCtl - kPairSBase) / 2 - 1)];
            if (v) __hip_atomic_fetch_add(gcf + tid + c * kBlock, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();   // (D) columns read
        for (uint32_t i = tid; i < kPairCtl / 16; i += kBlock) h4[i] = make_uint4(0u, 0u, 0u, 0u);
        if (tid == 0) hist[kPairCtl / 4 + par] = 0;   // this piece's counter, for the piece after next
        const uint64_t t_f2 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        __syncthreads();   // (E) P, S and the counter zero
        if (A.prof && tid == 0) {
            const uint64_t t_f3 = __builtin_amdgcn_s_memtime();
            atomicAdd(A.prof + 3, (unsigned long long)(t_f1 - t1));
            atomicAdd(A.prof + 4, 1ull);
            atomicAdd(A.prof + 5, (unsigned long long)(t_f2 - t_f1));
            atomicAdd(A.prof + 6, (unsigned long long)(t_f3 - t_f2));
        }
        if (g >= A.n_genomes) {
            if (A.prof && tid == 0) {
                const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
                atomicAdd(A.prof + 40, (unsigned long long)(__builtin_amdgcn_s_memtime() - tk0));
                atomicAdd(A.prof + 41, (unsigned long long)(rt1 - rt0));
                atomicMin(A.prof + 42, (unsigned long long)rt0);
                atomicMax(A.prof + 43, (unsigned long long)rt1);
                atomicMax(A.prof + 44, (unsigned long long)(rt1 - rt0));
                atomicMax(A.prof + 45, (unsigned long long)rt0);
            }
            break;
        }
        P = Pn;
        cur.load(A, P);   // re-base the interval cursor on the new piece
        par ^= 1u;
    }
}

// ---------------------------------------------------------------- k <= 7 dynamic-chunk kernel
// count_kernel's forward histogram (4^k u32 in LDS, two 1024-thread workgroups
// per CU) fed like the pair kernel: self-contained chunks (lane 0 = context)
// taken from an LDS counter.  The waves of a workgroup then finish a genome piece
// together instead of the flush waiting for the slowest SIMD slot (a static
// split left the oldest waves idle ~35 % of a piece), and no wave range needs a
// warm-up.

// Exact context before lane 1 of an irregular chunk whose lane-0 block B has tail
// own_t (lane 0's value): empty when that block is complete on its own, else the
// tail of the bytes before B (walk back, rare).
template <int K>
__device__ __forceinline__ uint32_t chunk_context(const CountArgs& A, const PPiece& P, uint64_t B, uint32_t own_t,
                                                  int lane) {
    uint32_t carry = tail_pack(0, 0, 0);
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)own_t, 0);
    if (!tail_complete<K>(t0)) {
        for (int64_t p = (int64_t)B; p > (int64_t)P.glo && !tail_complete<K>(carry);) {
            p -= kChunk;
            carry = tail_combine<K>(chunk_tail<K>(A.bytes, A.excl, A.n_excl, p, P.glo, lane), carry);
        }
    }
    return carry;
}

template <int K, bool MASKED>
__device__ __forceinline__ void count_chunk_fwd(const uint4 d, const CountArgs& A, const PPiece& P, uint32_t c,
                                                int lane, uint64_t iv0, uint32_t& lane_total) {
    constexpr uint32_t M4 = ((1u << (2 * K)) - 1u) << 2;
    if constexpr (!MASKED) {
        uint32_t Cf, NNL, bad;
        classify16_fast(d, Cf, NNL, bad);
        const uint32_t nef = (uint32_t)__builtin_popcount(NNL);
        const bool self_ok = bad == 0 && nef >= 15u;
        if (__builtin_amdgcn_ballot_w64(!self_ok) == 0) {
            // as count_chunk's fast case; lane 0's 15-16 bases are lane 1's context
            const uint32_t r = (uint32_t)__builtin_ctz((NNL ^ 0xFFFFu) | 0x10000u);
            const uint32_t lo1 = (1u << r) - 1u, lo2 = lo1 | (lo1 << r);
            const uint32_t C = bfi(lo2, Cf, Cf >> 2);
            const uint32_t pC = wave_shr1(0u, C);
            const uint32_t xlo = C << 2, xhi = (pC << ((2u * nef + 2u) & 31u)) | (C >> 30);
            uint32_t xv[8];
#pragma unroll
            for (int o = 0; o < 8; ++o) xv[o] = o ? __builtin_amdgcn_alignbit(xhi, xlo, 2 * o) : xlo;
            auto addr = [&](int w) -> uint32_t { return (w < 8 ? xv[w] : (xv[w - 8] >> 16)) & M4; };
            if (lane != 0) {
                const uint32_t inc15 = nef >> 4;   // window 15 exists iff no newline
#ifdef KF_K1_NOADD   // profiling only (tools/build_abl.sh): the fast path without its LDS adds
#pragma unroll
                for (int w = 0; w < 16; ++w) lane_total += addr(w);
#else
#pragma unroll
                for (int w = 0; w < 15; ++w) lds_add(addr(w), 1u);
                lds_add(addr(15), inc15);
#endif
                lane_total += 15u + inc15;
            }
            return;
        }
    }
    const uint64_t own = P.c0 + (uint64_t)kOwn * c;
    const uint64_t B = own - 16;   // lane 0's block (may lie before the genome: invalid)
    const ChunkMask m{P.glo, max(own, P.plo), min(own + kOwn, P.phi)};
    uint32_t C, V, EN, ne, own_t;
    front_end<K, true>(d, A, B, lane, m, iv0, C, V, EN, ne, own_t);
    const Windows win = windows<K, true>(C, V, EN, ne, chunk_context<K>(A, P, B, own_t, lane), lane);
    const uint32_t xlo = win.wlo << 2, xhi = __builtin_amdgcn_alignbit(win.whi, win.wlo, 30);
    uint32_t xv[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) xv[o] = o ? __builtin_amdgcn_alignbit(xhi, xlo, 2 * o) : xlo;
    auto addr = [&](int r) -> uint32_t { return (r < 8 ? xv[r] : (xv[r - 8] >> 16)) & M4; };
#pragma unroll
    for (int r = 0; r < 16; ++r) lds_add(addr(r), (win.R >> r) & 1u);
    lane_total += (uint32_t)__builtin_popcount(win.R);
}

template <int K, int V>
__global__ void __launch_bounds__(Shape<V>::block) __attribute__((amdgpu_waves_per_eu(Shape<V>::wpe, Shape<V>::wpe)))
    dyn_kernel(CountArgs A) {
    constexpr int kBlock = Shape<V>::block;
    constexpr int RING = Shape<V>::ring;
    constexpr uint32_t NCODES = 1u << (2 * K);
    constexpr uint32_t CTL = NCODES * 4;   // byte address of the chunk counter
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (uint32_t i = tid; i < NCODES + 4; i += kBlock) hist[i] = 0;
    __syncthreads();
    if ((uint32_t)(uintptr_t)(lds_u32*)hist != 0u) __builtin_trap();   // addresses assume LDS base 0

    const uint64_t base = A.goff[0];
    const uint64_t total = A.goff[A.n_genomes] - base;
    const uint64_t G = gridDim.x, b = blockIdx.x;
    const uint64_t span_lo = base + ((total / G * b + (total % G) * b / G) & ~(uint64_t)15);
    const uint64_t span_hi = (b + 1 == G) ? base + total
                                          : base + ((total / G * (b + 1) + (total % G) * (b + 1) / G) & ~(uint64_t)15);
    if (span_lo >= span_hi) return;
    const uint64_t tk0 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
    const uint64_t rt0 = A.prof ? __builtin_amdgcn_s_memrealtime() : 0;
    int32_t g = (int32_t)wave_upper_bound((uint64_t)A.n_genomes, span_lo, lane,
                                          [&](uint64_t i) { return A.goff[i + 1]; });
    PPiece P;
    g = pair_next_piece(A, g, span_lo, span_hi, P);
    IvCursor cur;
    cur.init(A, P.c0 >= 16 ? P.c0 - 16 : 0, lane);
    while (g < A.n_genomes) {
        cur.load(A, P);
        const uint64_t t0 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        uint32_t idx[RING];
        uint4 buf[RING];
#pragma unroll
        for (int j = 0; j < RING; ++j) {
            idx[j] = __builtin_amdgcn_readfirstlane(pair_grab(CTL, lane));
            buf[j] = pload(P, idx[j], lane);
        }
        uint32_t lt = 0, nproc = 0;
        for (;;) {
#pragma unroll
            for (int j = 0; j < RING; ++j) {
                const uint32_t tok = pair_grab(CTL, lane);   // refill of this slot, used below
                const uint32_t c = idx[j];
                if (c < P.nch) {
                    const uint32_t own_r = kOwn * c;
                    const bool msk = own_r < P.fast_lo || own_r + kOwn > P.fast_hi ||
                                     cur.hits(A, P, own_r, own_r + kChunk);
                    if (msk)
                        count_chunk_fwd<K, true>(buf[j], A, P, c, lane, cur.iv, lt);
                    else
                        count_chunk_fwd<K, false>(buf[j], A, P, c, lane, cur.iv, lt);
                    ++nproc;
                }
                idx[j] = __builtin_amdgcn_readfirstlane(tok);
                buf[j] = pload(P, idx[j], lane);
            }
            uint32_t mn = idx[0];
#pragma unroll
            for (int j = 1; j < RING; ++j) mn = min(mn, idx[j]);
            if (mn >= P.nch) break;
        }
        const unsigned long long s = wave_sum(lt);
        if (lane == 0 && s) atomicAdd(A.totals + g, s);
        const uint64_t t1 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        if (A.prof && lane == 0) {
            atomicAdd(A.prof + 1, (unsigned long long)(t1 - t0));
            atomicAdd(A.prof + 2, 1ull);
            atomicAdd(A.prof + 8 + wave, (unsigned long long)(t1 - t0));
            atomicAdd(A.prof + 24 + wave, (unsigned long long)nproc);
        }
        __syncthreads();
        const uint64_t t_f1 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        // canonical bin = forward count of the k-mer + forward count of its revcomp;
        // coalesced u32 atomics in column order, histogram re-zeroed on the way
        uint32_t* gc = A.counts + (uint64_t)g * A.nbins;
        for (uint32_t col = tid; col < A.nbins; col += kBlock) {
            const uint32_t rep = A.col2rep[col];
            const uint32_t rc = kf_revcomp<K>(rep);
            const uint32_t v = hist[rep] + (rc != rep ? hist[rc] : 0u);
            if (v) {
                hist[rep] = 0;
                hist[rc] = 0;
                __hip_atomic_fetch_add(gc + col, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (tid == 0) hist[NCODES] = 0;   // the chunk counter
        const uint64_t t_f2 = A.prof ? __builtin_amdgcn_s_memtime() : 0;
        __syncthreads();
        if (A.prof && tid == 0) {
            const uint64_t t_f3 = __builtin_amdgcn_s_memtime();
            atomicAdd(A.prof + 3, (unsigned long long)(t_f1 - t1));
            atomicAdd(A.prof + 4, 1ull);
            atomicAdd(A.prof + 5, (unsigned long long)(t_f2 - t_f1));
            atomicAdd(A.prof + 6, (unsigned long long)(t_f3 - t_f2));
        }
        g = pair_next_piece(A, g + 1, span_lo, span_hi, P);
    }
    if (A.prof && tid == 0) {
        const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
        atomicAdd(A.prof + 40, (unsigned long long)(__builtin_amdgcn_s_memtime() - tk0));
        atomicAdd(A.prof + 41, (unsigned long long)(rt1 - rt0));
        atomicMin(A.prof + 42, (unsigned long long)rt0);
        atomicMax(A.prof + 43, (unsigned long long)rt1);
        atomicMax(A.prof + 44, (unsigned long long)(rt1 - rt0));
        atomicMax(A.prof + 45, (unsigned long long)rt0);
        const int hb = blockIdx.x * 2 >= gridDim.x;
        atomicAdd(A.prof + 46 + hb, (unsigned long long)(rt1 - rt0));
        atomicMax(A.prof + 48 + hb, (unsigned long long)(rt1 - rt0));
        const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7u;   // HW_REG_XCC_ID[2:0]
        atomicAdd(A.prof + 56 + xcc, (unsigned long long)(rt1 - rt0));
        atomicMax(A.prof + 64 + xcc, (unsigned long long)(rt1 - rt0));
        atomicAdd(A.prof + 72 + xcc, 1ull);
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

__global__ void __launch_bounds__(256) synth_kernel(uint8_t* bytes, const uint64_t* goff, int64_t g0, int64_t gstride,
                                                     uint64_t seed0, uint64_t seq_len, int width, uint64_t n_period) {
    const int32_t gi = blockIdx.y;
    const uint64_t lo = goff[gi], hi = goff[gi + 1];
    const int64_t g = g0 + gi * gstride;
    // header ">syn_<g>\n"
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
// Reads a byte range with the count kernel's access pattern (per wave a
// contiguous range, 1 KiB chunks, 16 B per lane, 6-deep buffer-load ring) and
// XOR-folds it: the practical HBM read ceiling for this pattern (bench.py).
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

#ifdef KF_QUICK_ISA   // tools/isa.sh: one kernel's ISA without the whole variant zoo
template __global__ void kf::count_kernel<7, KF_QUICK_ISA>(kf::CountArgs);
#else
// ====================================================================== C-ABI
using namespace kf;

namespace {
template <int K, int V>
void* kernel_ptr() { return (void*)&count_kernel<K, V>; }

template <int V>
void* count_kernel_v(int k) {
    switch (k) {
    case 2: return kernel_ptr<2, V>();
    case 3: return kernel_ptr<3, V>();
    case 4: return kernel_ptr<4, V>();
    case 5: return kernel_ptr<5, V>();
    case 6: return kernel_ptr<6, V>();
    case 7: return kernel_ptr<7, V>();
    case 8: return kernel_ptr<8, V>();
    case 9: return kernel_ptr<9, V>();
    case 10: return kernel_ptr<10, V>();
    case 11: return kernel_ptr<11, V>();
    case 12: return kernel_ptr<12, V>();
    default: return nullptr;
    }
}

// Variants >= kFirstPairVariant are the pair kernel at k = 7 and variant 1 elsewhere.
bool is_pair(int k, int v) { return k == 7 && v >= kFirstPairVariant && v <= 7; }
bool is_dyn(int k, int v) { return k <= kLdsMaxK && (v == 8 || v == 9); }
bool is_static_pair(int k, int v) { return k == 7 && v >= 10 && v <= 23; }
bool is_k8x(int k, int v) { return k == 8 && v == 24; }
int effective_variant(int k, int v) {
    return (v >= kFirstPairVariant && !is_pair(k, v) && !is_dyn(k, v) && !is_static_pair(k, v) && !is_k8x(k, v)) ? 1
                                                                                                                : v;
}

template <int V>
void* dyn_kernel_v(int k) {
    switch (k) {
    case 2: return (void*)&dyn_kernel<2, V>;
    case 3: return (void*)&dyn_kernel<3, V>;
    case 4: return (void*)&dyn_kernel<4, V>;
    case 5: return (void*)&dyn_kernel<5, V>;
    case 6: return (void*)&dyn_kernel<6, V>;
    case 7: return (void*)&dyn_kernel<7, V>;
    default: return nullptr;
    }
}

void* count_kernel_for(int k, int v) {
    if (is_pair(k, v)) {
        if (v == 6) return (void*)&pair_kernel<6>;
        if (v == 7) return (void*)&pair_kernel<7>;
        return (void*)&pair_kernel<5>;
    }
    if (is_dyn(k, v)) return v == 9 ? dyn_kernel_v<9>(k) : dyn_kernel_v<8>(k);
    if (is_k8x(k, v)) return (void*)&count_kernel<8, 24>;
    if (is_static_pair(k, v)) {
        switch (v) {
        case 11: return (void*)&count_kernel<7, 11>;
        case 12: return (void*)&count_kernel<7, 12>;
        case 13: return (void*)&count_kernel<7, 13>;
        case 14: return (void*)&count_kernel<7, 14>;
        case 15: return (void*)&count_kernel<7, 15>;
        case 16: return (void*)&count_kernel<7, 16>;
        case 17: return (void*)&count_kernel<7, 17>;
        case 18: return (void*)&count_kernel<7, 18>;
        case 19: return (void*)&count_kernel<7, 19>;
        case 20: return (void*)&count_kernel<7, 20>;
        case 21: return (void*)&count_kernel<7, 21>;
        case 22: return (void*)&count_kernel<7, 22>;
        case 23: return (void*)&count_kernel<7, 23>;
        default: return (void*)&count_kernel<7, 10>;
        }
    }
    v = effective_variant(k, v);
#ifdef KF_ABLATION
    if (v == 3) return count_kernel_v<3>(k);
    if (v == 4) return count_kernel_v<4>(k);
#endif
    if (v == 2) return count_kernel_v<2>(k);
    return v == 0 ? count_kernel_v<0>(k) : count_kernel_v<1>(k);
}
int block_for(int v) { return v == 0 ? Shape<0>::block : Shape<1>::block; }   // all others 1024

// KF_BUCKET_MIN_K (A-B knob, read per launch): smallest k counted by the bucket
// kernels (kf_bucket.hip); below it k 8..9 use multi-pass LDS and k >= 10 global
// atomics.  Default 9.
int bucket_min_k() {
    const char* e = getenv("KF_BUCKET_MIN_K");
    if (!e || !*e) return kDefaultBucketMinK;
    const int v = atoi(e);
    return (v >= 9 && v <= KF_MAX_K + 1) ? v : kDefaultBucketMinK;
}

// KF_COUNT_VARIANT (tuning/A-B knob, read per launch): workgroup shape, see Shape<>.
// Default: K1x (variant 19) at k = 7, its k = 8 form (variant 24) at k = 8,
// variant 1 (K1 / K2) elsewhere.
int current_variant(int k) {
    const int dflt = k == 8 ? kDefaultVariantK8 : kDefaultVariant;
    const char* e = getenv("KF_COUNT_VARIANT");
    if (!e || !*e) return dflt;
    const int v = atoi(e);
    return (v >= 0 && v < kNumVariants) ? v : dflt;
}

// Variant 22's claim tickets: one u32 per workgroup (kClaimStride apart), per
// device and stream, allocated and zeroed on first use; a launch continues from
// the values the previous launch on that stream left, so nothing is reset per launch.
constexpr int kClaimMaxGrid = 1024;
uint32_t* claim_buffer(int dev, hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, uint32_t*> bufs;
    std::lock_guard<std::mutex> lk(mu);
    uint32_t*& p = bufs[{dev, s}];
    if (!p) {
        const size_t n = (size_t)kClaimMaxGrid * kClaimStride * sizeof(uint32_t);
        if (hipMalloc((void**)&p, n) != hipSuccess) return p = nullptr;
        if (hipMemset(p, 0, n) != hipSuccess) {
            (void)hipFree(p);
            return p = nullptr;
        }
    }
    return p;
}

// KF_DYN_FRAC (0..1, default 0.85): statically split share of a piece (variant 22);
// KF_DYN_UNIT (3 KiB iterations per claimed unit, 1..64, default 2).
uint32_t dyn_frac() {
    const char* e = getenv("KF_DYN_FRAC");
    double f = (e && *e) ? atof(e) : 0.85;
    if (!(f >= 0.0)) f = 0.0;
    if (f > 1.0) f = 1.0;
    return (uint32_t)(f * (double)(1u << 20));
}
uint32_t dyn_unit() {
    const char* e = getenv("KF_DYN_UNIT");
    int n = (e && *e) ? atoi(e) : 2;
    if (n < 1 || n > 64) n = 2;
    return (uint32_t)n * (uint32_t)kXChunk;
}

// KF_WAVE_WEIGHTS="a0,a1,a2,a3" (tuning/A-B knob, read per launch), each 1..255:
// K1x's share of a genome piece per wave of age slot 0..3 (split_at_w).
uint32_t wave_weights() {
    uint32_t w[4] = {kWaveW0, kWaveW1, kWaveW2, kWaveW3};
    const char* e = getenv("KF_WAVE_WEIGHTS");
    if (e && *e) {
        uint32_t t[4];
        if (sscanf(e, "%u,%u,%u,%u", &t[0], &t[1], &t[2], &t[3]) == 4 && t[0] >= 1 && t[0] <= 255 && t[1] >= 1 &&
            t[1] <= 255 && t[2] >= 1 && t[2] <= 255 && t[3] >= 1 && t[3] <= 255)
            for (int i = 0; i < 4; ++i) w[i] = t[i];
    }
    return w[0] | (w[1] << 8) | (w[2] << 16) | (w[3] << 24);
}

// histogram (4^k u32) + one u64 reduction slot per wave (16 waves max); pair
// kernel: P + S, nothing else
int lds_bytes_for(int k, int v) {
    if (is_pair(k, v)) return (int)kPairLdsBytes;
    if (is_static_pair(k, v) || is_k8x(k, v)) return (int)kFwdSEnd;
    if (is_dyn(k, v)) return (int)(sizeof(uint32_t) << (2 * k)) + 16;
    if (k <= kLdsMaxK) return (int)(sizeof(uint32_t) << (2 * k)) + 16 * 8;
    if (k <= kMultiMaxK) return (int)(sizeof(uint32_t) << kMultiBits) + 16 * 8;
    return 0;
}

struct LaunchCache {
    int grid[KF_MAX_K + 1][kNumVariants][64];
};
LaunchCache g_cache = {};
std::mutex g_cache_mu;

int launch_info(int k, int* grid, int* block, int* lds, int* variant) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kf_fail(KF_EHIP, "hipGetDevice failed");
    if (dev < 0 || dev >= 64) return kf_fail(KF_EINVAL, "device index out of range");
    const int v = current_variant(k);
    const int l = lds_bytes_for(k, v);
    std::lock_guard<std::mutex> lk(g_cache_mu);
    int& gr = g_cache.grid[k][v][dev];
    if (!gr) {
        void* fn = count_kernel_for(k, v);
        if (l > 0 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, l) != hipSuccess)
            return kf_fail(KF_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block_for(v), l) != hipSuccess)
            return kf_fail(KF_EHIP, "hipOccupancyMaxActiveBlocksPerMultiprocessor failed");
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return kf_fail(KF_EHIP, "hipDeviceGetAttribute(MultiprocessorCount) failed");
        if (per_cu < 1) per_cu = 1;
        // measurement knob: at most N workgroups per CU
        const char* e = getenv("KF_WGS_PER_CU");
        if (e && atoi(e) >= 1 && atoi(e) < per_cu) per_cu = atoi(e);
        gr = per_cu * cus;
    }
    *grid = gr;
    *block = block_for(v);
    *lds = l;
    *variant = v;
    return KF_OK;
}
}  // namespace

extern "C" int kf_count_launch_info(int k, int* grid, int* block, int* lds_bytes) {
    if (k < KF_MIN_K || k > KF_MAX_K) return kf_fail(KF_EINVAL, "k out of range [2, 12]");
    if (!grid || !block || !lds_bytes) return kf_fail(KF_EINVAL, "null output pointer");
    if (k >= bucket_min_k()) return bucket_launch_info(k, grid, block, lds_bytes);
    int v = 0;
    return launch_info(k, grid, block, lds_bytes, &v);
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
    const bool bucket = k >= bucket_min_k();
    if (!(flags & KF_ACCUMULATE)) {
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
    A.prof = nullptr;
    A.wave_w = wave_weights();
    A.flags = flags;
    const char* pe = getenv("KF_COUNT_PROFILE");   // debugging aid: synchronous, prints to stderr
    if (pe && *pe == '1' && !bucket) {
        if (hipMalloc((void**)&A.prof, 2304 * 8) != hipSuccess || hipMemsetAsync(A.prof, 0, 2304 * 8, s) != hipSuccess ||
            hipMemsetAsync(A.prof + 42, 0xFF, 8, s) != hipSuccess)
            return kf_fail(KF_EHIP, "profile buffer");
    }
    if (bucket) return bucket_launch(A, k, flags, s);
    int grid = 0, block = 0, lds = 0, variant = 0;
    int rc = launch_info(k, &grid, &block, &lds, &variant);
    if (rc) return rc;
    void* args[] = {&A};
    hipEvent_t pe0 = nullptr, pe1 = nullptr;
    if (A.prof && (hipEventCreate(&pe0) != hipSuccess || hipEventCreate(&pe1) != hipSuccess ||
                   hipEventRecord(pe0, s) != hipSuccess))
        return kf_fail(KF_EHIP, "profile events");
    A.claim = nullptr;
    A.dyn_frac = dyn_frac();
    A.dyn_unit = dyn_unit();
    if (k == 7 && (variant == 22 || variant == 23)) {
        int dev = 0;
        if (grid > kClaimMaxGrid) return kf_fail(KF_EINVAL, "grid %d exceeds the claim buffer", grid);
        if (hipGetDevice(&dev) != hipSuccess || !(A.claim = claim_buffer(dev, s)))
            return kf_fail(KF_EHIP, "claim buffer allocation failed");
    }
    if (hipLaunchKernel(count_kernel_for(k, variant), dim3(grid), dim3(block), args, (size_t)lds, s) != hipSuccess)
        return kf_fail(KF_EHIP, "count kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (A.prof) {
        static unsigned long long h[2304];
        float ms = 0.f;
        if (hipEventRecord(pe1, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess ||
            hipEventElapsedTime(&ms, pe0, pe1) != hipSuccess ||
            hipMemcpy(h, A.prof, sizeof h, hipMemcpyDeviceToHost) != hipSuccess)
            return kf_fail(KF_EHIP, "profile readback");
        (void)hipEventDestroy(pe0);
        (void)hipEventDestroy(pe1);
        fprintf(stderr, "  kernel %.3f ms (events); workgroup lifetime mean %.3f max %.3f ms; first start to "
                "last end %.3f ms, last start %.3f ms after the first\n", ms, (double)h[41] / (double)grid * 1e-5,
                (double)h[44] * 1e-5, (double)(h[43] - h[42]) * 1e-5, (double)(h[45] - h[42]) * 1e-5);
        fprintf(stderr, "  first half of the grid: mean %.3f max %.3f ms; second half: mean %.3f max %.3f ms\n",
                (double)h[46] / (double)(grid / 2) * 1e-5, (double)h[48] * 1e-5,
                (double)h[47] / (double)(grid - grid / 2) * 1e-5, (double)h[49] * 1e-5);
        (void)hipFree(A.prof);
        const double nf = h[4] ? (double)h[4] : 1.0, nr = h[2] ? (double)h[2] : 1.0;
        fprintf(stderr, "[count_kernel k=%d] wave ranges %llu: setup %.3g cyc/range, loop %.3g cyc/range; "
                "flushes %llu (wave 0): barrier-in %.3g, flush %.3g, barrier-out %.3g cyc\n", k, h[2],
                (double)h[0] / nr, (double)h[1] / nr, h[4], (double)h[3] / nf, (double)h[5] / nf, (double)h[6] / nf);
        if (h[41])
            fprintf(stderr, "  shader clock %.3f GHz over the workgroups' lifetimes\n", (double)h[40] / (double)h[41] * 0.1);
        for (int x = 0; x < 8; ++x)
            if (h[72 + x])
                fprintf(stderr, "  XCC %d: %llu workgroups, lifetime mean %.3f max %.3f ms\n", x, h[72 + x],
                        (double)h[56 + x] / (double)h[72 + x] * 1e-5, (double)h[64 + x] * 1e-5);
        const char* tl = getenv("KF_COUNT_TIMELINE");   // per-piece timeline of workgroup 0 (cycles from its start)
        if (tl && *tl == '1') {
            const unsigned long long z = h[112];
            for (int pc = 0; pc < 8; ++pc) {
                if (!h[112 + pc * 16 * 16]) break;
                fprintf(stderr, "  piece %d (top, setup, loop, end, barrier-in, barrier-out, sums, P read, F written, "
                        "columns, columns read, zeroed) per wave:\n", pc);
                for (int w = 0; w < 16; ++w) {
                    const unsigned long long* t = h + 112 + (pc * 16 + w) * 16;
                    fprintf(stderr, "    w%2d", w);
                    for (int q = 0; q < 12; ++q) fprintf(stderr, " %9lld", t[q] ? (long long)(t[q] - z) : -1ll);
                    fprintf(stderr, "\n");
                }
            }
        }
        for (int w = 0; w < 16; ++w)
            if (h[24 + w])
                fprintf(stderr, "  wave %2d: %.0f cyc/chunk over %llu chunks, setup %.3g, barrier wait %.3g cyc/piece\n", w,
                        (double)h[8 + w] / h[24 + w], h[24 + w], (double)h[96 + w] / nf, (double)h[80 + w] / nf);
    }
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
    const char* wpc = getenv("KF_PROBE_WGS_PER_CU");   // measurement knob: 1024-thread workgroups per CU
    const int per_cu = (wpc && atoi(wpc) >= 1 && atoi(wpc) <= 2) ? atoi(wpc) : 2;
    hipLaunchKernelGGL(stream_probe_kernel, dim3(per_cu * (cus > 0 ? cus : 1)), dim3(1024), 0, (hipStream_t)stream,
                       d_bytes, n, d_out);
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
#endif  // KF_QUICK_ISA
