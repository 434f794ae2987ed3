// kf_bucket.hip -- canonical k-mer counting for large k (4^k bins beyond LDS).
//
// Reference path: kf2vec/main.py:309-323 (`jellyfish count -C -m k` + dump), the
// same as kf_count.hip; this file serves k >= kBucketMinK, where one genome's
// canonical bins (2,097,152 at k=11) do not fit a 160 KiB LDS and per-k-mer
// global atomics run at ~25 G/s (measured), far below the byte stream.
//
// Two phases per genome piece, one workgroup (16 waves) per piece:
//   1. scatter: each wave walks its range of the piece with the shared front end
//      (kf_front.h); every counted window yields its canonical code in
//      lexicographic (A0 C1 G2 T3) order, s = min(fwd, revcomp).  Rounds of
//      16 chunks (one per wave, 16384 windows) are counting-sorted in LDS by
//      bucket b = s >> 15 and copied out contiguously; per round the bucket
//      offsets go to `meta`.
//   2. count: for each bucket, the runs of that bucket from every round are
//      histogrammed in LDS (32768 u32 = 128 KiB, index s & 0x7FFF) and flushed in
//      column order: columns are the canonical codes in ascending order, so a
//      bucket owns a contiguous column range [bcol[b], bcol[b+1]) and the flush
//      writes counts with coalesced stores (col_idx[col] = s & 0x7FFF).
// Traffic per input byte: read 1 B, write and re-read 2 B of records, plus the
// 4 B x nbins count row per genome.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <cstdio>
#include <mutex>
#include <vector>

#include "kf_front.h"
#include "kf_internal.h"

namespace kf {

// (The profiling ablations of rounds 3-5 -- wrong counts by design -- live in
// tools/zoo/bucket_ablations.patch, applied by `python -m kf2vecfsw_amd.build
// --ablation`; DESIGN.md section 4 lists them.)
// Phase 2 record groups: 1 = two groups of 4 windows alternate (the next one in
// flight while one is counted), 0 = one group of 8 windows (a bucket's further
// groups wait for their loads).
#ifndef KF_BK_DB
#define KF_BK_DB 1
#endif
// With KF_BK_DB, k <= 10: both groups of the next bucket are issued before the
// current bucket's flush, so its first two groups never wait for loads issued
// after the flush (one process: k=9 6.10 -> 5.83 ms, k=10 6.71 -> 6.52).  k >= 11
// issues one: k=11 buckets need ~1.2 groups per wave (8.69 vs 8.73 ms) and k=12
// ~0.3 (18.9 vs 19.2), so a second group is mostly empty loads.
#ifndef KF_BK_PRE2
#define KF_BK_PRE2 1
#endif
// Non-temporal stores for the record copy-out and the count rows: k=11 9.61 ->
// 8.97 ms, k=9 unchanged (one process, profiles/r03/v10_lib_ab_k*_nt_stores.json).
#ifndef KF_NT_STORES
#define KF_NT_STORES 1
#endif
// Staggered phases (see the piece loop) for k >= KF_BK_LAG (0: never): half of
// the workgroups run one phase behind the others, with two record slots per
// workgroup.  One process (profiles/r03/v18_lib_ab_k*_lag.json): k=10 6.55 ->
// 6.50 ms, k=11 8.71 -> 8.46, k=12 18.67 -> 18.26; k=9 5.69 -> 5.92 (off).
#ifndef KF_BK_LAG
#define KF_BK_LAG 10
#endif
#ifndef KF_BK_LAG_SHIFT   // lagged workgroups: bit KF_BK_LAG_SHIFT of blockIdx.x (3: half of each XCD)
#define KF_BK_LAG_SHIFT 3
#endif
#ifndef KF_BK_PRE2_MAXK   // KF_BK_PRE2 applies to k <= this
#define KF_BK_PRE2_MAXK 10
#endif
// Phase-2 rounds per wave: 0 = dealt round-robin (round wave + W j); otherwise a
// contiguous block of rounds per wave, its size proportional to byte (wave >> 2)
// of KF_BK_RW (the wave's age slot on its SIMD, as K1x's KF_WAVE_WEIGHTS): the
// SIMD issues its oldest wave first, so equal shares leave the older waves
// waiting at every bucket barrier for the youngest.
#ifndef KF_BK_RW
#define KF_BK_RW 0x060B1114   // (20, 17, 11, 6): k=11 8.35 -> 8.17 ms, k=9 unchanged (profiles/r04/v6_lib_ab_k*_rw_dup.json)
#endif
constexpr uint32_t kBkSlots = KF_BK_LAG ? 2u : 1u;   // record / meta / roff slots per workgroup
// Wave priority by age slot (tools/ A/B builds): bit 0 = phase 1, bit 1 = phase 2
// run at s_setprio(wave >> 2), so that the youngest wave of each SIMD (which the
// SIMD issues last) is not the one every barrier waits for.
#ifndef KF_BK_PRIO
#define KF_BK_PRIO 0
#endif
// Phase-1 staging slots (tools/ A/B builds): 1 = record position p goes to u16
// slot p with bits 0 and 2 swapped inside its 8-record unit, so the consecutive
// ranks one ds_add_rtn hands the lanes of a bucket land in different dwords
// (banks) instead of pairs sharing one; phase 2 counts a unit in any order.
// Measured and left off (profiles/r05/k11ab_*): phase-1 bank-conflict cycles
// unchanged (1.050e9 -> 1.066e9 at k = 11: same-dword pairs are not conflicts),
// VALU instructions +46 %, k = 11 8.59 -> 8.85 ms, k = 9/10/12 slower as well.
#ifndef KF_BK_SWZ
#define KF_BK_SWZ 0
#endif
__device__ __forceinline__ uint32_t stage_slot(uint32_t p) {
    if (!KF_BK_SWZ) return p;
    const uint32_t x = (p ^ (p >> 2)) & 1u;
    return p ^ (x | (x << 2));
}
__device__ __forceinline__ void bk_setprio(uint32_t p) {   // p wave-uniform
    if (p == 0) __builtin_amdgcn_s_setprio(0);
    else if (p == 1) __builtin_amdgcn_s_setprio(1);
    else if (p == 2) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(3);
}

// Workgroup shape (per k, compile time): W = 16 waves, one workgroup per CU,
// 32768-code buckets (a 128 KiB histogram); or W = 8 waves, two workgroups per
// CU, 16384-code buckets (64 KiB), so that one workgroup's barrier waits are
// filled by the other's waves and the two phases of different pieces overlap on
// one CU.  KF_BK_W<k> (tools/ A/B builds):
#ifndef KF_BK_W9
#define KF_BK_W9 16
#endif
#ifndef KF_BK_W10
#define KF_BK_W10 16
#endif
#ifndef KF_BK_W11
#define KF_BK_W11 16
#endif
constexpr int bk_w(int K) { return K == 9 ? KF_BK_W9 : K == 10 ? KF_BK_W10 : K == 11 ? KF_BK_W11 : 16; }
// bytes per piece (one workgroup): a wave range is <= piece / W + 16 bytes, so
// <= 1017 rounds at W = 8 (<= 128 phase-2 runs per wave, two per lane) and <= 509
// at W = 16
constexpr uint64_t kPieceMax = (8ull << 20) - (64ull << 10);
template <int W>
struct BkGeom {
    static_assert(W == 8 || W == 16, "8 or 16 waves");
    static constexpr int waves = W;
    static constexpr int block = W * kWave;
    static constexpr int bits = W == 16 ? 15 : 14;                        // code bits per bucket
    static constexpr uint32_t codes = 1u << bits;
    static constexpr uint32_t round_recs = W * kChunk;                   // windows per round
    static constexpr uint32_t rmax = (uint32_t)(kPieceMax / round_recs) + 2;   // rounds per piece
    static constexpr int halves = (rmax + W * kWave - 1) / (W * kWave);   // phase-2 runs per lane
    static_assert(halves <= 2, "phase-2 run tables hold two runs per lane");
};
// A record is the low 16 bits of s: its code in the bucket (s mod codes) plus the
// bucket's low 16 - bits bits (the same for a whole bucket; phase 1 stores s as
// it is, one op less per window).  Runs (one bucket, one round) are padded to
// whole 8-record units with sentinels x | ((b ^ 1) mod 2^(16-bits)) << bits
// (x < 64).  Phase 2 XORs each record with bucket b's high part (b mod
// 2^(16-bits)) << bits: records become s mod codes, sentinels codes + x, a trash
// area past the histogram, so a 16-byte unit never needs a range test.

// Phase-1 rank counters: each bucket's round counter is split into R = 2^rl
// lane replicas (lane L ranks into replica L mod R), so the 64 lanes of one
// ds_add_rtn spread over the banks instead of piling onto the few counters of
// random buckets.  A round's table has nbk x R entries (bucket major), 1 to 8
// per lane.  Measured (tools/lds_rank_rate.hip, cycles per wave-instruction per
// CU): 8 shared counters 28.7 -> 7.3 with 64 replicas; 32: 13.7 -> 7.3; 128:
// 11.2 -> 8.7 with 4.  In the kernel (profiles/r03/v5_lib_ab_k*_rank_replicas.json,
// one process): k = 9 R = 32 6.39 ms (shared counters 9.05), k = 10 R = 16 7.27
// (7.51); k = 11 stays at R = 1: R = 4 measured 9.59 vs 9.24 in round 3 (its
// 512-entry tables cost more than the conflicts they remove), and R = 2 leaves
// phase 1's bank-conflict cycles where they were (1.05e9 -> 1.10e9) and its time
// too (processes alternated: 8.58 vs 8.58 ms; profiles/r05/k11ab3_*).  log2 R
// per k (KF_BK_RL<k>, tools/ only):
#ifndef KF_BK_RL9
#define KF_BK_RL9 5
#endif
#ifndef KF_BK_RL10
#define KF_BK_RL10 4
#endif
#ifndef KF_BK_RL11
#define KF_BK_RL11 0
#endif
#ifndef KF_BK_RL12
#define KF_BK_RL12 0
#endif
constexpr uint32_t bk_rl(int K) {
    return K == 9 ? KF_BK_RL9 : K == 10 ? KF_BK_RL10 : K == 11 ? KF_BK_RL11 : KF_BK_RL12;
}

template <int K, int W = bk_w(K)>
struct Bk : BkGeom<W> {
    using G = BkGeom<W>;
    static constexpr uint32_t nbk = (1u << (2 * K)) >> G::bits;   // buckets
    // (W = 8: twice the buckets, half the replicas: the same counter count)
    static constexpr uint32_t rl = W == 16 || bk_rl(K) == 0 ? bk_rl(K) : bk_rl(K) - 1;
    static constexpr uint32_t nrep = 1u << rl;                      // rank replicas per bucket
    static constexpr uint32_t nent = nbk << rl;                     // rank entries per round
    static constexpr uint32_t epl = nent / kWave;                   // rank entries per lane
    static constexpr uint32_t round_cap = G::round_recs + 7 * nbk;  // records of a padded round
    static constexpr uint64_t rec_cap = (uint64_t)G::rmax * round_cap + 8;   // per workgroup
    // LDS byte layout.  Phase 2: the histogram (codes u32) at 0.  Phase 1 reuses it:
    // two round staging buffers, then one private rank-entry offset table per
    // wave.  After the histogram: three rotating sets of round rank counters
    // (phase 1), which phase 2 reuses as the sentinels' trash bins, and the
    // reduction slots.
    static constexpr uint32_t hist = 0;
    static constexpr uint32_t stage_bytes = (round_cap * 2 + 15) & ~15u;
    static constexpr uint32_t stage = 0;                            // + (r & 1) * stage_bytes
    static constexpr uint32_t tbl_bytes = nent * 4 + 16;            // per wave (16-byte aligned)
    static constexpr uint32_t rbase = 2 * stage_bytes;              // + wave * tbl_bytes
    static constexpr uint32_t dirty = rbase + W * tbl_bytes;       // phase-1 footprint in hist
    static constexpr uint32_t cnt = G::codes * 4;                   // + (r % 3) * nent * 4
    static constexpr uint32_t red = (cnt + 3 * nent * 4 + 7) & ~7u; // W u64
    static constexpr uint32_t lds_bytes =
        red + W * 8 > cnt + 256 ? red + W * 8 : cnt + 256;         // trash: 64 bins at cnt
    static constexpr uint32_t hmask = (1u << (16 - G::bits)) - 1u;  // bucket bits inside a record
    static_assert(epl >= 1 && epl <= 8 && (epl & (epl - 1)) == 0 && nent == epl * kWave, "1-8 entries per lane");
    static_assert(dirty <= G::codes * 4, "phase-1 tables must fit the histogram area");
    static_assert(lds_bytes * (16 / W) <= 160 * 1024, "LDS (16 / W workgroups per CU)");
    static_assert(round_cap < 65536, "round offsets are u16");
};

struct BucketArgs {
    const uint16_t* col_idx;   // nbins: canonical code mod codes per column
    const uint32_t* bcol;      // nbk+1: first column of each bucket
    const uint32_t* pstart;    // n_genomes+1: first piece of each genome
    uint16_t* rec;             // gridDim.x * Bk<K>::rec_cap records
    uint16_t* meta;            // gridDim.x * (nbk+1) * rmax round bucket offsets
    uint32_t* roff;            // gridDim.x * rmax round record offsets
    uint32_t accumulate;
    uint32_t skew;              // record slot i starts skew x hash(i) (0..63) records later
    unsigned long long* prof;   // optional (KF_BUCKET_PROFILE): per-workgroup phase cycles
};
// Record slot i of the scratch (one per workgroup and lag slot).
__device__ __forceinline__ uint16_t* rec_slot(const BucketArgs& B, uint64_t i, uint64_t cap) {
    return B.rec + i * cap + (uint64_t)(((uint32_t)i * 0x9E3779B1u) >> 26) * B.skew;
}

typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4u lds_v4u;

__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t a, uint32_t v) {
    return __hip_atomic_fetch_add((lds_u32*)(uintptr_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_xchg(uint32_t a, uint32_t v) {
    return __hip_atomic_exchange((lds_u32*)(uintptr_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Byte address (x 4) of the record in u16 half h of d: one SDWA shift.
__device__ __forceinline__ uint32_t rec_addr(uint32_t d, int h) {
    uint32_t r;
    if (h == 0)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
            : "=v"(r) : "v"(d));
    else
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
            : "=v"(r) : "v"(d));
    return r;
}
// v_bfe_u32 the compiler cannot take apart: (bfe(s) << n) + base then stays one
// v_lshl_add / v_lshl_or instead of lshr + and + add.
template <int OFF, int W>
__device__ __forceinline__ uint32_t bfe_opaque(uint32_t s) {
    uint32_t r;
    asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(r) : "v"(s), "i"(OFF), "i"(W));
    return r;
}
__device__ __forceinline__ uint32_t lds_ld(uint32_t a) { return *(volatile lds_u32*)(uintptr_t)a; }
__device__ __forceinline__ void lds_st(uint32_t a, uint32_t v) { *(volatile lds_u32*)(uintptr_t)a = v; }
typedef unsigned int v2u_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2u_t lds_v2u;
// N consecutive words at a (N = 1, 2, 4, 8; a aligned to min(4 N, 16) bytes)
template <uint32_t N>
__device__ __forceinline__ void lds_ldn(uint32_t a, uint32_t (&v)[N]) {
    if constexpr (N == 1) {
        v[0] = lds_ld(a);
    } else if constexpr (N == 2) {
        const v2u_t x = *(volatile lds_v2u*)(uintptr_t)a;
        v[0] = x.x, v[1] = x.y;
    } else {
#pragma unroll
        for (uint32_t i = 0; i < N / 4; ++i) {
            const v4u x = *(volatile lds_v4u*)(uintptr_t)(a + 16 * i);
            v[4 * i] = x.x, v[4 * i + 1] = x.y, v[4 * i + 2] = x.z, v[4 * i + 3] = x.w;
        }
    }
}
template <uint32_t N>
__device__ __forceinline__ void lds_stn(uint32_t a, const uint32_t (&v)[N]) {
    if constexpr (N == 1) {
        lds_st(a, v[0]);
    } else if constexpr (N == 2) {
        *(volatile lds_v2u*)(uintptr_t)a = v2u_t{v[0], v[1]};
    } else {
#pragma unroll
        for (uint32_t i = 0; i < N / 4; ++i)
            *(volatile lds_v4u*)(uintptr_t)(a + 16 * i) = v4u{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
    }
}
// Barrier for LDS traffic only: outstanding global loads (the byte-stream
// prefetch) stay in flight across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Number of pieces of a genome of `len` bytes (an empty genome still gets one:
// its count row is written by the piece's flush).
__device__ __forceinline__ uint32_t n_pieces(uint64_t len) {
    return len == 0 ? 1u : (uint32_t)((len + kPieceMax - 1) / kPieceMax);
}

// pstart[g] = sum of n_pieces over genomes < g; one workgroup.
__global__ void __launch_bounds__(1024) piece_scan_kernel(const uint64_t* goff, int32_t n, uint32_t* pstart) {
    __shared__ uint32_t sh[1024];
    const int t = threadIdx.x;
    uint32_t carry = 0;
    for (int32_t base = 0; base < n; base += 1024) {
        const int32_t i = base + t;
        const uint32_t v = i < n ? n_pieces(goff[i + 1] - goff[i]) : 0u;
        sh[t] = v;
        __syncthreads();
        for (int d = 1; d < 1024; d <<= 1) {
            const uint32_t o = t >= d ? sh[t - d] : 0u;
            __syncthreads();
            sh[t] += o;
            __syncthreads();
        }
        if (i < n) pstart[i] = carry + sh[t] - v;
        carry += sh[1023];
        __syncthreads();
    }
    if (t == 0) pstart[n] = carry;
}

// Zero the count rows of genomes split into several pieces (their pieces add
// with atomics); single-piece rows are written whole by their flush.
__global__ void __launch_bounds__(256) zero_split_rows_kernel(const uint64_t* goff, int32_t n, uint32_t* counts,
                                                               uint32_t nbins) {
    for (int32_t g = blockIdx.x; g < n; g += gridDim.x) {
        if (n_pieces(goff[g + 1] - goff[g]) <= 1) continue;
        uint32_t* row = counts + (uint64_t)g * nbins;
        for (uint32_t i = threadIdx.x; i < nbins; i += 256) row[i] = 0;
    }
}

// Canonical lexicographic codes of the 16 windows of a lane (kf codes in W).
// std code = kf ^ ((kf >> 1) & 0x55..) per base (A0 C1 T2 G3 -> A0 C1 G2 T3);
// complement in std code = code ^ 3, so the reversed complement of the whole
// 64-bit window register is ~revpairs, word-swapped.  DENSE (fast_windows):
// windows 0..14 are valid by construction, so only window 15 is tested.
template <int K, bool DENSE = false>
__device__ __forceinline__ void canon_std(const Windows& w, uint32_t (&s)[16]) {
    constexpr int W2 = 2 * K;
    const uint32_t slo = w.wlo ^ ((w.wlo >> 1) & 0x55555555u);
    const uint32_t shi = w.whi ^ ((w.whi >> 1) & 0x55555555u);
    const uint32_t rhi = ~revpairs(slo), rlo = ~revpairs(shi);
    constexpr int RS = 2 * (17 - K);
    const uint32_t rplo = __builtin_amdgcn_alignbit(rhi, rlo, RS), rphi = rhi >> RS;
    const uint32_t fv[4] = {slo, __builtin_amdgcn_alignbit(shi, slo, 8), __builtin_amdgcn_alignbit(shi, slo, 16),
                            __builtin_amdgcn_alignbit(shi, slo, 24)};
    const uint32_t rv[4] = {rplo, __builtin_amdgcn_alignbit(rphi, rplo, 8), __builtin_amdgcn_alignbit(rphi, rplo, 16),
                            __builtin_amdgcn_alignbit(rphi, rplo, 24)};
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int fo = (2 * r) & ~7;
        const uint32_t f = __builtin_amdgcn_ubfe(fv[fo >> 3], 2 * r - fo, W2);
        const int rr = 2 * (15 - r), ro = rr & ~7;
        const uint32_t c = __builtin_amdgcn_ubfe(rv[ro >> 3], rr - ro, W2);
        s[r] = ((DENSE && r < 15) || ((w.R >> r) & 1u)) ? min(f, c) : 0xFFFFFFFFu;
    }
}

// Window register of a 1 KiB chunk in the fast case (uniform): every lane's 16
// bytes are bases with at most one newline and the carry is complete (>= k-1
// bases).  Then the context is lane L-1's raw codes and no validity mask, tail
// or run mask is needed: windows 0..ne-1 are valid (ne = 15 or 16).  Returns
// false (w untouched) otherwise; the caller takes the general path.
template <int K>
__device__ __forceinline__ bool fast_windows(const uint4 d, uint32_t carry, Windows& w) {
    constexpr uint32_t TM = (1u << (2 * (K - 1))) - 1u;
    static_assert(K - 1 <= 11, "the carry holds 11 entries");
    uint32_t Cf, NNL, bad;
    classify16_fast(d, Cf, NNL, bad);
    const uint32_t nef = (uint32_t)__builtin_popcount(NNL);
    const bool self_ok = bad == 0 && nef >= 15u;
    carry = __builtin_amdgcn_readfirstlane(carry);
    if (t_n(carry) < (uint32_t)(K - 1) || __builtin_amdgcn_ballot_w64(!self_ok) != 0) return false;
    // drop the newline entry (none: r = 16, identity)
    const uint32_t r = (uint32_t)__builtin_ctz((NNL ^ 0xFFFFu) | 0x10000u);
    const uint32_t lo1 = (1u << r) - 1u, lo2 = lo1 | (lo1 << r);
    const uint32_t C = bfi(lo2, Cf, Cf >> 2);
    const uint32_t pC = wave_shr1(t_codes(carry), C);
    const uint64_t W = ((uint64_t)pC << (2u * nef)) | (uint64_t)C;
    w.wlo = (uint32_t)W;
    w.whi = (uint32_t)(W >> 32);
    w.R = (1u << nef) - 1u;
    // lane 63's block is all valid bases: its tail is complete
    w.next = tail_pack((uint32_t)__builtin_amdgcn_readlane((int)C, kWave - 1) & TM, 31u, 31u);
    return true;
}

template <int K>
__global__ void __launch_bounds__(Bk<K>::block) __attribute__((amdgpu_waves_per_eu(4, 4)))   // 16 waves per CU
bucket_kernel(CountArgs A, BucketArgs B) {
    using L = Bk<K>;
    constexpr int W = L::waves;
    constexpr uint32_t NBK = L::nbk;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((uint32_t)(uintptr_t)(lds_u32*)lds != 0u) __builtin_trap();   // raw LDS addresses assume base 0
    for (uint32_t i = tid; i < L::codes + NBK; i += L::block) lds[i] = 0;   // histogram + counters
    __syncthreads();

    const uint32_t npiece = B.pstart[A.n_genomes];
    // This workgroup's pieces are blockIdx.x + i gridDim.x (i < nmine).  With
    // lag = 1 it runs phase 1 of piece i before phase 2 of piece i - 1 (two record
    // slots), so that half of the CUs (every other group of 8 workgroups: half of
    // each XCD) are in the LDS-bound phase 1 while the others stream phase 2's
    // records and rows, instead of all CUs switching phase together.
    constexpr bool kLagK = KF_BK_LAG && K >= KF_BK_LAG;
    const uint32_t lag = kLagK ? ((blockIdx.x >> KF_BK_LAG_SHIFT) & 1u) : 0u;
    const uint32_t nmine = blockIdx.x < npiece ? (npiece - 1u - blockIdx.x) / gridDim.x + 1u : 0u;
    struct Piece {
        int32_t g;
        uint32_t np, pi, nround;
        uint64_t glo, ghi, plo, phi;
    };
    auto piece_at = [&](uint32_t p) -> Piece {
        Piece P;
        // genome of piece p: last g with pstart[g] <= p
        P.g = (int32_t)wave_upper_bound((uint64_t)A.n_genomes, p, lane,
                                        [&](uint64_t i) { return (uint64_t)B.pstart[i]; }) - 1;
        P.np = B.pstart[P.g + 1] - B.pstart[P.g];
        P.pi = p - B.pstart[P.g];
        P.glo = A.goff[P.g];
        P.ghi = A.goff[P.g + 1];
        P.plo = split_at(P.glo, P.ghi, P.pi, P.np);
        P.phi = split_at(P.glo, P.ghi, P.pi + 1, P.np);
        // rounds = the longest wave range in chunks (same value in every wave)
        P.nround = 0;
        for (int w = 0; w < W; ++w) {
            const uint64_t a = split_at(P.plo, P.phi, w, W), e = split_at(P.plo, P.phi, w + 1, W);
            if (e > a) P.nround = max(P.nround, (uint32_t)((e - (a & ~(uint64_t)15) + kChunk - 1) / kChunk));
        }
        return P;
    };

    for (uint32_t it = 0; it < nmine + lag; ++it) {
      if (it < nmine) {
        const uint32_t slot = kLagK ? (it & 1u) : 0u;
        uint16_t* rec = rec_slot(B, (uint64_t)blockIdx.x * kBkSlots + slot, L::rec_cap);
        uint16_t* meta = B.meta + ((uint64_t)blockIdx.x * kBkSlots + slot) * (NBK + 1) * L::rmax;
        uint32_t* roff = B.roff + ((uint64_t)blockIdx.x * kBkSlots + slot) * L::rmax;
        const Piece P = piece_at(blockIdx.x + it * gridDim.x);
        const int32_t g = P.g;
        const uint64_t glo = P.glo, ghi = P.ghi, plo = P.plo, phi = P.phi;
        const uint32_t nround = P.nround;
        const uint64_t lo = split_at(plo, phi, wave, W), hi = split_at(plo, phi, wave + 1, W);
        (void)g;

        // ---------------------------------------------------------- phase 1
        const uint64_t t_p1 = B.prof ? __builtin_amdgcn_s_memtime() : 0;
        if (KF_BK_PRIO) bk_setprio((KF_BK_PRIO & 1) ? (uint32_t)wave >> 2 : 0u);
        Range rg;
        uint32_t nch = 0;
        if (lo < hi) {
            rg.init(glo, ghi, lo, hi);
            nch = rg.nch;
        }
        uint4 buf[4];   // the first chunks go out before the warm-up's dependent loads
#pragma unroll
        for (int j = 0; j < 4; ++j)
            buf[j] = (uint32_t)j < nch ? rg.load(A.bytes, j * kChunk, lane) : make_uint4(0u, 0u, 0u, 0u);
        if (lo < hi) rg.warm<K>(A, lane);
        uint32_t carry = lo < hi ? rg.carry : 0u;
        uint32_t rel = 0;
        // One barrier per round.  Round r: zero the counter set of round r+1,
        // count + rank this round's records in set r % 3, barrier; then copy out
        // round r-1 (staged in the other buffer before this barrier), every wave
        // computes the bucket offsets of round r into its private table (no
        // serial scan, no second barrier), and stages its records.  A counter set
        // is zeroed two rounds after its last read, so the barriers order it.
        for (uint32_t i = tid; i < 3 * L::nent; i += L::block) lds_st(L::cnt + 4 * i, 0u);
        lds_barrier();
        uint64_t p1w = 0;                    // profile: phase-1 barrier wait of this wave
        uint32_t off = 0;                    // records of rounds before the current one (x8)
        uint32_t t_prev = 0, off_prev = 0;   // last staged round, copied out one round later
        const uint32_t rb = L::rbase + (uint32_t)wave * L::tbl_bytes;
        // byte offset of the rank entry of canonical code s for this lane (its replica)
        const uint32_t repo = ((uint32_t)lane & (L::nrep - 1u)) << 2;
        // bucket part of the entry offset (one bfe; the lshl folds into the
        // address op): a counter set base is 4 nent aligned, so `cb | ent` = cb + ent
        auto ent_b = [&](uint32_t s) -> uint32_t { return bfe_opaque<L::bits, 2 * K - L::bits>(s) << (L::rl + 2); };
        static_assert((L::cnt % (4 * L::nent)) == 0, "counter sets are 4 nent aligned");
        auto copy_out = [&](uint32_t r, uint32_t T, uint32_t o) {
            const uint32_t st = L::stage + (r & 1) * L::stage_bytes;
            for (uint32_t q = tid; q < T / 8; q += L::block) {
                const v4u v = *(lds_v4u*)(uintptr_t)(st + 16 * q);
#if KF_NT_STORES
                __builtin_nontemporal_store(v, (v4u*)(rec + o + 8 * q));
#else
                *(v4u*)(rec + o + 8 * q) = v;
#endif
            }
        };
        auto round = [&](uint32_t r, uint4& bf) {
            const uint32_t cb = L::cnt + 4 * L::nent * (r % 3);
            const uint32_t cz = L::cnt + 4 * L::nent * ((r + 1) % 3);
            const uint32_t cbr = cb | repo;   // rank address of s: cbr | ent_b(s)
            for (uint32_t e = tid; e < L::nent; e += L::block) lds_st(cz + 4 * e, 0u);
            uint32_t s[16], rk[16];
            const bool have = r < nch;
            bool dense = false;   // wave-uniform: windows 0..14 of every lane are valid (fast case)
            if (have) {
                Windows w;
                const bool msk = rg.masked(A, rel);
                if (!msk && fast_windows<K>(bf, carry, w)) {
                    // every lane's 16 bytes are bases with at most one newline and
                    // the carry is complete: windows 0..14 valid, 15 unless a
                    // newline; ranks without per-record branches
                    dense = true;
                    carry = w.next;
                    canon_std<K, true>(w, s);
#pragma unroll
                    for (int j = 0; j < 15; ++j) rk[j] = lds_add_rtn(cbr | ent_b(s[j]), 1u);
                    if (s[15] != 0xFFFFFFFFu) rk[15] = lds_add_rtn(cbr | ent_b(s[15]), 1u);
                } else {
                    uint32_t C, V, EN, ne, own;
                    if (msk) {
                        front_end<K, true, false>(bf, A, rg.c0 + rel, lane, rg.mask(), rg.iv, C, V, EN, ne, own);
                        w = windows<K, true>(C, V, EN, ne, carry, lane);
                    } else {
                        front_end<K, false, false>(bf, A, rg.c0 + rel, lane, rg.mask(), rg.iv, C, V, EN, ne, own);
                        w = windows<K, false>(C, V, EN, ne, carry, lane);
                    }
                    carry = w.next;
                    canon_std<K>(w, s);
#pragma unroll
                    for (int j = 0; j < 16; ++j)
                        if (s[j] != 0xFFFFFFFFu) rk[j] = lds_add_rtn(cbr | ent_b(s[j]), 1u);
                }
                rel += kChunk;
                if (rel + 3 * kChunk < nch * kChunk) bf = rg.load(A.bytes, rel + 3 * kChunk, lane);
            }
            if (B.prof) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const uint64_t t = __builtin_amdgcn_s_memtime();
                lds_barrier();
                p1w += __builtin_amdgcn_s_memtime() - t;
            } else {
                lds_barrier();
            }
            if (r > 0) copy_out(r - 1, t_prev, off_prev);
            // rank-entry offsets of round r, per wave (no serial scan, no second
            // barrier): entry e = b R + replica, bucket major, lane L holds entries
            // EPL L .. EPL L + EPL - 1.  A bucket's run is its replicas' records end
            // to end, padded to whole 8-record units.
            constexpr uint32_t NR = L::nrep, EPL = L::epl;
            constexpr uint32_t BPL = NR >= EPL ? 1u : EPL / NR;   // buckets described by this lane
            uint32_t c[EPL];
            lds_ldn<EPL>(cb + 4 * EPL * lane, c);
            uint32_t o[EPL];               // offsets of the lane's entries
            uint32_t T;                    // padded records of the round
            uint32_t bst[BPL], bcnt[BPL];  // run start and record count of the lane's buckets
            bool bown = true;              // this lane describes them (meta, sentinels)
            if constexpr (NR >= EPL) {
                // a bucket spans G lanes: segmented scan, then the padded runs
                // ended by each bucket's last lane
                constexpr int G = (int)(NR / EPL);
                uint32_t lp = 0;
#pragma unroll
                for (int j = 0; j < (int)EPL; ++j) {
                    o[j] = lp;
                    lp += c[j];
                }
                const uint32_t inc = wave_incl_scan(lp), exc = inc - lp;
                const int first = lane & ~(G - 1), last = first + G - 1;
                const uint32_t seg0 = (uint32_t)__shfl((int)exc, first, kWave);
                const uint32_t tot = (uint32_t)__shfl((int)inc, last, kWave) - seg0;
                const uint32_t pad = lane == last ? (tot + 7u) & ~7u : 0u;
                const uint32_t binc = wave_incl_scan(pad);
                const uint32_t base = binc - pad;   // padded runs of the buckets before
                const uint32_t add = base + (exc - seg0);
#pragma unroll
                for (int j = 0; j < (int)EPL; ++j) o[j] += add;
                T = (uint32_t)__builtin_amdgcn_readlane((int)binc, kWave - 1);
                bst[0] = base;
                bcnt[0] = tot;
                bown = lane == first;
            } else {
                // BPL whole buckets of NR entries per lane
                uint32_t tot[BPL], lsum = 0;
#pragma unroll
                for (uint32_t q = 0; q < BPL; ++q) {
                    tot[q] = 0;
#pragma unroll
                    for (uint32_t t = 0; t < NR; ++t) tot[q] += c[q * NR + t];
                    lsum += (tot[q] + 7u) & ~7u;
                }
                const uint32_t inc = wave_incl_scan(lsum);
                uint32_t base = inc - lsum;
                T = (uint32_t)__builtin_amdgcn_readlane((int)inc, kWave - 1);
#pragma unroll
                for (uint32_t q = 0; q < BPL; ++q) {
                    bst[q] = base;
                    bcnt[q] = tot[q];
                    uint32_t x = base;
#pragma unroll
                    for (uint32_t t = 0; t < NR; ++t) {
                        o[q * NR + t] = x;
                        x += c[q * NR + t];
                    }
                    base += (tot[q] + 7u) & ~7u;
                }
            }
            lds_stn<EPL>(rb + 4 * EPL * lane, o);
            // bucket of the lane's q-th described run
            auto bid = [&](uint32_t q) -> uint32_t {
                if constexpr (NR >= EPL) return (uint32_t)lane / (NR / EPL);
                else return (uint32_t)lane * BPL + q;
            };
            if (wave == 0 && bown) {
#pragma unroll
                for (uint32_t q = 0; q < BPL; ++q) meta[(uint64_t)bid(q) * L::rmax + r] = (uint16_t)bst[q];
            }
            if (wave == 0 && lane == kWave - 1) {
                meta[(uint64_t)NBK * L::rmax + r] = (uint16_t)T;
                roff[r] = off;
            }
            const uint32_t st = L::stage + (r & 1) * L::stage_bytes;
            // sentinels after each run, up to its unit boundary (one wave per
            // round, rotating)
            if ((r % W) == (uint32_t)wave && bown) {
#pragma unroll
                for (uint32_t q = 0; q < BPL; ++q) {
                    const uint32_t e = bst[q] + bcnt[q], npad = (8u - (bcnt[q] & 7u)) & 7u;
#pragma unroll
                    for (uint32_t x = 0; x < 7; ++x)
                        if (x < npad)
                            *(volatile lds_u16*)(uintptr_t)(st + 2 * stage_slot(e + x)) =
                                (uint16_t)((((bid(q) ^ 1u) & L::hmask) << L::bits) | ((e + x) & 63u));
                }
            }
            // Staging: every table read is issued before the first record write
            // (a read after a write would wait for the write's round trip: the
            // accesses are volatile, so the compiler keeps their order).
            const uint32_t rbr = rb + repo;
            if (dense) {
#pragma unroll
                for (int j = 0; j < 15; ++j) rk[j] += lds_ld(rbr + ent_b(s[j]));
                if (s[15] != 0xFFFFFFFFu) rk[15] += lds_ld(rbr + ent_b(s[15]));
#pragma unroll
                for (int j = 0; j < 15; ++j) {
                    *(volatile lds_u16*)(uintptr_t)(st + 2 * stage_slot(rk[j])) = (uint16_t)s[j];
                }
                if (s[15] != 0xFFFFFFFFu)
                    *(volatile lds_u16*)(uintptr_t)(st + 2 * stage_slot(rk[15])) = (uint16_t)s[15];
            } else if (have) {
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (s[j] != 0xFFFFFFFFu) rk[j] += lds_ld(rbr + ent_b(s[j]));
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (s[j] != 0xFFFFFFFFu)
                        *(volatile lds_u16*)(uintptr_t)(st + 2 * stage_slot(rk[j])) = (uint16_t)s[j];
            }
            t_prev = T;
            off_prev = off;
            off += T;
        };
        uint32_t r = 0;
        for (; r + 4 <= nround; r += 4) {
            round(r, buf[0]);
            round(r + 1, buf[1]);
            round(r + 2, buf[2]);
            round(r + 3, buf[3]);
        }
        if (r < nround) round(r++, buf[0]);
        if (r < nround) round(r++, buf[1]);
        if (r < nround) round(r++, buf[2]);
        lds_barrier();
        if (nround > 0) copy_out(nround - 1, t_prev, off_prev);
        if (B.prof && tid == 0) B.prof[8 * blockIdx.x] += __builtin_amdgcn_s_memtime() - t_p1;
        if (B.prof && lane == 0) B.prof[8 * gridDim.x + 4 * (W * blockIdx.x + wave) + 2] += p1w;
      }
      if (it >= lag) {
        const uint32_t slot = kLagK ? ((it - lag) & 1u) : 0u;
        uint16_t* rec = rec_slot(B, (uint64_t)blockIdx.x * kBkSlots + slot, L::rec_cap);
        uint16_t* meta = B.meta + ((uint64_t)blockIdx.x * kBkSlots + slot) * (NBK + 1) * L::rmax;
        uint32_t* roff = B.roff + ((uint64_t)blockIdx.x * kBkSlots + slot) * L::rmax;
        const Piece P = piece_at(blockIdx.x + (it - lag) * gridDim.x);
        const int32_t g = P.g;
        const uint32_t np = P.np, nround = P.nround;

        // ---------------------------------------------------------- phase 2
        // records and meta were stored by other waves of this workgroup: wait for
        // the stores, and read them with L1-bypassing loads below
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (KF_BK_PRIO) bk_setprio((KF_BK_PRIO & 2) ? (uint32_t)wave >> 2 : 0u);
        const uint64_t t_p2 = B.prof ? __builtin_amdgcn_s_memtime() : 0;
        for (uint32_t i = tid; i < L::dirty / 4; i += L::block) lds_st(L::hist + 4 * i, 0u);   // phase-1 area
        lds_barrier();
        uint32_t* row = A.counts + (uint64_t)g * A.nbins;
        const bool split = np > 1;
        unsigned long long tsum = 0;
        // Run table of this wave: run j (< nrun) <-> round wave + W j, held by lane
        // j mod 64 in half j / 64 (W = 8 needs up to 128 runs).  A run is the whole
        // units of one bucket in one round (padded by phase 1), and the units of
        // all the wave's runs are laid end to end (prefix P over the runs), so
        // every load instruction carries 64 units whatever the run lengths.  A
        // group is kGW windows of 64 units; the next bucket's first group is
        // issued before this bucket's flush, so its loads are in flight during the
        // flush.  Loads are unconditional (inactive lanes read unit 0) so vmcnt
        // stays exact.
        constexpr int H = L::halves;
        bool myr_ok[H];
        uint32_t myr_c[H], ro[H];
        uint32_t nrun = 0;
        constexpr bool kRw = KF_BK_RW != 0 && W == 16;
        uint32_t rw0 = 0, rw1 = 0;   // kRw: this wave's rounds [rw0, rw1)
        if constexpr (kRw) {
            constexpr uint32_t wts = (uint32_t)KF_BK_RW;
            constexpr uint32_t w0 = wts & 0xFFu, w1 = (wts >> 8) & 0xFFu, w2 = (wts >> 16) & 0xFFu, w3 = wts >> 24;
            constexpr uint32_t m01 = w0 > w1 ? w0 : w1, m23 = w2 > w3 ? w2 : w3, mx = m01 > m23 ? m01 : m23;
            constexpr uint32_t tot = 4u * (w0 + w1 + w2 + w3);
            static_assert((uint64_t)L::rmax * mx <= (uint64_t)tot * 64u * H - tot, "a wave's rounds must fit its run table");
            rw0 = (nround * wave_frac((uint32_t)wave, wts)) >> 20;
            rw1 = (nround * wave_frac((uint32_t)wave + 1, wts)) >> 20;
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const uint32_t myr = kRw ? rw0 + 64u * h + (uint32_t)lane : (uint32_t)wave + (uint32_t)W * (64u * h + (uint32_t)lane);
            myr_ok[h] = kRw ? myr < rw1 : myr < nround;
            myr_c[h] = myr_ok[h] ? myr : 0u;
            nrun += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(myr_ok[h]));
            const uint32_t ro_l = __builtin_nontemporal_load(roff + myr_c[h]);
            ro[h] = myr_ok[h] ? ro_l : 0u;
        }
        struct Hv {
            uint32_t v[H];
        };
        // raw (lanes without a run read round 0; make_tbl masks them), so that
        // the load is not waited for until its table is built
        auto meta_at = [&](uint32_t b) -> Hv {
            Hv m;
#pragma unroll
            for (int h = 0; h < H; ++h) m.v[h] = __builtin_nontemporal_load(meta + (uint64_t)b * L::rmax + myr_c[h]);
            return m;
        };
        struct Tbl {
            uint32_t P[H], DL[H];    // per run: first unit in the bucket's unit space, unit delta
            uint32_t U, jn, cur, w0; // wave-uniform
        };
        auto make_tbl = [&](const Hv& rs, const Hv& re) {
            Tbl t;
            uint32_t tot = 0;
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const uint32_t n = myr_ok[h] ? (re.v[h] - rs.v[h]) >> 3 : 0u;   // rs, re: 8-aligned
                const uint32_t inc = wave_incl_scan(n) + tot;
                t.P[h] = inc - n;
                tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, kWave - 1);
                t.DL[h] = ((ro[h] + rs.v[h]) >> 3) - t.P[h];   // unit u of the bucket is record unit u + DL
            }
            t.U = tot;
            t.jn = 0;
            t.cur = 0;
            t.w0 = 0;
            return t;
        };
        // run j's entry of a per-run table (wave-uniform j)
        auto run_at = [&](const uint32_t (&x)[H], uint32_t j) -> uint32_t {
            if (H == 1 || j < 64u) return (uint32_t)__builtin_amdgcn_readlane((int)x[0], (int)j);
            return (uint32_t)__builtin_amdgcn_readlane((int)x[H - 1], (int)(j - 64u));
        };
        constexpr int kGW = KF_BK_DB ? 4 : 8;
        constexpr bool kPre2 = KF_BK_PRE2 && K <= KF_BK_PRE2_MAXK;
        struct Grp {
            v4u v[kGW];
            uint32_t act;   // bit x: this lane's unit of window x exists
            uint32_t w0;    // first unit of the group
        };
        // next kGW windows of 64 units of table t -> loads in flight
        auto issue = [&](Tbl& t, Grp& G) {
            G.act = 0;
            G.w0 = t.w0;
#pragma unroll
            for (int x = 0; x < kGW; ++x) {
                const uint32_t w0 = t.w0 + x * kWave, u = w0 + (uint32_t)lane;
                uint32_t dl = t.cur;
                while (t.jn < nrun) {   // runs starting in this window
                    const uint32_t pj = run_at(t.P, t.jn);
                    if (pj >= w0 + kWave) break;
                    const uint32_t dj = run_at(t.DL, t.jn);
                    dl = u >= pj ? dj : dl;
                    t.cur = dj;
                    ++t.jn;
                }
                const bool a = u < t.U;
                G.act |= a ? 1u << x : 0u;
                const uint32_t q = a ? 8 * (u + dl) : 0u;
                G.v[x] = __builtin_nontemporal_load((const v4u*)(rec + q));
            }
            t.w0 += kGW * kWave;
        };
        auto consume = [&](const Grp& G, uint32_t U, uint32_t pm) {   // pm: bucket parity mask
#pragma unroll
            for (int x = 0; x < kGW; ++x) {
                if (G.w0 + x * kWave >= U) break;   // wave-uniform
                if (G.act & (1u << x)) {
                    const uint32_t d[4] = {G.v[x].x ^ pm, G.v[x].y ^ pm, G.v[x].z ^ pm, G.v[x].w ^ pm};
#pragma unroll
                    for (int t = 0; t < 8; ++t) lds_add(rec_addr(d[t >> 1], t & 1), 1u);
                }
            }
        };
        // The flush handles 4 consecutive columns per lane, lanes consecutive: one
        // 8-byte col_idx load and one 16-byte count store per lane (coalesced
        // rows; consecutive columns also spread the LDS reads over the banks).
        // col_idx of up to kFG groups per lane (32768 columns: any bucket) is
        // loaded before the barrier.
        constexpr int kFG = 8;
        typedef unsigned int v2u __attribute__((ext_vector_type(2)));
        auto col_at = [&](uint32_t g4) -> v2u {
            return *(const v2u*)(B.col_idx + g4);
        };
        // c0, c1: the bucket's column range, loaded here (before the next bucket's
        // record loads) so the flush does not wait on those.
        auto flush_issue = [&](uint32_t b, v2u (&ci)[kFG], uint32_t& c0, uint32_t& c1) {
            typedef __attribute__((address_space(4))) const uint32_t const_u32;   // scalar loads (lgkmcnt)
            const const_u32* bc = (const const_u32*)(uintptr_t)B.bcol;
            c0 = bc[b];
            c1 = bc[b + 1];
#pragma unroll
            for (int x = 0; x < kFG; ++x) {
                const uint32_t g4 = (c0 & ~3u) + 4 * ((uint32_t)tid + x * L::block);
                const v2u c = col_at(g4 < c1 ? g4 : 0u);   // unconditional load
                ci[x] = g4 < c1 ? c : v2u{0u, 0u};
            }
        };
        auto flush_cols = [&](uint32_t g4, const v2u ci, uint32_t c0, uint32_t c1) {
            if (g4 >= c1) return;
            uint32_t v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t col = g4 + t;
                v[t] = (col >= c0 && col < c1) ? lds_xchg(((ci[t >> 1] >> (16 * (t & 1))) & 0xFFFFu) << 2, 0u) : 0u;
                tsum += v[t];
            }
            if (!split && !B.accumulate && g4 >= c0 && g4 + 4 <= c1) {
#if KF_NT_STORES
                __builtin_nontemporal_store(v4u{v[0], v[1], v[2], v[3]}, (v4u*)(row + g4));
#else
                *(v4u*)(row + g4) = v4u{v[0], v[1], v[2], v[3]};
#endif
                return;
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t col = g4 + t;
                if (col < c0 || col >= c1) continue;
                if (split) {
                    if (v[t]) __hip_atomic_fetch_add(row + col, v[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else if (B.accumulate) {
                    row[col] += v[t];
                } else {
                    row[col] = v[t];
                }
            }
        };

        Hv re_next = meta_at(1);
        Tbl tb = make_tbl(meta_at(0), re_next);
        Hv re_cur = re_next;
        re_next = meta_at(NBK > 1 ? 2 : 1);
        Grp G0;
#if KF_BK_DB
        Grp G1;
#endif
        issue(tb, G0);
#if KF_BK_DB
        if constexpr (kPre2) issue(tb, G1);
#endif
        uint64_t tp[4] = {0, 0, 0, 0};   // profile: records, barrier, flush, barrier
        uint64_t tcons = 0;              // profile: consume part of records
        for (uint32_t b = 0; b < NBK; ++b) {
            uint64_t t0 = B.prof ? __builtin_amdgcn_s_memtime() : 0;
            const uint32_t pm = ((b & L::hmask) << L::bits) * 0x10001u;   // both records of a word
#if KF_BK_DB
            // two groups alternate: the bucket's next group is always in flight
            // while one is counted (issued unconditionally -- past the bucket's
            // end its lanes are inactive and read unit 0 -- so the compiler's
            // vmcnt stays exact: wait for the consumed group only)
            if constexpr (kPre2) {
                // both groups were issued before the previous flush
                for (;;) {
                    consume(G0, tb.U, pm);
                    if (G1.w0 >= tb.U) break;
                    issue(tb, G0);
                    consume(G1, tb.U, pm);
                    if (G0.w0 >= tb.U) break;
                    issue(tb, G1);
                }
            } else {
                for (;;) {
                    issue(tb, G1);
                    consume(G0, tb.U, pm);
                    if (G1.w0 >= tb.U) break;
                    issue(tb, G0);
                    consume(G1, tb.U, pm);
                    if (G0.w0 >= tb.U) break;
                }
            }
#else
            consume(G0, tb.U, pm);
            while (tb.w0 < tb.U) {   // a bucket beyond one group: synchronous groups
                issue(tb, G0);
                consume(G0, tb.U, pm);
            }
#endif
            if (B.prof) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); tcons += __builtin_amdgcn_s_memtime() - t0; }
            v2u ci[kFG];
            // issue order: bucket b+2's run ends, the flush's col_idx, bucket
            // b+1's records (vmcnt is in order: each is waited for only when used)
            const Hv m = meta_at(b + 3 < NBK ? b + 3 : NBK);
            uint32_t c0, c1;
            flush_issue(b, ci, c0, c1);
            if (b + 1 < NBK) {               // next bucket: table, first group in flight
                tb = make_tbl(re_cur, re_next);   // this bucket's run ends start the next
                re_cur = re_next;
                issue(tb, G0);
#if KF_BK_DB
                if constexpr (kPre2) issue(tb, G1);
#endif
            }
            re_next = m;
            if (B.prof) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const uint64_t t = __builtin_amdgcn_s_memtime(); tp[0] += t - t0; t0 = t; }
            lds_barrier();
            if (B.prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); tp[1] += t - t0; t0 = t; }
#pragma unroll
            for (int x = 0; x < kFG; ++x) flush_cols((c0 & ~3u) + 4 * ((uint32_t)tid + x * L::block), ci[x], c0, c1);
            for (uint32_t g4 = (c0 & ~3u) + 4 * ((uint32_t)tid + kFG * L::block); g4 < c1; g4 += 4 * L::block)
                flush_cols(g4, col_at(g4), c0, c1);
            if (B.prof) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const uint64_t t = __builtin_amdgcn_s_memtime(); tp[2] += t - t0; t0 = t; }
            lds_barrier();
            if (B.prof) { const uint64_t t = __builtin_amdgcn_s_memtime(); tp[3] += t - t0; }
        }
        if (B.prof && lane == 0) {   // per wave: records, barrier, (phase-1 barrier), consume
            unsigned long long* pw = B.prof + 8 * gridDim.x + 4 * (W * blockIdx.x + wave);
            pw[0] += tp[0];
            pw[1] += tp[1];
            pw[3] += tcons;
        }
        tsum = wave_sum(tsum);
        unsigned long long* red = (unsigned long long*)((char*)lds + L::red);
        if (lane == 0) red[wave] = tsum;
        __syncthreads();
        if (tid == 0) {
            unsigned long long t = 0;
            for (int w = 0; w < W; ++w) t += red[w];
            if (t) atomicAdd(A.totals + g, t);
            if (B.prof) {
                const uint64_t t_end = __builtin_amdgcn_s_memtime();
                B.prof[8 * blockIdx.x + 1] += t_end - t_p2;
                B.prof[8 * blockIdx.x + 2] += 1;
                for (int x = 0; x < 4; ++x) B.prof[8 * blockIdx.x + 3 + x] += tp[x];
            }
        }
        __syncthreads();
      }
    }
}

}  // namespace kf

// ====================================================================== host
using namespace kf;

namespace {

template <int K>
void* bucket_ptr() { return (void*)&bucket_kernel<K>; }

void* bucket_kernel_for(int k) {
    switch (k) {
    case 9: return bucket_ptr<9>();
    case 10: return bucket_ptr<10>();
    case 11: return bucket_ptr<11>();
    case 12: return bucket_ptr<12>();
    default: return nullptr;
    }
}
template <typename F>
auto bucket_geom(int k, F f) {   // f(Bk<k>{}) for the compiled k
    switch (k) {
    case 9: return f(Bk<9>{});
    case 10: return f(Bk<10>{});
    case 11: return f(Bk<11>{});
    default: return f(Bk<12>{});
    }
}
uint32_t bucket_lds_for(int k) {
    return bucket_geom(k, [](auto b) { return decltype(b)::lds_bytes; });
}
int bucket_waves_for(int k) {
    return bucket_geom(k, [](auto b) { return decltype(b)::waves; });
}
int bucket_bits_for(int k) {
    return bucket_geom(k, [](auto b) { return decltype(b)::bits; });
}

// Per-device state: bucket tables per k and the scratch of the last launch
// size.  A launch on another stream waits for the previous user of the scratch.
struct DevState {
    uint16_t* col_idx[KF_MAX_K + 1] = {};
    uint32_t* bcol[KF_MAX_K + 1] = {};
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    uint32_t* pstart = nullptr;
    size_t pstart_n = 0;
    hipEvent_t done = nullptr;
    int cus = 0;
};
DevState g_dev[64];
std::mutex g_mu;

uint32_t rc_std(uint32_t s, int k) {
    uint32_t r = 0;
    for (int i = 0; i < k; ++i) {
        r = (r << 2) | (3u - (s & 3u));
        s >>= 2;
    }
    return r;
}

int ensure_tables(DevState& d, int k) {
    if (d.col_idx[k]) return KF_OK;
    const int bits = bucket_bits_for(k);
    const uint32_t codes = 1u << bits;
    const uint32_t ncode = 1u << (2 * k), nbk = ncode >> bits;
    std::vector<uint16_t> ci;
    std::vector<uint32_t> bc(nbk + 1, 0);
    ci.reserve(kf_num_bins(k));
    for (uint32_t s = 0; s < ncode; ++s) {
        if ((s & (codes - 1)) == 0) bc[s >> bits] = (uint32_t)ci.size();
        if (s <= rc_std(s, k)) ci.push_back((uint16_t)(s & (codes - 1)));
    }
    bc[nbk] = (uint32_t)ci.size();
    if (ci.size() != kf_num_bins(k)) return kf_fail(KF_EINVAL, "bucket table: %zu canonical codes", ci.size());
    if (hipMalloc((void**)&d.col_idx[k], ci.size() * 2) != hipSuccess ||
        hipMalloc((void**)&d.bcol[k], bc.size() * 4) != hipSuccess)
        return kf_fail(KF_EHIP, "hipMalloc of bucket tables failed");
    if (hipMemcpy(d.col_idx[k], ci.data(), ci.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d.bcol[k], bc.data(), bc.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return kf_fail(KF_EHIP, "hipMemcpy of bucket tables failed");
    return KF_OK;
}

// Scratch of one device: records, round metadata, round offsets, sized for the
// largest of the compiled geometries (so a launch at another k reuses it).
// Record slot skew in records (profiling builds: KF_BUCKET_SKEW, bytes).
uint32_t rec_skew() {
#ifdef KF_PROFILE_BUILD
    const char* e = getenv("KF_BUCKET_SKEW");
    return e ? (uint32_t)(strtoul(e, nullptr, 0) / 2) : 0u;
#else
    return 0u;
#endif
}
void scratch_layout(int cus, size_t& rec_b, size_t& meta_b, size_t& roff_b) {
    rec_b = meta_b = roff_b = 0;
    for (int kk = 9; kk <= KF_MAX_K; ++kk) {   // the bucket kernels: k >= 9
        const size_t g = (size_t)cus * (16 / bucket_waves_for(kk)) * kBkSlots;
        bucket_geom(kk, [&](auto b) {
            using Lk = decltype(b);
            rec_b = std::max(rec_b, g * (size_t)Lk::rec_cap * 2 + (size_t)128 * rec_skew());
            meta_b = std::max(meta_b, g * ((size_t)Lk::nbk + 1) * Lk::rmax * 2);
            roff_b = std::max(roff_b, g * (size_t)Lk::rmax * 4);
            return 0;
        });
    }
}

}  // namespace

namespace kf {

int bucket_launch_info(int k, int* grid, int* block, int* lds) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return kf_fail(KF_EHIP, "device query failed");
    *grid = (cus > 0 ? cus : 1) * (16 / bucket_waves_for(k));
    *block = bucket_waves_for(k) * kWave;
    *lds = (int)bucket_lds_for(k);
    return KF_OK;
}

// Everything a launch at k over n_genomes needs on device `dev` (caller holds
// g_mu): the bucket tables of k, the kernel's LDS attribute, the scratch (sized
// for the largest compiled geometry, so every k shares it) and a piece table of
// at least n_genomes+1 words (grown 2x at a time; a regrowth synchronises the
// device, since a launch in flight may still read the old one).
int ensure_scratch(DevState& d, int dev, size_t need);

int ensure_workspace(DevState& d, int dev, int k, int32_t n_genomes) {
    void* fn = bucket_kernel_for(k);
    if (!fn) return kf_fail(KF_EINVAL, "no bucket kernel for k=%d", k);
    const uint32_t lds = bucket_lds_for(k);
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return kf_fail(KF_EHIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    int rc0 = ensure_scratch(d, dev, 0);   // the device state
    if (rc0) return rc0;
    size_t rec_b = 0, meta_b = 0, roff_b = 0;
    scratch_layout(d.cus, rec_b, meta_b, roff_b);
    const size_t need = rec_b + meta_b + roff_b;
#ifdef KF_PROFILE_BUILD
    if (getenv("KF_BUCKET_TABLES_FIRST")) {
        const int rc = ensure_tables(d, k);
        if (rc) return rc;
    }
#endif
    rc0 = ensure_scratch(d, dev, need);
    if (rc0) return rc0;
    // the tables after the scratch (KF_BUCKET_TABLES_FIRST=1, profiling builds:
    // before it, the order of rounds 2-4)
#ifdef KF_PROFILE_BUILD
    const bool tables_first = getenv("KF_BUCKET_TABLES_FIRST") != nullptr;
#else
    const bool tables_first = false;
#endif
    if (!tables_first) {
        const int rc = ensure_tables(d, k);
        if (rc) return rc;
    }
#ifdef KF_PROFILE_BUILD
    if (getenv("KF_BUCKET_DEBUG"))   // profiling builds: where the scratch and tables landed
        fprintf(stderr, "[kf_bucket] scratch %p (%zu B) col_idx %p bcol %p\n", d.scratch, d.scratch_bytes,
                (void*)d.col_idx[k], (void*)d.bcol[k]);
#endif
    if (d.pstart_n < (size_t)n_genomes + 1) {
        const size_t cap = std::max((size_t)n_genomes + 1, 2 * d.pstart_n);
        if (d.pstart && (hipDeviceSynchronize() != hipSuccess || hipFree(d.pstart) != hipSuccess))
            return kf_fail(KF_EHIP, "hipFree of piece table failed");
        d.pstart = nullptr;
        d.pstart_n = 0;
        if (hipMalloc((void**)&d.pstart, cap * 4) != hipSuccess)
            return kf_fail(KF_EHIP, "hipMalloc of piece table failed");
        d.pstart_n = cap;
    }
    return KF_OK;
}

// The device state (CU count, the scratch's event) and a scratch of at least
// `need` bytes (caller holds g_mu).
int ensure_scratch(DevState& d, int dev, size_t need) {
    if (!d.cus) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return kf_fail(KF_EHIP, "hipDeviceGetAttribute(MultiprocessorCount) failed");
        d.cus = cus > 0 ? cus : 1;
        if (hipEventCreateWithFlags(&d.done, hipEventDisableTiming) != hipSuccess)
            return kf_fail(KF_EHIP, "hipEventCreate failed");
    }
    if (d.scratch_bytes < need) {
        if (d.scratch && (hipDeviceSynchronize() != hipSuccess || hipFree(d.scratch) != hipSuccess))
            return kf_fail(KF_EHIP, "hipFree of bucket scratch failed");
        d.scratch = nullptr;
        d.scratch_bytes = 0;
#ifdef KF_PROFILE_BUILD
        // profiling builds: KF_BUCKET_CONTIG=1 asks for physically contiguous scratch
        if (!(getenv("KF_BUCKET_CONTIG") && hipExtMallocWithFlags(&d.scratch, need, hipDeviceMallocContiguous) == hipSuccess))
#endif
        if (hipMalloc(&d.scratch, need) != hipSuccess)
            return kf_fail(KF_EHIP, "hipMalloc of %zu bytes of bucket scratch failed", need);
        d.scratch_bytes = need;
    }
    return KF_OK;
}

int bucket_reserve(int k, int32_t max_genomes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kf_fail(KF_EHIP, "hipGetDevice failed");
    if (dev < 0 || dev >= 64) return kf_fail(KF_EINVAL, "device index out of range");
    std::lock_guard<std::mutex> lk(g_mu);
    return ensure_workspace(g_dev[dev], dev, k, max_genomes);
}

int bucket_launch(const CountArgs& A, int k, uint32_t flags, hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kf_fail(KF_EHIP, "hipGetDevice failed");
    if (dev < 0 || dev >= 64) return kf_fail(KF_EINVAL, "device index out of range");
    void* fn = bucket_kernel_for(k);
    if (!fn) return kf_fail(KF_EINVAL, "no bucket kernel for k=%d", k);
    std::lock_guard<std::mutex> lk(g_mu);
    DevState& d = g_dev[dev];
    int rc = ensure_workspace(d, dev, k, A.n_genomes);
    if (rc) return rc;
    const uint32_t lds = bucket_lds_for(k);
    const int waves = bucket_waves_for(k);
    const int grid = d.cus * (16 / waves);   // 16 waves per CU
    size_t rec_b = 0, meta_b = 0, roff_b = 0;
    scratch_layout(d.cus, rec_b, meta_b, roff_b);
    if (d.done && hipStreamWaitEvent(s, d.done, 0) != hipSuccess)
        return kf_fail(KF_EHIP, "hipStreamWaitEvent failed");
    BucketArgs B;
    B.col_idx = d.col_idx[k];
    B.bcol = d.bcol[k];
    B.pstart = d.pstart;
    B.rec = (uint16_t*)d.scratch;
    B.meta = (uint16_t*)((char*)d.scratch + rec_b);
    B.roff = (uint32_t*)((char*)d.scratch + rec_b + meta_b);
    B.accumulate = (flags & KF_ACCUMULATE) ? 1u : 0u;
    B.skew = rec_skew();
    B.prof = nullptr;
#ifdef KF_PROFILE_BUILD
    const char* pe = getenv("KF_BUCKET_PROFILE");   // debugging aid: synchronous, prints to stderr
#else
    const char* pe = nullptr;   // (kf_count_batch stays asynchronous and allocation-free per launch)
#endif
    std::vector<unsigned long long> prof_h;
    if (pe && *pe == '1') {
        if (hipMalloc((void**)&B.prof, (size_t)grid * (8 + 4 * waves) * 8) != hipSuccess ||
            hipMemsetAsync(B.prof, 0, (size_t)grid * (8 + 4 * waves) * 8, s) != hipSuccess)
            return kf_fail(KF_EHIP, "profile buffer");
    }
    hipLaunchKernelGGL(piece_scan_kernel, dim3(1), dim3(1024), 0, s, A.goff, A.n_genomes, d.pstart);
    if (!B.accumulate)
        hipLaunchKernelGGL(zero_split_rows_kernel, dim3(1024), dim3(256), 0, s, A.goff, A.n_genomes, A.counts,
                           A.nbins);
    void* args[] = {(void*)&A, (void*)&B};
    if (hipLaunchKernel(fn, dim3(grid), dim3(waves * kWave), args, lds, s) != hipSuccess)
        return kf_fail(KF_EHIP, "bucket kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (hipEventRecord(d.done, s) != hipSuccess) return kf_fail(KF_EHIP, "hipEventRecord failed");
    if (B.prof) {
        prof_h.resize((size_t)grid * (8 + 4 * waves));
        if (hipStreamSynchronize(s) != hipSuccess ||
            hipMemcpy(prof_h.data(), B.prof, prof_h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
            return kf_fail(KF_EHIP, "profile readback");
        (void)hipFree(B.prof);
        double sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < grid; ++i)
            for (int x = 0; x < 8; ++x) sum[x] += (double)prof_h[8 * i + x];
        const double np = sum[2] > 0 ? sum[2] : 1;
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)fn, waves * kWave, lds);
        fprintf(stderr, "[kf_bucket k=%d] grid %d x %d waves, LDS %u B, resident workgroups per CU %d\n", k, grid,
                waves, lds, occ);
        fprintf(stderr, "[kf_bucket k=%d] pieces %.0f cycles/piece: phase1 %.3g phase2 %.3g "
                "(records %.3g, barrier %.3g, flush %.3g, barrier %.3g)\n",
                k, sum[2], sum[0] / np, sum[1] / np, sum[3] / np, sum[4] / np, sum[5] / np, sum[6] / np);
        fprintf(stderr, "[kf_bucket k=%d] per wave, cycles per piece:", k);
        for (int w = 0; w < waves; ++w) {
            double v[4] = {0, 0, 0, 0};
            for (int i = 0; i < grid; ++i)
                for (int x = 0; x < 4; ++x) v[x] += (double)prof_h[8 * grid + 4 * (waves * i + w) + x];
            fprintf(stderr, "\n  w%d records %.3g (consume %.3g) barrier %.3g | phase-1 barrier %.3g", w, v[0] / np,
                    v[3] / np, v[1] / np, v[2] / np);
        }
        fprintf(stderr, "\n");
    }
    return KF_OK;
}

}  // namespace kf

extern "C" int kf_workspace_release(void) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kf_fail(KF_EHIP, "hipGetDevice failed");
    if (dev < 0 || dev >= 64) return kf_fail(KF_EINVAL, "device index out of range");
    std::lock_guard<std::mutex> lk(g_mu);
    DevState& d = g_dev[dev];
    if (hipDeviceSynchronize() != hipSuccess) return kf_fail(KF_EHIP, "hipDeviceSynchronize failed");
    for (int k = 0; k <= KF_MAX_K; ++k) {
        if (d.col_idx[k]) (void)hipFree(d.col_idx[k]);
        if (d.bcol[k]) (void)hipFree(d.bcol[k]);
        d.col_idx[k] = nullptr;
        d.bcol[k] = nullptr;
    }
    if (d.scratch) (void)hipFree(d.scratch);
    if (d.pstart) (void)hipFree(d.pstart);
    d.scratch = nullptr;
    d.scratch_bytes = 0;
    d.pstart = nullptr;
    d.pstart_n = 0;
    return KF_OK;
}
