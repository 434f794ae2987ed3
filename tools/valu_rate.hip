// VALU issue cost per wave64 instruction on gfx950, by opcode and by waves per
// SIMD: the front end of the k=7 counters is VALU-bound, so
// which opcodes cost 2 vs 4 cycles decides how the classify / window code is
// written.  Each lane runs 8 independent chains of one opcode; cycles are
// s_memtime deltas per wave (shader clock), so the result does not depend on DVFS.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_rate tools/valu_rate.hip && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// one op on each of the 8 chains; operands: %0..%7 chains, %8 = a second VGPR, %9 = SGPR constant
#define BODY(OPSTR)                                                                                   \
    asm volatile(OPSTR(0) OPSTR(1) OPSTR(2) OPSTR(3) OPSTR(4) OPSTR(5) OPSTR(6) OPSTR(7)                 \
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)    \
                 : "v"(y), "s"(sc))

#define OP_AND(i) "v_and_b32 %" #i ", %" #i ", %8\n"
#define OP_LSHR(i) "v_lshrrev_b32 %" #i ", 3, %" #i "\n"
#define OP_ADD(i) "v_add_u32 %" #i ", %" #i ", %8\n"
#define OP_PERM(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n"
#define OP_ALIGN(i) "v_alignbit_b32 %" #i ", %" #i ", %8, 5\n"
#define OP_BFE(i) "v_bfe_u32 %" #i ", %" #i ", 3, 14\n"
#define OP_DOT4(i) "v_dot4_u32_u8 %" #i ", %" #i ", %9, 0\n"
#define OP_BITOP3(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x60\n"
#define OP_LSHLOR(i) "v_lshl_or_b32 %" #i ", %" #i ", 3, %8\n"
#define OP_SDWA(i) "v_and_b32_sdwa %" #i ", %" #i ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
#define OP_DPP(i) "v_mov_b32_dpp %" #i ", %" #i " wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define OP_DPPROW(i) "v_mov_b32_dpp %" #i ", %" #i " row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define OP_BCNT(i) "v_bcnt_u32_b32 %" #i ", %" #i ", %8\n"
#define OP_BFI(i) "v_bfi_b32 %" #i ", %" #i ", %8, %9\n"
#define OP_OR3(i) "v_or3_b32 %" #i ", %" #i ", %8, %9\n"
#define OP_CNDMASK(i) "v_cndmask_b32 %" #i ", %" #i ", %8, vcc\n"
#define OP_PKADD(i) "v_pk_add_u16 %" #i ", %" #i ", %8\n"
#define OP_PKLSHR(i) "v_pk_lshrrev_b16 %" #i ", 1, %" #i "\n"
#define OP_SDWASHL(i) "v_lshlrev_b32_sdwa %" #i ", %" #i ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n"
#define OP_LSHLADD(i) "v_lshl_add_u32 %" #i ", %" #i ", 2, %8\n"
#define OP_FFBL(i) "v_ffbl_b32 %" #i ", %" #i "\n"
#define OP_MAD24(i) "v_mad_u32_u24 %" #i ", %" #i ", %8, %9\n"
#define OP_XOR(i) "v_xor_b32 %" #i ", %" #i ", %8\n"
#define OP_AND_E64S(i) "v_and_b32_e64 %" #i ", %" #i ", %9\n"
#define OP_AND_LIT(i) "v_and_b32_e32 %" #i ", 0x3030303, %" #i "\n"
#define OP_AND_SGPR(i) "v_and_b32_e32 %" #i ", %9, %" #i "\n"
#define OP_AND_INL(i) "v_and_b32_e32 %" #i ", 63, %" #i "\n"
#define OP_LSHR_V(i) "v_lshrrev_b32_e32 %" #i ", %8, %" #i "\n"
#define OP_MOV(i) "v_mov_b32_e32 %" #i ", %8\n"
#define OP_DOT4C(i) "v_dot4c_i32_i8_e32 %" #i ", %9, %8\n"
#define OP_LSHR64(i) "v_alignbyte_b32 %" #i ", %" #i ", %8, 1\n"
#define OP_MUL24(i) "v_mul_u32_u24_e32 %" #i ", %9, %" #i "\n"
#define OP_MIN(i) "v_min_u32_e32 %" #i ", %9, %" #i "\n"
#define OP_SUB(i) "v_sub_u32_e32 %" #i ", %9, %" #i "\n"
#define OP_CNDE32(i) "v_cndmask_b32_e32 %" #i ", %8, %" #i ", vcc\n"
#define OP_NOT(i) "v_not_b32_e32 %" #i ", %" #i "\n"
#define OP_BFREV(i) "v_bfrev_b32_e32 %" #i ", %" #i "\n"
#define OP_OR(i) "v_or_b32_e32 %" #i ", %9, %" #i "\n"
#define OP_DOT4CV(i) "v_dot4c_i32_i8_e32 %" #i ", %8, %" #i "\n"
#define OP_MUL24V(i) "v_mul_u32_u24_e32 %" #i ", %8, %" #i "\n"
#define OP_MULHI24V(i) "v_mul_hi_u32_u24_e32 %" #i ", %8, %" #i "\n"
#define OP_SUBV(i) "v_sub_u32_e32 %" #i ", %8, %" #i "\n"
#define OP_MINV(i) "v_min_u32_e32 %" #i ", %8, %" #i "\n"
#define OP_LSHLV(i) "v_lshlrev_b32_e32 %" #i ", %8, %" #i "\n"
#define OP_MIXFF(i) "v_and_b32_e32 %" #i ", 0x3030303, %" #i "\nv_xor_b32_e32 %" #i ", %8, %" #i "\n"
#define OP_MIX3F1S(i) "v_and_b32_e32 %" #i ", 0x3030303, %" #i "\nv_xor_b32_e32 %" #i ", %8, %" #i "\nv_lshrrev_b32_e32 %" #i ", 3, %" #i "\nv_perm_b32 %" #i ", %" #i ", %8, %9\n"
#define OP_LSHL_INL(i) "v_lshlrev_b32_e32 %" #i ", 3, %" #i "\n"
#define OP_CNDV(i) "v_cndmask_b32_e32 %" #i ", %8, %" #i ", vcc\n"
#define OP_MIX(i) "v_and_b32_e32 %" #i ", %9, %" #i "\nv_perm_b32 %" #i ", %" #i ", %8, %9\n"

template <int OP>
__device__ __forceinline__ void body(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& x4,
                                     uint32_t& x5, uint32_t& x6, uint32_t& x7, uint32_t y, uint32_t sc) {
    switch (OP) {
    case 0: BODY(OP_AND); break;
    case 1: BODY(OP_LSHR); break;
    case 2: BODY(OP_ADD); break;
    case 3: BODY(OP_PERM); break;
    case 4: BODY(OP_ALIGN); break;
    case 5: BODY(OP_BFE); break;
    case 6: BODY(OP_DOT4); break;
    case 7: BODY(OP_BITOP3); break;
    case 8: BODY(OP_LSHLOR); break;
    case 9: BODY(OP_SDWA); break;
    case 10: BODY(OP_DPP); break;
    case 11: BODY(OP_DPPROW); break;
    case 12: BODY(OP_BCNT); break;
    case 13: BODY(OP_BFI); break;
    case 14: BODY(OP_OR3); break;
    case 15: BODY(OP_CNDMASK); break;
    case 16: BODY(OP_PKADD); break;
    case 17: BODY(OP_PKLSHR); break;
    case 18: BODY(OP_SDWASHL); break;
    case 19: BODY(OP_LSHLADD); break;
    case 20: BODY(OP_FFBL); break;
    case 21: BODY(OP_MAD24); break;
    case 22: BODY(OP_XOR); break;
    case 23: BODY(OP_AND_E64S); break;
    case 24: BODY(OP_AND_LIT); break;
    case 25: BODY(OP_AND_SGPR); break;
    case 26: BODY(OP_AND_INL); break;
    case 27: BODY(OP_LSHR_V); break;
    case 28: BODY(OP_MOV); break;
    case 29: BODY(OP_DOT4C); break;
    case 30: BODY(OP_LSHR64); break;
    case 31: BODY(OP_MUL24); break;
    case 32: BODY(OP_MIN); break;
    case 33: BODY(OP_SUB); break;
    case 34: BODY(OP_CNDE32); break;
    case 35: BODY(OP_NOT); break;
    case 36: BODY(OP_BFREV); break;
    case 37: BODY(OP_OR); break;
    case 38: BODY(OP_MIX); break;
    case 39: BODY(OP_DOT4CV); break;
    case 40: BODY(OP_MUL24V); break;
    case 41: BODY(OP_MULHI24V); break;
    case 42: BODY(OP_SUBV); break;
    case 43: BODY(OP_MINV); break;
    case 44: BODY(OP_LSHLV); break;
    case 45: BODY(OP_MIXFF); break;
    case 46: BODY(OP_MIX3F1S); break;
    case 47: BODY(OP_AND_LIT); BODY(OP_PERM); break;
    case 48: BODY(OP_AND_LIT); BODY(OP_AND_LIT); BODY(OP_PERM); BODY(OP_PERM); break;
    case 49: BODY(OP_AND_LIT); BODY(OP_XOR); BODY(OP_LSHR); BODY(OP_AND_LIT); BODY(OP_PERM); BODY(OP_BITOP3); break;
    case 50: BODY(OP_LSHL_INL); break;
    }
}
static const char* kNames[] = {"v_and_b32 (VOP2)", "v_lshrrev_b32", "v_add_u32", "v_perm_b32", "v_alignbit_b32",
                               "v_bfe_u32", "v_dot4_u32_u8", "v_bitop3_b32", "v_lshl_or_b32", "v_and_b32_sdwa",
                               "v_mov_b32_dpp wave_shr", "v_mov_b32_dpp row_shr", "v_bcnt_u32_b32", "v_bfi_b32",
                               "v_or3_b32", "v_cndmask_b32", "v_pk_add_u16", "v_pk_lshrrev_b16",
                               "v_lshlrev_b32_sdwa", "v_lshl_add_u32", "v_ffbl_b32", "v_mad_u32_u24",
                               "v_xor_b32", "v_and_b32_e64 sgpr", "v_and_b32_e32 literal", "v_and_b32_e32 sgpr",
                               "v_and_b32_e32 inline", "v_lshrrev_b32_e32 vgpr", "v_mov_b32_e32",
                               "v_dot4c_i32_i8_e32", "v_alignbyte_b32", "v_mul_u32_u24_e32", "v_min_u32_e32",
                               "v_sub_u32_e32", "v_cndmask_b32_e32", "v_not_b32_e32", "v_bfrev_b32_e32",
                               "v_or_b32_e32 sgpr", "and_e32 + perm (per pair)",
                               "v_dot4c_i32_i8_e32 vgpr", "v_mul_u32_u24_e32 vgpr", "v_mul_hi_u32_u24 vgpr",
                               "v_sub_u32_e32 vgpr", "v_min_u32_e32 vgpr", "v_lshlrev_b32_e32 vgpr",
                               "and_lit + xor (per pair)", "3 fast + perm (per quad)",
                               "runs 8 and + 8 perm (per 2)", "runs 16 and + 16 perm (per 4)",
                               "runs 32 fast + 16 cplx (per 6)", "v_lshlrev_b32_e32 inline"};
constexpr int kOps = 51;
constexpr int kUnroll = 8;   // BODY calls per iteration: 64 instructions

template <int OP>
__global__ void k_valu(unsigned long long* cyc, uint32_t* sink, int iters, uint32_t seed) {
    uint32_t x0 = threadIdx.x ^ seed, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 11, x5 = x0 * 13,
             x6 = x0 * 17, x7 = x0 * 19;
    const uint32_t y = seed * 0x9E3779B9u + threadIdx.x;
    const uint32_t sc = __builtin_amdgcn_readfirstlane(seed | 0x01010101u);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_barrier" ::: "memory");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) body<OP>(x0, x1, x2, x3, x4, x5, x6, x7, y, sc);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
    if ((x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) == 0x12345678u) sink[0] = 1;
}

typedef void (*KFn)(unsigned long long*, uint32_t*, int, uint32_t);

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    KFn fns[kOps] = {k_valu<0>,  k_valu<1>,  k_valu<2>,  k_valu<3>,  k_valu<4>,  k_valu<5>,
                     k_valu<6>,  k_valu<7>,  k_valu<8>,  k_valu<9>,  k_valu<10>, k_valu<11>,
                     k_valu<12>, k_valu<13>, k_valu<14>, k_valu<15>, k_valu<16>, k_valu<17>,
                     k_valu<18>, k_valu<19>, k_valu<20>, k_valu<21>, k_valu<22>, k_valu<23>,
                     k_valu<24>, k_valu<25>, k_valu<26>, k_valu<27>, k_valu<28>, k_valu<29>,
                     k_valu<30>, k_valu<31>, k_valu<32>, k_valu<33>, k_valu<34>, k_valu<35>,
                     k_valu<36>, k_valu<37>, k_valu<38>, k_valu<39>, k_valu<40>, k_valu<41>,
                     k_valu<42>, k_valu<43>, k_valu<44>, k_valu<45>, k_valu<46>, k_valu<47>,
                     k_valu<48>, k_valu<49>, k_valu<50>};
    unsigned long long* cyc;
    uint32_t* sink;
    const int max_waves = cus * 32;
    (void)hipMalloc(&cyc, sizeof(unsigned long long) * max_waves);
    (void)hipMalloc(&sink, 4);
    unsigned long long* h = (unsigned long long*)malloc(sizeof(unsigned long long) * max_waves);
    const int iters = 400;
    const double instr_per_wave = (double)iters * kUnroll * 8;
    printf("cycles per wave64 instruction per SIMD (s_memtime), %d CUs, one block of W*4 waves per CU\n", cus);
    printf("%-26s %8s %8s %8s %8s\n", "op", "1w/SIMD", "2w/SIMD", "4w/SIMD", "8w/SIMD");
    for (int op = 0; op < kOps; ++op) {
        printf("%-26s", kNames[op]);
        for (int wps : {1, 2, 4, 8}) {
            // wps waves on each SIMD: 256 * wps threads per CU, in one or two workgroups
            const int block = wps <= 4 ? 256 * wps : 1024, per_cu = 256 * wps / block;
            hipLaunchKernelGGL(fns[op], dim3(cus * per_cu), dim3(block), 0, 0, cyc, sink, 4, 1u);
            hipLaunchKernelGGL(fns[op], dim3(cus * per_cu), dim3(block), 0, 0, cyc, sink, iters, 7u);
            if (hipDeviceSynchronize() != hipSuccess) {
                printf("  launch failed\n");
                return 1;
            }
            const int nw = cus * per_cu * block / 64;
            (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
            unsigned long long mx = 0;
            double mean = 0;
            for (int i = 0; i < nw; ++i) {
                mx = h[i] > mx ? h[i] : mx;
                mean += (double)h[i] / nw;
            }
            // wps waves share a SIMD: per-SIMD issue cost = span / (wps x instructions); the
            // waves start together (barrier), so the longest wave is the SIMD's span
            (void)mean;
            printf(" %8.2f", (double)mx / (instr_per_wave * wps));
        }
        printf("\n");
    }
    return 0;
}
