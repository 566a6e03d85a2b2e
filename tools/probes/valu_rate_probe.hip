// VALU issue-rate probe (gfx950): cycles per wave64 instruction for the instruction kinds the codec
// uses, with 8 independent chains per wave, at 1..8 waves per SIMD (every CU busy).
// build: hipcc --offload-arch=gfx950 -O3 tools/probes/valu_rate_probe.hip -o build/valu_rate_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define BODY8(INS) INS(a0) INS(a1) INS(a2) INS(a3) INS(a4) INS(a5) INS(a6) INS(a7)
#define K_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x6c" : "+v"(x) : "v"(k), "v"(s));
#define K_SDWA(x) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "+v"(x) : "v"(k));
#define K_DOT4(x) asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(x) : "v"(k), "v"(s));
#define K_ALIGN(x) asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(x) : "v"(k));
#define K_BFE(x) asm volatile("v_bfe_u32 %0, %0, 8, 4" : "+v"(x));
#define K_MUL24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_LIT(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "s"(0x7f7f7f7fu), "v"(k));
#define K_LSHLADD(x) asm volatile("v_lshl_add_u32 %0, %0, 8, %1" : "+v"(x) : "v"(k));
#define K_PKMAX(x) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_DPP(x) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(k));
#define K_CND(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(k) : "vcc");

// each wave: shader-clock cycles (s_memtime) and 100 MHz ticks (s_memrealtime) around its loop
#define K_OR(x) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_ORL(x) asm volatile("v_or_b32 %0, 0x80808080, %0" : "+v"(x));
#define K_XORL(x) asm volatile("v_xor_b32 %0, 0x80808080, %0" : "+v"(x));
#define K_ADDL(x) asm volatile("v_add_u32 %0, 0x7f7f7f7f, %0" : "+v"(x));
#define K_SUB(x) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_NOT(x) asm volatile("v_not_b32 %0, %0" : "+v"(x));
#define K_ASHR(x) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(x) : "v"(k));
#define K_LSHRI(x) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(x));
#define K_ANDI(x) asm volatile("v_and_b32 %0, 15, %0" : "+v"(x));
#define K_BITOP3S(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x6c" : "+v"(x) : "v"(k), "s"(0x1cu));
#define K_BITOP3I(x) asm volatile("v_bitop3_b32 %0, %0, %1, 28 bitop3:0x6c" : "+v"(x) : "v"(k));
#define K_MIN(x) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_FFBL(x) asm volatile("v_ffbl_b32 %0, %0" : "+v"(x));
#define K_MBCNT(x) asm volatile("v_mbcnt_lo_u32_b32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_ADDC(x) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(k) : "vcc");
#define K_MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_PKADD(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_ADDSDWAB(x) asm volatile("v_add_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(x) : "v"(k));
#define K_CMP(x) asm volatile("v_cmp_ne_u32 vcc, %0, %1" :: "v"(x), "v"(k) : "vcc");
#define K_LSHL(x) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x) : "v"(k));
#define K_LSHLI(x) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x));
#define K_AND(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_ANDS(x) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x) : "s"(0x7f7f7f7fu));
#define K_ANDL(x) asm volatile("v_and_b32 %0, 0x7f7f7f7f, %0" : "+v"(x));
#define K_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_ADDI(x) asm volatile("v_add_u32 %0, 5, %0" : "+v"(x));
#define K_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_OR3(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_ANDORV(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_LSHLADDV(x) asm volatile("v_lshl_add_u32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_MAX(x) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_BCNT(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_BFI(x) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_MOV(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(k));
#define K_BFEV(x) asm volatile("v_bfe_u32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_ALIGNV(x) asm volatile("v_alignbyte_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(s));
#define K_CNDV(x) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "s"(0xffffffffffull));
#define K_SUBREV(x) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_ADDSDWA0(x) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD" : "+v"(x) : "v"(k));
#define K_ADDE64(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(k));
#define K_LSHR(x) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x) : "v"(k));
#define KERN(NAME, INS)                                                            \
    __global__ void NAME(unsigned* out, unsigned long long* tm, int iters) {      \
        unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
                 a6 = a0 + 6, a7 = a0 + 7;                                        \
        unsigned k = threadIdx.x * 77u, s = 0x03020100u;                          \
        const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
        for (int i = 0; i < iters; ++i) { BODY8(INS) BODY8(INS) }                 \
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
        if ((threadIdx.x & 63) == 0) {                                            \
            const unsigned wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;     \
            tm[2 * wv] = c1 - c0;                                                 \
            tm[2 * wv + 1] = r1 - r0;                                             \
        }                                                                         \
    }
KERN(k_add, K_ADD)
KERN(k_perm, K_PERM)
KERN(k_bitop3, K_BITOP3)
KERN(k_sdwa, K_SDWA)
KERN(k_dot4, K_DOT4)
KERN(k_align, K_ALIGN)
KERN(k_bfe, K_BFE)
KERN(k_mul24, K_MUL24)
KERN(k_mullo, K_MULLO)
KERN(k_lit, K_LIT)
KERN(k_lshladd, K_LSHLADD)
KERN(k_pkmax, K_PKMAX)
KERN(k_dpp, K_DPP)
KERN(k_cnd, K_CND)
KERN(k_lshl, K_LSHL)
KERN(k_lshli, K_LSHLI)
KERN(k_and, K_AND)
KERN(k_ands, K_ANDS)
KERN(k_andl, K_ANDL)
KERN(k_xor, K_XOR)
KERN(k_addi, K_ADDI)
KERN(k_add3, K_ADD3)
KERN(k_or3, K_OR3)
KERN(k_andorv, K_ANDORV)
KERN(k_lshlor, K_LSHLOR)
KERN(k_lshladdv, K_LSHLADDV)
KERN(k_max, K_MAX)
KERN(k_bcnt, K_BCNT)
KERN(k_bfi, K_BFI)
KERN(k_mov, K_MOV)
KERN(k_bfev, K_BFEV)
KERN(k_alignv, K_ALIGNV)
KERN(k_cndv, K_CNDV)
KERN(k_subrev, K_SUBREV)
KERN(k_addsdwa0, K_ADDSDWA0)
KERN(k_adde64, K_ADDE64)
KERN(k_lshr, K_LSHR)
KERN(k_or, K_OR)
KERN(k_orl, K_ORL)
KERN(k_xorl, K_XORL)
KERN(k_addl, K_ADDL)
KERN(k_sub, K_SUB)
KERN(k_not, K_NOT)
KERN(k_ashr, K_ASHR)
KERN(k_lshri, K_LSHRI)
KERN(k_andi, K_ANDI)
KERN(k_bitop3s, K_BITOP3S)
KERN(k_bitop3i, K_BITOP3I)
KERN(k_min, K_MIN)
KERN(k_ffbl, K_FFBL)
KERN(k_mbcnt, K_MBCNT)
KERN(k_addc, K_ADDC)
KERN(k_mulhi, K_MULHI)
KERN(k_pkadd, K_PKADD)
KERN(k_addsdwab, K_ADDSDWAB)
KERN(k_cmp, K_CMP)

typedef void (*KF)(unsigned*, unsigned long long*, int);
int main() {
    unsigned* out;
    unsigned long long* tm;
    (void)hipMalloc(&out, 256 * 8 * 256 * 4);
    (void)hipMalloc(&tm, 256 * 8 * 4 * 16);
    static unsigned long long h[256 * 8 * 4 * 2];
    const struct { const char* n; KF f; } ks[] = {
        {"v_add_u32", k_add}, {"v_or v", k_or}, {"v_or literal", k_orl}, {"v_xor literal", k_xorl},
        {"v_add literal", k_addl}, {"v_sub v", k_sub}, {"v_not", k_not}, {"v_ashrrev v", k_ashr},
        {"v_lshrrev imm", k_lshri}, {"v_and imm", k_andi}, {"v_bitop3 sgpr", k_bitop3s}, {"v_bitop3 imm", k_bitop3i},
        {"v_min_u32", k_min}, {"v_ffbl", k_ffbl}, {"v_mbcnt_lo", k_mbcnt}, {"v_add_co vcc", k_addc},
        {"v_mul_hi_u32", k_mulhi}, {"v_pk_add_u16", k_pkadd}, {"v_add sdwa src0 byte1", k_addsdwab},
        {"v_cmp_ne (vcc)", k_cmp}, {"v_lshlrev v", k_lshl}, {"v_lshrrev v", k_lshr}, {"v_bitop3_b32", k_bitop3},
        {"v_add_u32", k_add}};
    const int iters = 4000;
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    // warm the clock
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_add, dim3(ncu * 4), dim3(256), 0, 0, out, tm, iters);
    (void)hipDeviceSynchronize();
    printf("cycles (s_memtime) per wave-instruction per SIMD, 8 independent chains per wave; [MHz from s_memtime/s_memrealtime]\n");
    printf("%-20s", "waves/SIMD:");
    for (int w : {1, 2, 4, 8}) printf("%8d", w);
    printf("   MHz\n");
    for (auto& k : ks) {
        printf("%-20s", k.n);
        double mhz = 0;
        for (int w : {1, 2, 4, 8}) {
            const int nb = ncu * w;   // 256-thread blocks: one wave per SIMD each
            hipLaunchKernelGGL(k.f, dim3(nb), dim3(256), 0, 0, out, tm, iters);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h, tm, (size_t)nb * 4 * 16, hipMemcpyDeviceToHost);
            double cyc = 0, rt = 0;
            for (int i = 0; i < nb * 4; ++i) { cyc += (double)h[2 * i]; rt += (double)h[2 * i + 1]; }
            cyc /= nb * 4;
            rt /= nb * 4;
            mhz = cyc / rt * 100.0;
            printf("%8.2f", cyc / ((double)iters * 16 * w));
        }
        printf("   %.0f\n", mhz);
    }
    return 0;
}
