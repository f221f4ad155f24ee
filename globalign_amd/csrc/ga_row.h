// ga_row.h -- one row of the row-scan fill for one 64-column stripe, as a hand-scheduled
// gfx950 instruction sequence (included by ga_kernels.hip and tools/micro/row_bench.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ga {

// One row of one stripe, hand-scheduled (gfx950 wave64: a dependent VALU issues every 4
// cycles; a DPP op whose source OR old-value (destination) VGPR was written by one of the
// two previous VALU ops must wait 2 states: the previous row's traceback-code ops fill them).  Inputs: Hprev = H'(i-1, j), Yc = h2'(i-1, j),
// eh = H'(i-1, edge) (becomes the diagonal), ev = V~(i, edge), q = the profile word holding
// sub'(a_i, b_j) at selector SEL; p* = M', X', Y', H' of the row whose code is emitted
// into acc at bit sh (W-bit fields).  Outputs: M', X', H', V~ of this row and h2' below it.
#define GA_ROW_ASM(SEL)                                                                              \
    asm volatile(                                                                                    \
        "v_sub_u32 %[c1], %[pX], %[pH]\n\t"                                                         \
        "v_sub_u32 %[c2], %[pY], %[pH]\n\t"                                                         \
        "v_mov_b32_dpp %[eh], %[Hp] wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"                      \
        "v_add_u32_sdwa %[M], sext(%[q]), %[eh] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:" SEL " src1_sel:DWORD\n\t"\
        "v_min_i32 %[S], %[M], %[Yc]\n\t"                                                           \
        "v_sub_u32 %[c3], %[pM], %[pH]\n\t"                                                         \
        "v_min_u32 %[c1], %[c1], %[op1]\n\t"                                                        \
        "v_min_i32_dpp %[S], %[S], %[S] row_shr:1 row_mask:0xf bank_mask:0xf\n\t"                   \
        "v_min_u32 %[c2], %[c2], %[op1]\n\t"                                                        \
        "v_min_u32 %[c3], %[c3], 1\n\t"                                                             \
        "v_min_i32_dpp %[S], %[S], %[S] row_shr:2 row_mask:0xf bank_mask:0xf\n\t"                   \
        "v_lshl_or_b32 %[c1], %[c2], %[W], %[c1]\n\t"                                               \
        "v_lshl_or_b32 %[c1], %[c3], %[W2], %[c1]\n\t"                                              \
        "v_min_i32_dpp %[S], %[S], %[S] row_shr:4 row_mask:0xf bank_mask:0xf\n\t"                   \
        "v_lshl_or_b32 %[acc], %[c1], %[SH], %[acc]\n\t"                                            \
        "s_nop 0\n\t"                                                                               \
        "v_min_i32_dpp %[S], %[S], %[S] row_shr:8 row_mask:0xf bank_mask:0xf\n\t"                   \
        "s_nop 1\n\t"                                                                               \
        "v_min_i32_dpp %[S], %[S], %[S] row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"                \
        "s_nop 1\n\t"                                                                               \
        "v_min_i32_dpp %[S], %[S], %[S] row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"                \
        "v_min_i32 %[Vt], %[S], %[ev]\n\t"                                                          \
        "s_nop 1\n\t"                                                                               \
        "v_mov_b32_dpp %[ev], %[Vt] wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"                      \
        "v_add_u32 %[X], %[ev], %[o]\n\t"                                                           \
        "v_min3_i32 %[H], %[M], %[X], %[Yc]\n\t"                                                    \
        "v_add_u32 %[c2], %[H], %[o]\n\t"                                                           \
        "v_min_i32 %[Ycn], %[Yc], %[c2]"                                                            \
        : [eh] "+v"(eh), [ev] "+v"(ev), [acc] "+v"(acc), [M] "=&v"(M), [S] "=&v"(S), [c1] "=&v"(c1),     \
          [c2] "=&v"(c2), [c3] "=&v"(c3), [Vt] "=&v"(Vt), [X] "=&v"(X), [H] "=&v"(H), [Ycn] "=&v"(Ycn)  \
        : [Hp] "v"(Hprev), [q] "v"(qw), [Yc] "v"(Yc), [pX] "v"(pX), [pY] "v"(pY), [pM] "v"(pM),          \
          [pH] "v"(pH), [op1] "s"(op1), [o] "s"(o), [W] "i"(W), [W2] "i"(2 * W), [SH] "s"(sh))

template <int W, int SELI, bool Q16>
__device__ __forceinline__ void row_asm(int Hprev, int Yc, int eh, int ev, uint32_t qw, int pM, int pX, int pY,
                                        int pH, unsigned op1, int o, unsigned sh, uint32_t& acc, int& M, int& X,
                                        int& H, int& Vt, int& Ycn) {
    int S, c1, c2, c3;
    if (Q16) {
        if (SELI == 0) GA_ROW_ASM("WORD_0");
        else GA_ROW_ASM("WORD_1");
    } else {
        if (SELI == 0) GA_ROW_ASM("BYTE_0");
        else if (SELI == 1) GA_ROW_ASM("BYTE_1");
        else if (SELI == 2) GA_ROW_ASM("BYTE_2");
        else GA_ROW_ASM("BYTE_3");
    }
}
#undef GA_ROW_ASM

}  // namespace ga
