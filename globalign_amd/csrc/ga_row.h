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

// one step of an inclusive prefix-min scan over the wave (DPP; disabled lanes keep INT_MAX)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_min(int x) {
    return min(x, __builtin_amdgcn_update_dpp(0x7fffffff, x, CTRL, ROWMASK, 0xf, false));
}
__device__ __forceinline__ int wave_scan_min(int x) {
    x = dpp_min<0x111, 0xf>(x);  // row_shr:1
    x = dpp_min<0x112, 0xf>(x);  // row_shr:2
    x = dpp_min<0x114, 0xf>(x);  // row_shr:4
    x = dpp_min<0x118, 0xf>(x);  // row_shr:8
    x = dpp_min<0x142, 0xa>(x);  // row_bcast:15 -> rows 1, 3
    x = dpp_min<0x143, 0xc>(x);  // row_bcast:31 -> rows 2, 3
    return x;
}
// lane l takes lane l-1's value; lane 0 takes `edge`
__device__ __forceinline__ int shr1(int edge, int x) { return __builtin_amdgcn_update_dpp(edge, x, 0x138, 0xf, 0xf, false); }

// One row of a blocked stripe (T columns per lane; fill_blocked in ga_kernels.hip):
//   M' = H'(i-1, j-1) + sub', U = min(M', Y'), P = the lane's prefix-min of U, one wave scan
//   of the lanes' totals, C = the scan of the lane to the left (lane 0: ev = V~(i, left edge)),
//   V~ = min(C, P), X' = V~(j-1) + o, H' = min(U, X'), h2' = min(Y', H' + o).
// Hprev/Yc: H'(i-1, j) / h2'(i-1, j) in, H'(i, j) / h2'(i, j) out; eh = H'(i-1, left edge);
// oH / oV: what the next stripe needs from this lane's last column (H'(i-1), V~(i)).
// TB: the cell's traceback code goes into acc[k] at byte uu*CB (W-bit fields, fill_kernel).
template <int T, bool TB, int CB>
__device__ __forceinline__ void blocked_row(int (&Hprev)[T], int (&Yc)[T], int eh, int ev, const int (&sub)[T], int o,
                                            unsigned op1, int uu, uint32_t (&acc)[T][4 * CB], int& oH, int& oV) {
    constexpr int W = (8 * CB - 1) / 2;
    int M[T], U[T], P[T];
    M[0] = shr1(eh, Hprev[T - 1]) + sub[0];
#pragma unroll
    for (int k = 1; k < T; k++) M[k] = Hprev[k - 1] + sub[k];
#pragma unroll
    for (int k = 0; k < T; k++) U[k] = min(M[k], Yc[k]);
    P[0] = U[0];
#pragma unroll
    for (int k = 1; k < T; k++) P[k] = min(P[k - 1], U[k]);
    const int Wv = min(wave_scan_min(P[T - 1]), ev);  // V~ at this lane's last column
    const int C = shr1(ev, Wv);                       // V~ left of this lane's first column
    oH = Hprev[T - 1];
    oV = Wv;
    int Vl = C;
#pragma unroll
    for (int k = 0; k < T; k++) {
        const int X = Vl + o;
        const int H = min(U[k], X);
        if (TB) {
            const unsigned code = min((unsigned)(X - H), op1) | (min((unsigned)(Yc[k] - H), op1) << W) |
                                  (min((unsigned)(M[k] - H), 1u) << (2 * W));
            const int pu = uu * CB;
            acc[k][pu >> 2] |= code << (pu * 8 & 31);
        }
        if (k + 1 < T) Vl = min(C, P[k]);
        Yc[k] = min(Yc[k], H + o);
        Hprev[k] = H;
    }
}


// Four steps of the anti-diagonal fill (fill_diag_kernel), hand-scheduled: per step two DPP
// lane shifts (the left lane's H' and h1' of the previous step; lane 0 keeps the stripe's
// left edge that is already in the register), M' = H'(diag) + sub' (SDWA byte/word of the
// profile dword), H' = min3, h1' and h2' = min(., H' + o).  A DPP source is always written
// >= 2 VALU ops earlier (the gfx950 DPP read hazard), so no s_nop is needed.
//   eh[u], ex[u]: in: the edge (H', h1') of step u's row in lane 0; out: HL / XL of step u
//   Hd: H'(i-1, j-1) of step 0 (in) -> of the next sub-chunk's step 0 (out: eh[3])
//   H, X: the previous step's H' / h1' (in) -> step 3's (out); oH/oX: every step's
#define GA_DIAG_STEP(EH, EX, HD, HIN, XIN, QV, SEL, OH, OX)                                          \
    "v_mov_b32_dpp " EH ", " HIN " wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"                         \
    "v_mov_b32_dpp " EX ", " XIN " wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"                         \
    "v_add_u32_sdwa %[M], sext(" QV "), " HD " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:" SEL " src1_sel:DWORD\n\t" \
    "v_min3_i32 " OH ", %[M], " EX ", %[Y]\n\t"                                                       \
    "v_add_u32 %[Ho], " OH ", %[o]\n\t"                                                               \
    "v_min_i32 " OX ", " EX ", %[Ho]\n\t"                                                             \
    "v_min_i32 %[Y], %[Y], %[Ho]\n\t"
// step 0 of a block: its M' first and one wait state, so the DPPs are clear of whatever VALU
// op the compiler placed just before the block (e.g. a copy into H or X)
#define GA_DIAG_STEP0(EH, EX, HD, HIN, XIN, QV, SEL, OH, OX)                                         \
    "v_add_u32_sdwa %[M], sext(" QV "), " HD " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:" SEL " src1_sel:DWORD\n\t" \
    "s_nop 0\n\t"                                                                                   \
    "v_mov_b32_dpp " EH ", " HIN " wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"                         \
    "v_mov_b32_dpp " EX ", " XIN " wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"                         \
    "v_min3_i32 " OH ", %[M], " EX ", %[Y]\n\t"                                                       \
    "v_add_u32 %[Ho], " OH ", %[o]\n\t"                                                               \
    "v_min_i32 " OX ", " EX ", %[Ho]\n\t"                                                             \
    "v_min_i32 %[Y], %[Y], %[Ho]\n\t"

// e0..e3 / x0..x3: the left edge (H', h1') of the block's four rows, taken by lane 0; the
// registers are overwritten (the DPP shifts land in them), so the caller hands its read buffer
template <bool Q16>
__device__ __forceinline__ void diag4_asm(int& e0, int& e1, int& e2, int& e3, int& x0, int& x1, int& x2, int& x3,
                                          int Hd, int& H, int& X, int& Y, uint32_t q0, uint32_t q1, int o,
                                          int (&oH)[4], int (&oX)[4]) {
    int M, Ho;
    if (!Q16) {
        asm volatile(GA_DIAG_STEP0("%[e0]", "%[x0]", "%[Hd]", "%[H]", "%[X]", "%[q0]", "BYTE_0", "%[h0]", "%[y0]")
                     GA_DIAG_STEP("%[e1]", "%[x1]", "%[e0]", "%[h0]", "%[y0]", "%[q0]", "BYTE_1", "%[h1]", "%[y1]")
                     GA_DIAG_STEP("%[e2]", "%[x2]", "%[e1]", "%[h1]", "%[y1]", "%[q0]", "BYTE_2", "%[h2]", "%[y2]")
                     GA_DIAG_STEP("%[e3]", "%[x3]", "%[e2]", "%[h2]", "%[y2]", "%[q0]", "BYTE_3", "%[h3]", "%[y3]")
                     : [e0] "+v"(e0), [e1] "+v"(e1), [e2] "+v"(e2), [e3] "+v"(e3), [x0] "+v"(x0),
                       [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [h0] "=&v"(oH[0]), [h1] "=&v"(oH[1]),
                       [h2] "=&v"(oH[2]), [h3] "=&v"(oH[3]), [y0] "=&v"(oX[0]), [y1] "=&v"(oX[1]), [y2] "=&v"(oX[2]),
                       [y3] "=&v"(oX[3]), [Y] "+v"(Y), [M] "=&v"(M), [Ho] "=&v"(Ho)
                     : [Hd] "v"(Hd), [H] "v"(H), [X] "v"(X), [q0] "v"(q0), [o] "s"(o));
    } else {
        asm volatile(GA_DIAG_STEP0("%[e0]", "%[x0]", "%[Hd]", "%[H]", "%[X]", "%[q0]", "WORD_0", "%[h0]", "%[y0]")
                     GA_DIAG_STEP("%[e1]", "%[x1]", "%[e0]", "%[h0]", "%[y0]", "%[q0]", "WORD_1", "%[h1]", "%[y1]")
                     GA_DIAG_STEP("%[e2]", "%[x2]", "%[e1]", "%[h1]", "%[y1]", "%[q1]", "WORD_0", "%[h2]", "%[y2]")
                     GA_DIAG_STEP("%[e3]", "%[x3]", "%[e2]", "%[h2]", "%[y2]", "%[q1]", "WORD_1", "%[h3]", "%[y3]")
                     : [e0] "+v"(e0), [e1] "+v"(e1), [e2] "+v"(e2), [e3] "+v"(e3), [x0] "+v"(x0),
                       [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [h0] "=&v"(oH[0]), [h1] "=&v"(oH[1]),
                       [h2] "=&v"(oH[2]), [h3] "=&v"(oH[3]), [y0] "=&v"(oX[0]), [y1] "=&v"(oX[1]), [y2] "=&v"(oX[2]),
                       [y3] "=&v"(oX[3]), [Y] "+v"(Y), [M] "=&v"(M), [Ho] "=&v"(Ho)
                     : [Hd] "v"(Hd), [H] "v"(H), [X] "v"(X), [q0] "v"(q0), [q1] "v"(q1), [o] "s"(o));
    }
    H = oH[3];
    X = oX[3];
}
#undef GA_DIAG_STEP
#undef GA_DIAG_STEP0

}  // namespace ga
