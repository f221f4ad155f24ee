// ga_group.h -- one step of the group-scan fill, shared by the kernel
// (ga_group.hip) and tools/micro/group_bench.hip.
//
// A stripe is 64*T columns.  The 64 lanes form G = 64/L groups of L lanes; lane (g, k) owns the T
// adjacent columns j0 + (g*L + k)*T + 1 .. + T, and at step t group g works on row t - g + 1.
// Within a group a row is a prefix-min scan (the row scan of fill_kernel over L lanes instead of
// 64); between groups it is skewed by one row per group, as the lane kernel skews lanes.  So a
// stripe hands its right edge on G steps after its first row (the lane kernel: 64), and a step
// costs log2(L) DPP scan ops (the row scan: 6).
//
// Shifted-potential recurrence of row r, columns c of a lane:
//   M'  = H'(r-1, c-1) + sub'            U = min(M', Y')   with Y' = h2'(r-1, c)
//   h1'(r, c) = min(h1'(r, c-1), U + o)  X'(r, c) = h1'(r, c-1)
//   H'  = min(U, X')                     h2'(r, c) = min(Y', H' + o)
// The lane's T candidates U + o are prefix-minimised in registers (P); one group scan of the lanes'
// totals, seeded at the group's first lane with the left group's h1' of the same row (computed one
// step earlier), gives E = h1' left of the lane's first column; then X'(c) = min(E, P[c-1]).
//   left group's h1'(r, last)    : its last lane's V of step t-1  -> wave_shr:1 of B = last ? V : P
//   left column's H'(r-1, last)   : in-group the left lane's H of step t-1; from the left group its
//                                   last lane's H of step t-2      -> wave_shr:1 of B2 = last ? Hold : Hnew
// Lane 0 of the wave (group 0's first lane) takes the stripe's left edge as the DPP "old" value.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ga {

// inclusive prefix-min within groups of L lanes (4, 8 or 16); a lane without a source in its group
// takes its own value (min(x, x) = x)
template <int L>
__device__ __forceinline__ int gscan_min(int x) {
    static_assert(L == 4 || L == 8 || L == 16, "groups of 4, 8 or 16 lanes");
    if constexpr (L == 16) {
        x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x111, 0xf, 0xf, false));  // row_shr:1
        x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x112, 0xf, 0xf, false));  // row_shr:2
        x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x114, 0xf, 0xf, false));  // row_shr:4
        x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x118, 0xf, 0xf, false));  // row_shr:8
    } else {
        x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x90, 0xf, 0xf, false));  // quad_perm [0,0,1,2]
        x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x44, 0xf, 0xf, false));  // quad_perm [0,1,0,1]
        if constexpr (L == 8)
            x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x114, 0xf, 0xa, false));  // row_shr:4, banks 1 and 3
    }
    return x;
}

// lane l takes lane l-1's x; lane 0 takes `edge`
__device__ __forceinline__ int gshr1(int edge, int x) { return __builtin_amdgcn_update_dpp(edge, x, 0x138, 0xf, 0xf, false); }
// mk ? a : b for a per-lane all-ones / zero mask (one v_bfi_b32: a v_cndmask on the step's dependent
// chain measured 22 cycles of latency, tools/micro/group_bench.hip)
__device__ __forceinline__ int gsel(int mk, int a, int b) {
    int r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mk), "v"(a), "v"(b));
    return r;
}

// One step of a lane.  State in: H = H'(r-1, c), Y = h2'(r-1, c), V = h1'(r-1, last column), Hd0 =
// H'(r-1, first column - 1) (the diagonal of column 0); out: the same for row r.  eX = h1'(r0, j0) and
// eH = H'(r0, j0) of group 0's row r0 (lane 0 only).  q[c]: profile dword of column c, sub' of this row
// in byte U.  lastmk: all ones where k == L-1.  MASKED: lanes whose row is outside 1.. keep their state (act false).
template <int T, int L, int U, bool MASKED>
__device__ __forceinline__ void group_step(int (&H)[T], int (&Y)[T], int& V, int& Hd0, int eX, int eH,
                                           const uint32_t (&q)[T], int o, int lastmk, bool act) {
    int M[T], Um[T], P[T], Hn[T];
    int Hd = Hd0;
#pragma unroll
    for (int c = 0; c < T; c++) {
        M[c] = Hd + (int)(int8_t)(q[c] >> (8 * U));
        Hd = H[c];
    }
#pragma unroll
    for (int c = 0; c < T; c++) Um[c] = min(M[c], Y[c]);
    P[0] = Um[0] + o;
#pragma unroll
    for (int c = 1; c < T; c++) P[c] = min(P[c - 1], Um[c] + o);
    const int E = gscan_min<L>(gshr1(eX, gsel(lastmk, V, P[T - 1])));
    Hn[0] = min(Um[0], E);
#pragma unroll
    for (int c = 1; c < T; c++) Hn[c] = min(min(Um[c], E), P[c - 1]);
    if (MASKED) {
#pragma unroll
        for (int c = 0; c < T; c++) Hn[c] = act ? Hn[c] : H[c];
    }
    Hd0 = gshr1(eH, gsel(lastmk, H[T - 1], Hn[T - 1]));
    V = min(E, P[T - 1]);
#pragma unroll
    for (int c = 0; c < T; c++) {
        const int y = min(Y[c], Hn[c] + o);
        Y[c] = (!MASKED || act) ? y : Y[c];
        H[c] = Hn[c];
    }
}

}  // namespace ga
