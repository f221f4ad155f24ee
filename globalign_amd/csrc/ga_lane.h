// ga_lane.h -- the lane-skewed step and its traceback-code helpers, shared by the
// lane fill (ga_lane.hip) and the tile recompute beside the walk (ga_rcwalk.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace ga {

// LDS counters of the lane kernel (dwords of the 256-byte counter block): cons(k) = rows of ring k
// its reader no longer needs at [2k], prod(k) = rows of ring k written at [2k-1] (k >= 1) and
// [LK_PROD0] (ring 0, the IO wave's), so compute wave w publishes {cons(w), prod(w+1)} in one store
enum { LK_PROD0 = 31, LK_PRODQ = 40, LK_ABORT = 41, LK_SLAB = 42 };
constexpr int LK_CNT_BYTES = 256;
// after the counters: a zero block (16 rows of int2) that lanes 1..63 read as their "edge" rows, so that a step
// can add its edge register to a zero-filled DPP shift (ga_lane_asm.h); then a scratch slot of 8 bytes per lane for
// the lean sub-chunk's all-lane row stores (lanes that carry no row write there); the rings start after it
constexpr int LK_ZERO_OFF = LK_CNT_BYTES;
constexpr int LK_SCR_OFF = LK_ZERO_OFF + 16 * 8;
constexpr int LK_HEAD_BYTES = LK_SCR_OFF + 64 * 8;
constexpr int LK_QMIRROR = 16;  // profile slots mirrored past the ring's end (a window reads idx .. idx+12)
constexpr unsigned LK_DONE = 0x7fffffffu;
// DBG stamps per stripe (tools/lane_stamps.py): start, end, wait cycles (edges, profile, ring space), total cycles,
// HW_ID, XCC_ID; the row-m/2 probe: edge row known landed, own row published, (the workgroup's first stripe) landed
// in ring 0 by the IO wave, (its last stripe) stored to HBM by the out-path
constexpr int LK_DBG_WORDS = 20;  // + [12] the first edge wait's cycles, [13] when it ended, [14..19] when the
                                   // wave started the sub-chunk of row 256, 1024, 4096, 16384, 64, 128
typedef unsigned lk_v2u __attribute__((ext_vector_type(2)));
// waves of a lane-fill workgroup: NWC compute waves, the IO wave, the profile wave and, for NWC <= 4, an out wave that
// only moves the last compute wave's rows to HBM (at NWC = 8 a third extra wave would put three waves on a SIMD and
// cap every wave at 168 VGPRs)
constexpr bool lane_out_wave(int nwc) { return nwc <= 4; }
constexpr int lane_block_threads(int nwc) { return 64 * (nwc + (lane_out_wave(nwc) ? 3 : 2)); }


// traceback code of a cell (CB bytes, W = (8*CB-1)/2 bits per field; fill_kernel's TbFmt): the
// saturated X'-H', Y'-H' and M' != H', all dp_array_backward's rank test needs
template <int CB>
__device__ __forceinline__ unsigned lk_code(int M, int X, int Y, int H, unsigned op1) {
    constexpr int W = (8 * CB - 1) / 2;
    return min((unsigned)(X - H), op1) | (min((unsigned)(Y - H), op1) << W) | (min((unsigned)(M - H), 1u) << (2 * W));
}
// a cell's code into byte UU*CB of its column's 16-step window
template <int CB, int UU>
__device__ __forceinline__ void lk_put(uint32_t (&acc)[4 * (CB > 0 ? CB : 1)], unsigned code) {
    if constexpr (CB > 0) {
        constexpr int bo = UU * CB, dw = bo >> 2, sh = (bo & 3) * 8;
        if constexpr (sh == 0) acc[dw] = code;
        else acc[dw] |= code << sh;
    }
}

// one step; U: the step's byte in the profile dwords; CB > 0: traceback codes into window byte UU*CB;
// MASKED: lanes above row 1 keep their row-0 state, and a partial stripe captures H'(m, n) into Hm
template <int TD, int U, int CB, int UU, bool MASKED>
__device__ __forceinline__ void lane_step(int (&H)[TD], int (&Y)[TD], int& Xl, int& Hl, int& HLp, int& RH, int& RX,
                                          int eh, int ex, const uint32_t (&q)[TD], int o,
                                          uint32_t (&acc)[TD][4 * (CB > 0 ? CB : 1)], unsigned op1, int row, bool cap,
                                          int ck, int& Hm) {
    int X = __builtin_amdgcn_update_dpp(ex, Xl, 0x138, 0xf, 0xf, false);          // h1'(i, left): lane 0 the edge
    const int HLn = __builtin_amdgcn_update_dpp(eh, Hl, 0x138, 0xf, 0xf, false);  // H'(i, left), the next diagonal
    const bool act = !MASKED || row >= 1;
    int Hd = HLp;
#pragma unroll
    for (int k = 0; k < TD; k++) {
        const int M = Hd + (int)(int8_t)(q[k] >> (8 * U));
        const int Hn = min(min(M, X), Y[k]);
        const int Ho = Hn + o;
        if constexpr (CB > 0) lk_put<CB, UU>(acc[k], lk_code<CB>(M, X, Y[k], Hn, op1));
        X = min(X, Ho);
        if (MASKED && cap && k == ck) Hm = Hn;
        Y[k] = act ? min(Y[k], Ho) : Y[k];
        Hd = H[k];
        H[k] = act ? Hn : H[k];
    }
    Xl = X;
    Hl = H[TD - 1];
    HLp = HLn;
    RH = __builtin_amdgcn_update_dpp(Hl, RH, 0x130, 0xf, 0xf, false);  // lane 63 shifts its output in
    RX = __builtin_amdgcn_update_dpp(Xl, RX, 0x130, 0xf, 0xf, false);
}

// End of a 16-step window c of traceback codes.  Byte u*CB of lane l's window holds row 16c+u-l+1
// (the lane skew), so with phi = l mod 16 the window rotated by phi cells, R_c, holds at cell
// position p < 16-phi row 16(c-l/16)+p+1 and at p >= 16-phi the row 16 earlier: the aligned word
// a = c-1-l/16 (rows 16a+1 .. 16a+16, the layout fill_kernel writes and the walk reads) is R_(c-1)
// below 16-phi and R_c above.  Per column: log2(4CB) dword-rotation stages (per-lane v_cndmask),
// 4CB v_alignbyte for the byte remainder, 4CB v_bfi for the merge, CB 16-byte stores.
template <int TD, int CB>
struct LkRot {
    static constexpr int N = 4 * CB;  // dwords per window
    bool qbit[4];                     // dword rotation (phi*CB / 4) bits
    unsigned rb;                      // byte remainder (phi*CB & 3)
    uint32_t mask[N];                 // bytes below CB*(16-phi): from R_(c-1)
    __device__ __forceinline__ void init(int phi) {
        const int q = (phi * CB) >> 2;
#pragma unroll
        for (int b = 0; b < 4; b++) qbit[b] = ((q >> b) & 1) != 0;
        rb = (unsigned)((phi * CB) & 3);
        const int lowb = CB * (16 - phi);
#pragma unroll
        for (int d = 0; d < N; d++) {
            uint32_t mk = 0;
#pragma unroll
            for (int y = 0; y < 4; y++) mk |= (4 * d + y < lowb) ? (0xffu << (8 * y)) : 0u;
            mask[d] = mk;
        }
    }
    __device__ __forceinline__ void rotate(const uint32_t (&w)[N], uint32_t (&r)[N]) const {
        uint32_t v[N];
#pragma unroll
        for (int d = 0; d < N; d++) v[d] = w[d];
#pragma unroll
        for (int b = 0; (1 << b) < N; b++) {
            uint32_t t[N];
#pragma unroll
            for (int d = 0; d < N; d++) t[d] = qbit[b] ? v[(d + (1 << b)) % N] : v[d];
#pragma unroll
            for (int d = 0; d < N; d++) v[d] = t[d];
        }
#pragma unroll
        for (int d = 0; d < N; d++) r[d] = __builtin_amdgcn_alignbyte(v[(d + 1) % N], v[d], rb);
    }
};

// compile-time loop U .. N-1 over a generic lambda (steps of a sub-chunk)
template <int U, int N>
struct LkUnroll {
    template <class F>
    __device__ __forceinline__ static void run(F& f) {
        f(std::integral_constant<int, U>{});
        LkUnroll<U + 1, N>::run(f);
    }
};
template <int N>
struct LkUnroll<N, N> {
    template <class F>
    __device__ __forceinline__ static void run(F&) {}
};

}  // namespace ga
