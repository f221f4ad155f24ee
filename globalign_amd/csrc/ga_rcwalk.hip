// ga_rcwalk.hip -- the recompute walk (dp_array_backward, globaligner.py:395-593).
//
// The whole-problem fill stores no traceback words: the lane fill (ga_lane.hip, RC variant) leaves only
// checkpoints -- every stripe's right edge column and, every stck_every steps, each lane's state (a
// staircase across the stripe).  One launch then runs the walk and the traceback words it needs side by
// side:
//   workgroup 0   the walk (walk_body, ga_walk.h) with its loaders reading 64x64 tiles of words from a
//                 small direct-mapped cache in HBM, each tile once its block's flag says it is written;
//   workgroups 1+ recompute workers, one per wave: a worker claims (CAS on the block's flag) the nearest
//                 block of the window ahead of the walker that nobody has claimed, re-runs the lane fill's
//                 steps for it from the staircase checkpoint above (up to stck_every + 126 steps of the
//                 stripe's 64*TD columns), stages the cells' traceback codes in LDS and writes the block's
//                 words into the cache with write-through (sc1) stores, then the flag.
// A block is 64 rows of one fill stripe: TD walker tiles.  The walk path only moves up and left, so the
// window (up to 32 block rows x 8 stripes up-left of the walker's block) always holds the tiles it can reach
// next, and a 64 x 32-block cache never overwrites a block the walker may still read.  The words are the ones the
// full traceback fill writes (lk_code of the same exact int32 cells), so the walk is unchanged.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ga_device.h"
#include "ga_lane.h"
#include "ga_sync.h"
#include "ga_walk.h"
#ifdef GA_EXPERIMENTS  // the tie-to-tie walk: measured slower than the word walk, experiments only
#include "ga_jump.h"
#endif

namespace ga {

constexpr int RC_ROWS = 64;   // rows per block (one walker tile row)

// stage bytes per column: rows t0-63 .. t0+nst (every row a lane visits in a block's steps, so the code
// stores need no range test; only rows R0+1 .. R0+64 are read back), +16 against bank conflicts
__host__ __device__ inline int rc_sp(int CB, int every) { return (((every + 136) * CB + 16) + 15) & ~15; }
__host__ __device__ inline int rc_aw(int every) { return every + 256; }    // a-window dwords / edge-window rows
int rc_worker_bytes(int TD, int CB, int every) {
    return 64 * TD * rc_sp(CB, every) + rc_aw(every) * 4 + rc_aw(every) * 8;
}

__device__ __forceinline__ void st16_sc1(uint4* p, uint4 v) {
    const wk_u4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
}

// A block's code window (dword i: a[base+i .. base+i+3]) and left-edge window (rows t0+1 ..) into LDS: four rounds of
// loads issued before any store, so the block waits for one memory latency, not one per 64 entries.
__device__ __forceinline__ void rc_windows(const RcArgs& r, uint32_t* awin, int2* ewin, int nst, int base, int t0, int s,
                                           int lane) {
    const int m = r.m;
    for (int i0 = lane; i0 < nst + 72; i0 += 256) {
        uint32_t v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            v[q] = 0;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int x = base + i0 + 64 * q + u;
                v[q] |= (x >= 0 && x < m) ? (uint32_t)r.a[x] << (8 * u) : 0u;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (i0 + 64 * q < nst + 72) awin[i0 + 64 * q] = v[q];
    }
    const int2* E = s == 0 ? r.left : r.colck + (long long)(s - 1) * (m + 1 + COLCK_PAD);
    for (int i0 = lane; i0 < nst + 8; i0 += 256) {
        int2 v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = E[min(t0 + 1 + i0 + 64 * q, m)];
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (i0 + 64 * q < nst + 8) ewin[i0 + 64 * q] = v[q];
    }
}

// Recompute block (bi, bs): rows 64*bi+1 .. 64*bi+64 of fill stripe bs, its traceback words into the cache.
template <int TD, int CB>
__device__ bool rc_block(const RcArgs& r, const int8_t* stab, uint8_t* wl, int bi, int bs, int lane) {
    const int SP = rc_sp(CB, r.stck_every), AW = rc_aw(r.stck_every);
    uint8_t* stage = wl;                                                  // [64*TD columns][SP]
    uint32_t* awin = reinterpret_cast<uint32_t*>(wl + 64 * TD * SP);  // dword i: a[base+i .. base+i+3]
    int2* ewin = reinterpret_cast<int2*>(awin + AW);                      // left edge of rows t0+1 ..
    const int m = r.m, n = r.n, o = r.o;
    const int R0 = bi * RC_ROWS;
    const int nrow = min(RC_ROWS, m - R0);
    const int ck = R0 / r.stck_every;  // the staircase checkpoint above the block (0: row 0)
    const int t0 = ck * r.stck_every;
    const int nst = ((R0 + nrow + 62) - t0 + 1 + 7) & ~7;  // steps, whole pairs of 4-step groups (lane 63 ends the block)
    const int base = t0 - 63;                               // a index of lane 63's row at step t0
    const int s = bs;
    const int j0 = s * 64 * TD, jl = j0 + lane * TD;
    // (a lane reads dwords up to nst + 67: one group ahead)
    rc_windows(r, awin, ewin, nst, base, t0, s, lane);
    int bcode[TD];
    int H[TD], Y[TD];
    int Xl = 0, HLp = 0;
#pragma unroll
    for (int c = 0; c < TD; c++) bcode[c] = jl + c + 1 <= n ? r.b[jl + c] : 0;
    if (ck == 0) {
#pragma unroll
        for (int c = 0; c < TD; c++) {
            const int2 t = r.top[min(jl + c + 1, n)];
            H[c] = t.x;
            Y[c] = t.y;
        }
        HLp = r.top[min(jl, n)].x;
    } else {
        const int2* st = r.stck + ((long long)(ck - 1) * r.nstripes + s) * (TD + 1) * 64 + lane;
#pragma unroll
        for (int c = 0; c < TD; c++) {
            const int2 v = st[c * 64];
            H[c] = v.x;
            Y[c] = v.y;
        }
        const int2 v = st[TD * 64];
        Xl = v.x;
        HLp = v.y;
    }
    int Hl = H[TD - 1];
    const unsigned op1 = (unsigned)o + 1u;
    // this lane's code bytes: column c at stage + (lane*TD + c)*SP, row r at (r - t0 + 63)*CB
    uint8_t* lst = stage + lane * TD * SP + (63 - t0) * CB;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the windows written by this wave
    __builtin_amdgcn_wave_barrier();
    // the profile and edges of a group of 4 steps, read one group ahead
    auto reads = [&](int g, int (&sb)[4][TD], int (&eh)[4], int (&ex)[4]) {
        const uint32_t aw = awin[t0 + g - lane - base];  // this lane's a codes at steps t .. t+3
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int ac = (int)((aw >> (8 * u)) & 0xffu) * 32;
#pragma unroll
            for (int c = 0; c < TD; c++) sb[u][c] = stab[ac + bcode[c]];
        }
        const int4 e01 = *reinterpret_cast<const int4*>(ewin + g);
        const int4 e23 = *reinterpret_cast<const int4*>(ewin + g + 2);
        eh[0] = e01.x; eh[1] = e01.z; eh[2] = e23.x; eh[3] = e23.z;
        ex[0] = e01.y; ex[1] = e01.w; ex[2] = e23.y; ex[3] = e23.w;
    };
    auto group = [&](int g, const int (&sb)[4][TD], const int (&eh)[4], const int (&ex)[4], auto MK) {
        constexpr bool MASKED = decltype(MK)::value;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int row = t0 + g + u - lane + 1;
            const bool act = !MASKED || row >= 1;
            int X = __builtin_amdgcn_update_dpp(ex[u], Xl, 0x138, 0xf, 0xf, false);  // h1'(row, left)
            const int HLn = __builtin_amdgcn_update_dpp(eh[u], Hl, 0x138, 0xf, 0xf, false);
            int Hd = HLp;
            uint8_t* dst = lst + row * CB;
#pragma unroll
            for (int c = 0; c < TD; c++) {
                const int M = Hd + sb[u][c];
                const int Hn = min(min(M, X), Y[c]);
                const unsigned code = lk_code<CB>(M, X, Y[c], Hn, op1);
                if constexpr (CB == 1) dst[c * SP] = (uint8_t)code;
                else if constexpr (CB == 2) *reinterpret_cast<uint16_t*>(dst + c * SP) = (uint16_t)code;
                else *reinterpret_cast<uint32_t*>(dst + c * SP) = code;
                const int Ho = Hn + o;
                X = min(X, Ho);
                Y[c] = act ? min(Y[c], Ho) : Y[c];
                Hd = H[c];
                H[c] = act ? Hn : H[c];
            }
            Xl = X;
            Hl = H[TD - 1];
            HLp = HLn;
        }
    };
    int sbA[4][TD], ehA[4], exA[4], sbB[4][TD], ehB[4], exB[4];
    reads(0, sbA, ehA, exA);
    // (row 0: lanes above row 1 keep their state for the first 64 steps)
    const int gmask = ck == 0 ? 64 : 0;
    for (int g = 0; g < nst; g += 8) {
        reads(g + 4, sbB, ehB, exB);
        if (g < gmask) group(g, sbA, ehA, exA, std::true_type{});
        else group(g, sbA, ehA, exA, std::false_type{});
        reads(g + 8, sbA, ehA, exA);
        if (g + 4 < gmask) group(g + 4, sbB, ehB, exB, std::true_type{});
        else group(g + 4, sbB, ehB, exB, std::false_type{});
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    // The cache: block (bi, bs) at slot (bi mod RC_CACHE_I, bs mod RC_CACHE_S); TC words per lane per 64-column
    // stripe of the cache (RC_CACHE_I * 4 * CB).  Only a block the walker can still reach is written: the walk
    // moves up and left and its loaders read tiles of the 4 x 4 block at its tile, so a block below the
    // walker's tile row, or right of its tile column, is never read again.  Safety: a block Y written now passed
    // this check, so at this moment the walker's block row V is >= Y.  A block X sharing Y's slot (X = Y - 64k
    // above it; the column axis alike with 32 and 7) is claimed only from a view V' of the walker with
    // X >= V' - 31, i.e. V' <= Y - 33: after the walker has moved >= 33 block rows (>= 2112 steps) past where it
    // is now.  Y's stores issued here drain (vmcnt(0), rc_server) long before, so X's words, written after X's
    // recompute, are the slot's last.  (With a 16-deep cache and 16-deep candidates the margin was zero, and
    // two workers with different views could leave the walker another block's words)
    {
        const unsigned pv = (unsigned)sgpr((int)g_ld(r.pos));
        const int tile = pv ? (int)(pv - 1u) : r.tile0;
        if (bi > (tile >> 16) || bs * TD > (tile & 0xffff)) return false;  // out of reach: nobody reads it
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slot's owner tag cleared (rc_server) before any word
#pragma unroll
    for (int p = 0; p < TD; p++) {
        const uint4* src = reinterpret_cast<const uint4*>(stage + (p * 64 + lane) * SP + (R0 - t0 + 64) * CB);  // row R0+1
        uint4* dst = reinterpret_cast<uint4*>(r.tb) +
                     ((long long)((bs % RC_CACHE_S) * TD + p) * r.TC + (bi % RC_CACHE_I) * 4 * CB) * 64 + lane;
#pragma unroll
        for (int d = 0; d < 4 * CB; d++) st16_sc1(dst + d * 64, src[d]);
    }
    return true;
}

constexpr int JLUT_OFF = 2048;                 // (tie-to-tie walk) after the int16 sub' table
constexpr int JWORK_OFF = JLUT_OFF + 1024 * 16;  // then the workers

#ifdef GA_EXPERIMENTS
// ---------------------------------------------------------------------------------------------------------------
// The tie-to-tie walk's workers (ga_jump.h): the same recompute, but instead of traceback codes each
// cell's three jump entries (one per entering level), built in the same skewed order as the cells themselves: the
// entry of (r, c, L) is the cell's singleton move at level L prepended to the entry of the successor it moves to,
// (r-1, c-1) at level 0, (r, c-1) at level 1 or (r-1, c) at level 2, which are exactly the cells the recurrence
// reads (the diagonal and the left column come from lane l-1 by the same two DPP shifts as H' and h1').  A tie,
// or a successor outside the block (the stripe's left edge, the block's first checkpoint row), ends the run.
//
// Per cell: an index from the saturated differences X'-H', Y'-H' (<= o+1, so o <= 14), M' != H' and a_i != b_j,
// one 16-byte LUT read {selectors of (E0, E1), selector of E2, tie words of levels 0/1, of level 2}, three
// prepends (one v_lshl_or each), two v_perm that pick each level's candidate (diag / left / up / none), and the
// tie words or'ed in for the stored copy.
constexpr int JSTAGE_ROWS = 65;  // the block's 64 rows + a scratch row for lanes outside them
__host__ __device__ inline int rc_jump_worker_bytes(int TD, int every) {
    return 3 * JSTAGE_ROWS * 64 * TD * 2 + rc_aw(every) * 4 + rc_aw(every) * 8;
}

template <int TD>
__device__ bool rc_block_jump(const RcArgs& r, const int16_t* stab, const uint4* lut, uint8_t* wl, int bi, int bs,
                              int lane) {
    static_assert(TD == 1 || TD == 2 || TD == 4, "jump entries: at most 4 columns per lane");
    const int AW = rc_aw(r.stck_every);
    constexpr int SC = 64 * TD;                                         // stage columns
    uint16_t* stage = reinterpret_cast<uint16_t*>(wl);                  // [3][JSTAGE_ROWS][SC]
    uint32_t* awin = reinterpret_cast<uint32_t*>(wl + 3 * JSTAGE_ROWS * SC * 2);
    int2* ewin = reinterpret_cast<int2*>(awin + AW);
    const int m = r.m, n = r.n, o = r.o;
    const int R0 = bi * RC_ROWS;
    const int nrow = min(RC_ROWS, m - R0);
    const int ck = R0 / r.stck_every;
    const int t0 = ck * r.stck_every;
    const int nst = ((R0 + nrow + 62) - t0 + 1 + 7) & ~7;
    const int base = t0 - 63;
    const int s = bs;
    const int j0 = s * 64 * TD, jl = j0 + lane * TD;
    // (a lane reads dwords up to nst + 67: one group ahead)
    rc_windows(r, awin, ewin, nst, base, t0, s, lane);
    int bcode[TD];
    int H[TD], Y[TD];
    int Xl = 0, HLp = 0;
#pragma unroll
    for (int c = 0; c < TD; c++) bcode[c] = jl + c + 1 <= n ? r.b[jl + c] : 0;
    if (ck == 0) {
#pragma unroll
        for (int c = 0; c < TD; c++) {
            const int2 t = r.top[min(jl + c + 1, n)];
            H[c] = t.x;
            Y[c] = t.y;
        }
        HLp = r.top[min(jl, n)].x;
    } else {
        const int2* st = r.stck + ((long long)(ck - 1) * r.nstripes + s) * (TD + 1) * 64 + lane;
#pragma unroll
        for (int c = 0; c < TD; c++) {
            const int2 v = st[c * 64];
            H[c] = v.x;
            Y[c] = v.y;
        }
        const int2 v = st[TD * 64];
        Xl = v.x;
        HLp = v.y;
    }
    int Hl = H[TD - 1];
    const unsigned op1 = (unsigned)o + 1u;
    // jump entries (as successors: a tie or a cell outside the block counts 0) of the previous step per column
    int E0p[TD], E2p[TD];
#pragma unroll
    for (int c = 0; c < TD; c++) E0p[c] = E2p[c] = 0;
    int E1last = 0, E0last = 0, E0dgn = 0;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    auto reads = [&](int g, int (&sb)[4][TD], int (&eh)[4], int (&ex)[4]) {
        const uint32_t aw = awin[t0 + g - lane - base];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int ac = (int)((aw >> (8 * u)) & 0xffu) * 32;
#pragma unroll
            for (int c = 0; c < TD; c++) sb[u][c] = stab[ac + bcode[c]];
        }
        const int4 e01 = *reinterpret_cast<const int4*>(ewin + g);
        const int4 e23 = *reinterpret_cast<const int4*>(ewin + g + 2);
        eh[0] = e01.x; eh[1] = e01.z; eh[2] = e23.x; eh[3] = e23.z;
        ex[0] = e01.y; ex[1] = e01.w; ex[2] = e23.y; ex[3] = e23.w;
    };
    // A group of 4 steps in two phases: the scores and every cell's LUT index first (a VALU chain), then the 4*TD
    // LUT loads all in flight at once, then the entries (the E chains need the selectors).  Interleaved, the
    // compiler kept two loads in flight and the block's steps waited on the LUT (44 us per C3 block).
    auto group = [&](int g, const int (&sb)[4][TD], const int (&eh)[4], const int (&ex)[4], auto MK) {
        constexpr bool MASKED = decltype(MK)::value;
        unsigned idx[4][TD];
        bool actv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int row = t0 + g + u - lane + 1;
            const bool act = !MASKED || row >= 1;
            actv[u] = act;
            int X = __builtin_amdgcn_update_dpp(ex[u], Xl, 0x138, 0xf, 0xf, false);
            const int HLn = __builtin_amdgcn_update_dpp(eh[u], Hl, 0x138, 0xf, 0xf, false);
            int Hd = HLp;
#pragma unroll
            for (int c = 0; c < TD; c++) {
                const int sw = sb[u][c];
                const int M = Hd + (int)(int8_t)(sw & 0xff);
                const int Hn = min(min(M, X), Y[c]);
                idx[u][c] = min((unsigned)(X - Hn), op1) | (min((unsigned)(Y[c] - Hn), op1) << 4) |
                            (min((unsigned)(M - Hn), 1u) << 8) | ((unsigned)sw & 0x200u);  // bit 9: a_i != b_j
                const int Ho = Hn + o;
                X = min(X, Ho);
                Y[c] = act ? min(Y[c], Ho) : Y[c];
                Hd = H[c];
                H[c] = act ? Hn : H[c];
            }
            Xl = X;
            Hl = H[TD - 1];
            HLp = HLn;
        }
        uint4 f[4][TD];
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int c = 0; c < TD; c++) f[u][c] = lut[idx[u][c]];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int row = t0 + g + u - lane + 1;
            const bool act = actv[u];
            // the left lane's last-column entries: E1 of this row (its step t-1), E0 of the row above (t-2)
            int El = __builtin_amdgcn_update_dpp(0, E1last, 0x138, 0xf, 0xf, false);
            int Ed = E0dgn;
            E0dgn = __builtin_amdgcn_update_dpp(0, E0last, 0x138, 0xf, 0xf, false);
            // the block's rows go to the stage, the others to its scratch row
            const unsigned rel = (unsigned)(row - R0 - 1);
            uint16_t* dst = stage + (rel < 64u ? rel : 64u) * SC + lane * TD;
            unsigned S01[TD], S2[TD];
#pragma unroll
            for (int c = 0; c < TD; c++) {
                const uint4 fc = f[u][c];
                const unsigned Pd = ((unsigned)Ed << 2) | 3u, Pl = ((unsigned)El << 2) | 1u,
                               Pu = ((unsigned)E2p[c] << 2) | 2u;
                const unsigned src0 = __builtin_amdgcn_perm(Pl, Pd, 0x05040100u);
                const unsigned E01 = __builtin_amdgcn_perm(src0, Pu, fc.x);
                const unsigned E2v = __builtin_amdgcn_perm(src0, Pu, fc.y);
                S01[c] = E01 | fc.z;
                S2[c] = E2v | fc.w;
                Ed = E0p[c];
                El = (int)(E01 >> 16);
                E0p[c] = act ? (int)(E01 & 0xffffu) : E0p[c];
                E2p[c] = act ? (int)E2v : E2p[c];
            }
            E1last = act ? El : 0;
            E0last = E0p[TD - 1];
            // the three levels' stored entries of this row's TD columns
            if constexpr (TD == 4) {
                typedef unsigned u2v __attribute__((ext_vector_type(2)));
                const u2v w0 = {__builtin_amdgcn_perm(S01[1], S01[0], 0x05040100u), __builtin_amdgcn_perm(S01[3], S01[2], 0x05040100u)};
                const u2v w1 = {__builtin_amdgcn_perm(S01[1], S01[0], 0x07060302u), __builtin_amdgcn_perm(S01[3], S01[2], 0x07060302u)};
                const u2v w2 = {__builtin_amdgcn_perm(S2[1], S2[0], 0x05040100u), __builtin_amdgcn_perm(S2[3], S2[2], 0x05040100u)};
                *reinterpret_cast<u2v*>(dst) = w0;
                *reinterpret_cast<u2v*>(dst + JSTAGE_ROWS * SC) = w1;
                *reinterpret_cast<u2v*>(dst + 2 * JSTAGE_ROWS * SC) = w2;
            } else if constexpr (TD == 2) {
                *reinterpret_cast<unsigned*>(dst) = __builtin_amdgcn_perm(S01[1], S01[0], 0x05040100u);
                *reinterpret_cast<unsigned*>(dst + JSTAGE_ROWS * SC) = __builtin_amdgcn_perm(S01[1], S01[0], 0x07060302u);
                *reinterpret_cast<unsigned*>(dst + 2 * JSTAGE_ROWS * SC) = __builtin_amdgcn_perm(S2[1], S2[0], 0x05040100u);
            } else {
                dst[0] = (uint16_t)S01[0];
                dst[JSTAGE_ROWS * SC] = (uint16_t)(S01[0] >> 16);
                dst[2 * JSTAGE_ROWS * SC] = (uint16_t)S2[0];
            }
        }
    };
    int sbA[4][TD], ehA[4], exA[4], sbB[4][TD], ehB[4], exB[4];
    reads(0, sbA, ehA, exA);
    const int gmask = ck == 0 ? 64 : 0;
    for (int g = 0; g < nst; g += 8) {
        reads(g + 4, sbB, ehB, exB);
        if (g < gmask) group(g, sbA, ehA, exA, std::true_type{});
        else group(g, sbA, ehA, exA, std::false_type{});
        reads(g + 8, sbA, ehA, exA);
        if (g + 4 < gmask) group(g + 4, sbB, ehB, exB, std::true_type{});
        else group(g + 4, sbB, ehB, exB, std::false_type{});
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    {
        // (the reach check of rc_block: a block the walker can no longer reach is not written)
        const unsigned pv = (unsigned)sgpr((int)g_ld(r.pos));
        const int tile = pv ? (int)(pv - 1u) : r.tile0;
        if (bi > (tile >> 16) || bs * TD > (tile & 0xffff)) return false;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slot's owner tag cleared (rc_server) before any word
    // the block's 2 x 2TD tiles of 32 x 32 cells, 6 KB each ([level][32 rows][32 columns], ga_jump.h), into its
    // cache slot with write-through stores
    uint8_t* blk = r.tb + (size_t)((bi % RC_CACHE_I) * RC_CACHE_S + bs % RC_CACHE_S) * (4 * TD * JTILE_BYTES);
#pragma unroll
    for (int tr = 0; tr < 2; tr++)
#pragma unroll
        for (int tc = 0; tc < 2 * TD; tc++) {
            uint4* dst = reinterpret_cast<uint4*>(blk + (tr * 2 * TD + tc) * JTILE_BYTES) + lane;
#pragma unroll
            for (int q = 0; q < 6; q++) {
                const int p = q >> 1, row = tr * 32 + (q & 1) * 16 + (lane >> 2), col = tc * 32 + (lane & 3) * 8;
                const uint4 v = *reinterpret_cast<const uint4*>(stage + (p * JSTAGE_ROWS + row) * SC + col);
                st16_sc1(dst + q * 64, v);
            }
        }
    return true;
}
#endif  // GA_EXPERIMENTS

template <int TD, int CB, bool JUMP = false>
__device__ void rc_server(const RcArgs& r, uint8_t* dyn) {
    const int lane = threadIdx.x & 63;
    const int wave = sgpr((int)(threadIdx.x >> 6));
    int8_t* stab = reinterpret_cast<int8_t*>(dyn);  // [K][32] sub'
    int16_t* stab16 = reinterpret_cast<int16_t*>(dyn);  // JUMP: [K][32] sub' | (a != b) << 9
    uint4* lut = reinterpret_cast<uint4*>(dyn + JLUT_OFF);
    if constexpr (JUMP) {
        for (int q = threadIdx.x; q < r.K * r.K; q += blockDim.x)
            stab16[(q / r.K) * 32 + q % r.K] = (int16_t)((r.subp[q] & 0xff) | (q / r.K != q % r.K ? 0x200 : 0));
        for (int q = threadIdx.x; q < 1024; q += blockDim.x) lut[q] = r.jlut[q];  // built by the host (jump_lut_build)
    } else {
        for (int q = threadIdx.x; q < r.K * r.K; q += blockDim.x) stab[(q / r.K) * 32 + q % r.K] = (int8_t)r.subp[q];
    }
    __syncthreads();
    if (wave >= r.workers) return;
    uint8_t* wl = dyn + (JUMP ? JWORK_OFF : 1024) + wave * r.worker_bytes;
    const unsigned claimed = 2u * r.epoch, ready = claimed + 1u;
    const int dbi = r.off[lane] >> 3, dbs = r.off[lane] & 7;
    unsigned idle = 0, nblk = 0;
    for (;;) {
        if (sgpr((int)g_ld(r.pos + 1))) break;  // the walk has ended
        const unsigned pv = (unsigned)sgpr((int)g_ld(r.pos));
        const int tile = pv ? (int)(pv - 1u) : r.tile0;
        const int BI = tile >> 16, BS = (tile & 0xffff) / TD;
        const int bi = BI - dbi, bs = BS - dbs;
        const bool valid = lane < r.nwin && bi >= 0 && bs >= 0 && bi < r.nbi && bs < r.nbs;
        unsigned* fl = r.flags + (long long)(valid ? bi : 0) * r.nbs + (valid ? bs : 0);
        const unsigned st = valid ? g_ld(fl) : ready;
        unsigned long long freem = __ballot(valid && st < claimed);
        bool did = false;
        while (freem && !did) {
            // the likeliest free block first (the window is in priority order); a lost claim tries the next
            const int i = __builtin_ctzll(freem);
            const int bi_i = __builtin_amdgcn_readlane(bi, i), bs_i = __builtin_amdgcn_readlane(bs, i);
            unsigned exp = (unsigned)__builtin_amdgcn_readlane((int)st, i);
            int won = 0;
            if (lane == 0)
                won = __hip_atomic_compare_exchange_strong(r.flags + (long long)bi_i * r.nbs + bs_i, &exp, claimed,
                                                           __ATOMIC_RELAXED, __ATOMIC_RELAXED, AGENT);
            if (sgpr(won)) {
                const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
                // the slot's words are about to change: its owner tag cleared first (ga::rc_slot_tag)
                unsigned long long* const own = r.own + rc_slot(bi_i, bs_i);
                if (lane == 0) __hip_atomic_store(own, 0ull, RLX, AGENT);
                bool wrote;
#ifdef GA_EXPERIMENTS
                if constexpr (JUMP) wrote = rc_block_jump<TD>(r, stab16, lut, wl, bi_i, bs_i, lane);
                else
#endif
                    wrote = rc_block<TD, CB>(r, stab, wl, bi_i, bs_i, lane);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every word written before the tag
                // (GA_RC_TAG_FAULT: a lost tag, which the walk's loaders must repair through a recompute)
                const bool fault = r.tag_fault > 0 && ++nblk % (unsigned)r.tag_fault == 0;
                if (lane == 0 && wrote && !fault) __hip_atomic_store(own, rc_slot_tag(bi_i, bs_i, r.nbs, ready), RLX, AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tag before the flag
                if (lane == 0) g_st(r.flags + (long long)bi_i * r.nbs + bs_i, ready);
                if (lane == 0) {  // diagnostics: blocks recomputed, their total time (100 MHz ticks)
                    atomicAdd(r.pos + 2, 1u);
                    atomicAdd(r.pos + 3, (unsigned)(__builtin_amdgcn_s_memrealtime() - c0));
                }
                did = true;
            }
            freem &= ~(1ull << i);
        }
        if (did) {
            idle = 0;
            continue;
        }
        if (++idle > r.spin_limit) break;  // the walk's own bounded tile wait reports the failure
        __builtin_amdgcn_s_sleep(4);
    }
}

template <int CB, int TD>
__global__ void __launch_bounds__(64 * WALK_WAVES) walk_rc_kernel(WalkArgs w, RcArgs r) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    if (blockIdx.x == 0) walk_body<CB, true>(w, w.rng, reinterpret_cast<uint16_t*>(dyn));
    else rc_server<TD, CB>(r, dyn);
}

#ifdef GA_EXPERIMENTS
// the tie-to-tie walk: workgroup 0 walks with jump entries, the others build them
template <int TD>
__global__ void __launch_bounds__(64 * JWALK_WAVES) walk_rc_jump_kernel(WalkArgs w, RcArgs r) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    if (blockIdx.x == 0) walk_jump_body(w, w.rng, reinterpret_cast<uint16_t*>(dyn));
    else rc_server<TD, 1, true>(r, dyn);
}

template <int TD>
static void launch_rc_jump_one(hipStream_t s, const WalkArgs& w, const RcArgs& r, int nserv) {
    const size_t lds = std::max<size_t>(jump_torus_bytes(), (size_t)JWORK_OFF + (size_t)r.workers * r.worker_bytes);
    auto* fn = walk_rc_jump_kernel<TD>;
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fn<<<dim3(1 + nserv), dim3(64 * JWALK_WAVES), lds, s>>>(w, r);
}

int rc_jump_worker_bytes_host(int TD, int every) { return rc_jump_worker_bytes(TD, every); }
size_t rc_jump_lds_bytes(int TD, int every) { return (size_t)JWORK_OFF + (size_t)rc_jump_worker_bytes(TD, every); }

void launch_walk_rc_jump(hipStream_t s, const WalkArgs& w, const RcArgs& r, int nserv) {
    switch (r.TD) {
        case 1: launch_rc_jump_one<1>(s, w, r, nserv); break;
        case 2: launch_rc_jump_one<2>(s, w, r, nserv); break;
        default: launch_rc_jump_one<4>(s, w, r, nserv); break;
    }
}
#endif  // GA_EXPERIMENTS

template <int CB, int TD>
static void launch_rc_one(hipStream_t s, const WalkArgs& w, const RcArgs& r, int nserv) {
    const size_t lds = std::max<size_t>((size_t)TP * TP * sizeof(uint16_t), 1024 + (size_t)r.workers * r.worker_bytes);
    auto* fn = walk_rc_kernel<CB, TD>;
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fn<<<dim3(1 + nserv), dim3(64 * WALK_WAVES), lds, s>>>(w, r);
}

template <int CB>
static void launch_rc_cb(hipStream_t s, const WalkArgs& w, const RcArgs& r, int nserv) {
    switch (r.TD) {
        case 1: launch_rc_one<CB, 1>(s, w, r, nserv); break;
        case 2: launch_rc_one<CB, 2>(s, w, r, nserv); break;
        case 4: launch_rc_one<CB, 4>(s, w, r, nserv); break;
        default: launch_rc_one<CB, 8>(s, w, r, nserv); break;
    }
}

void launch_walk_rc(hipStream_t s, const WalkArgs& w, const RcArgs& r, int nserv) {
    if (w.CB == 1) launch_rc_cb<1>(s, w, r, nserv);
    else if (w.CB == 2) launch_rc_cb<2>(s, w, r, nserv);
    else launch_rc_cb<4>(s, w, r, nserv);
}

}  // namespace ga
