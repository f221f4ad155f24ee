// ga_walk.h -- the traceback walk (dp_array_backward, globaligner.py:395-593): tile decode, the
// walker / loader / helper roles of one workgroup (walk_body), walk_kernel and walk_chain_kernel.
// Included by ga_kernels.hip and by ga_rcwalk.hip (the walk beside the tile recompute).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ga_device.h"
#include "ga_sync.h"

namespace ga {

// ----------------------------------------------------------------------------------
// Traceback walk (dp_array_backward, globaligner.py:395-593).
//
// One workgroup of twelve waves.  Nine loader waves keep a 4x4 direct-mapped
// cache of decoded 64x64 tiles (tile = 64 rows x one 64-column stripe) filled
// ahead of the walker: the path is monotone (up/left), so the tiles it can
// reach next are the 4x4 block above-left of its current tile.  The cache is a
// 256x256 torus: cell (i, j) lives at ((i-1) mod 256, (j-1) mod 256), so every
// tile of that block has its own place and any 8x8 window is two masks.
// Wave 4 streams the host's tie-break table into an LDS ring and the chosen
// levels back to HBM; wave 8 idles so the walker (wave 0) shares its SIMD with
// the mostly-sleeping helper only.
//
// A cached cell is a u16 of three 5-bit shifts, one per entering level L:
// sh_L = 2*S_L - 2 + 14*(a_i != b_j), S_L (1..7) the rank set of sets_from_code.
// The host table entry of dispatch D holds, at bits sh+3..sh+4, the level the
// reference's random.choice picks for that set (match half at 2S+1, mismatch
// half at 15+2S), so a step's level comes out already times 8 (the bit offset
// of the next entering level's field): L8 = (tab >> sh_L) & 0x18.
//
// Wave 0 walks with scalar code only, in groups of 4 steps: each group issues
// the LDS read of the 8x8 window anchored at its first cell (lane r*8+c =
// cell (i-r, j-c), fields widened to bits 0/8/16) for the NEXT group -- a
// window anchored at p covers every cell reachable from p in 7 steps -- and
// each step reads its cell with v_readlane.  Four groups make an iteration of
// 16 steps that runs without a single check when the walk is far from the
// matrix edge and inside the tiles verified cached.  Chosen levels are packed
// 2 bits per dispatch: dispatch D at bits 30 - 2*(D & 15) of u32 word D >> 4.
// Degenerate walks (the walk visits row 0 / column 0 and wraps
// with Python negative indexing) run a slower per-step path reproduced cell by
// cell from HBM.

__device__ __forceinline__ int argmin3(long long x, long long y, long long z) {
    long long h = x < y ? x : y;
    h = h < z ? h : z;
    return (x == h) | ((y == h) << 1) | ((z == h) << 2);
}

// rank sets of an interior cell from its traceback word
__device__ __forceinline__ int sets_from_code(unsigned code, int CB, int o) {
    const int W = (8 * CB - 1) / 2;
    const unsigned fm = (1u << W) - 1u;
    const unsigned sX = code & fm, sY = (code >> W) & fm;
    const unsigned zM = ((code >> (2 * W)) & 1u) ^ 1u;
    const unsigned uo = (unsigned)o;
    const unsigned zX = sX == 0, zY = sY == 0;
    const unsigned leX = sX <= uo, geX = sX >= uo, leY = sY <= uo, geY = sY >= uo;
    const unsigned S0 = zM | (zX << 1) | (zY << 2);
    const unsigned S1 = (zM & geX) | (leX << 1) | ((zY & geX) << 2);
    const unsigned S2 = (zM & geY) | ((zX & geY) << 1) | (leY << 2);
    return (int)(S0 | (S1 << 3) | (S2 << 6));
}

// three 5-bit table shifts (one per entering level) from the rank sets and a_i == b_j
// (every walked cell has three non-empty sets; an empty one -- cells outside the matrix, never
// walked -- borrows from the next field, which is then garbage nobody reads)
__device__ __forceinline__ unsigned cell_shifts(int sets, bool am) {
    const unsigned u = (unsigned)sets;
    const unsigned s2 = ((u & 7u) | ((u & 0x38u) << 2) | ((u & 0x1c0u) << 4)) << 1;  // 2*S_L at bits 0/5/10
    return s2 + (am ? 0u - 2u * 0x421u : 12u * 0x421u);                            // + (mm - 2) per field
}

__device__ __forceinline__ unsigned tb_code(const uint8_t* tb, int CB, int TC, int i, int j) {
    const int s = (j - 1) >> 6, l = (j - 1) & 63, t = i - 1;
    const int spc = 16 / CB;
    const uint8_t* p = tb + (((long long)s * TC + t / spc) * 64 + l) * 16 + (t % spc) * CB;
    unsigned v = p[0];
    if (CB >= 2) v |= (unsigned)p[1] << 8;
    if (CB == 4) v |= ((unsigned)p[2] << 16) | ((unsigned)p[3] << 24);
    return v;
}


constexpr int TT = 64;       // tile edge
constexpr int TB4 = 4;       // tile block edge (tiles cached per axis)
constexpr int TP = TB4 * TT; // torus pitch (256)
constexpr int NSLOT = TB4 * TB4;

__device__ __forceinline__ int slot_of(int ti, int tj) { return (ti & (TB4 - 1)) * TB4 + (tj & (TB4 - 1)); }
__device__ __forceinline__ int torus_of(int i, int j) { return ((i - 1) & (TP - 1)) * TP + ((j - 1) & (TP - 1)); }

// Four 16-byte traceback words of a lane, 1 KiB apart (one 64-row tile of a column at one byte per cell), as
// write-through-coherent (sc1) loads: the recompute walk's tiles are written by other workgroups of the
// same launch with sc1 stores (ga_rcwalk.hip; MI355X_MICROARCH.md, inter-workgroup visibility)
typedef unsigned wk_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ld4_sc1(const uint4* p, uint4 (&ch)[4]) {
    wk_u4 c0, c1, c2, c3;
    asm volatile(
        "global_load_dwordx4 %0, %4, off sc1\n\t"
        "global_load_dwordx4 %1, %4, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %2, %4, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %3, %4, off offset:3072 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
        : "v"(p)
        : "memory");
    ch[0] = make_uint4(c0.x, c0.y, c0.z, c0.w);
    ch[1] = make_uint4(c1.x, c1.y, c1.z, c1.w);
    ch[2] = make_uint4(c2.x, c2.y, c2.z, c2.w);
    ch[3] = make_uint4(c3.x, c3.y, c3.z, c3.w);
}

// One loader wave decodes tile (ti, tj) into the torus: lane = column; the
// tile's 64 rows of a column are 64/SPC whole 16-byte words of its stripe's
// traceback stream (the general path; one-byte words use load_tile_b1).
template <int CB, bool RC = false>
__device__ void load_tile(const WalkArgs& w, int ti, int tj, uint16_t* torus, uint8_t* sa, const uint16_t* lut,
                          const uint8_t* lutF, int lane) {
    uint16_t* dst = torus + (ti & (TB4 - 1)) * TT * TP + (tj & (TB4 - 1)) * TT;
    constexpr int SPC = 16 / CB;
    constexpr int KW = TT / SPC;
    const int i0 = ti * TT + 1;                       // first row of the tile
    const int j = tj * TT + lane + 1;                 // this lane's column
    sa[lane] = (i0 + lane <= w.m) ? w.a[i0 + lane - 1] : 0xff;
    const bool colok = j <= w.n;
    const int bj = colok ? w.b[j - 1] : 0xfe;
    // RC: the recompute walk's tile cache (ga_rcwalk.hip): block row ti mod RC_CACHE_I, fill stripe tj / td mod RC_CACHE_S
    const int tic = RC ? ti % RC_CACHE_I : ti, tjc = RC ? ((tj / w.rc_td) % RC_CACHE_S) * w.rc_td + tj % w.rc_td : tj;
    const uint4* base = reinterpret_cast<const uint4*>(w.tb) + ((long long)tjc * w.TC + tic * KW) * 64 + lane;
    const int nq = min(KW, w.TC - ti * KW);
    uint4 ch[KW];
    if constexpr (RC) {
        // whole 1 KiB runs, 4 per call (the recompute walk's buffer has a tile of slack past its end)
#pragma unroll
        for (int k = 0; k < KW; k += 4) {
            uint4 c4[4];
            ld4_sc1(base + (long long)k * 64, c4);
#pragma unroll
            for (int u = 0; u < 4 && k + u < KW; u++) ch[k + u] = c4[u];
        }
    } else {
#pragma unroll
        for (int k = 0; k < KW; k++) ch[k] = (colok && k < nq) ? base[(long long)k * 64] : make_uint4(0, 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): sa[] visible to this wave
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < KW; k++) {
        const unsigned wd[4] = {ch[k].x, ch[k].y, ch[k].z, ch[k].w};
#pragma unroll
        for (int u = 0; u < SPC; u++) {
            const int r = k * SPC + u;   // tile row
            unsigned code = wd[(u * CB) >> 2] >> ((u * CB * 8) & 31);
            if (CB == 1) code &= 0xffu;
            else if (CB == 2) code &= 0xffffu;
            if constexpr (CB == 2) {
                // two-byte words: each 7-bit field's (== 0, <= o, >= o) flags from lutF, the three
                // levels' shifts from lut (zM bit, both fields' flags, a_i == b_j): the general decode
                // below made the C5 walk wait on tile loads (9.7 us a tile)
                const unsigned idx = ((code >> 14) & 1u) | ((unsigned)lutF[code & 127u] << 1) |
                                     ((unsigned)lutF[(code >> 7) & 127u] << 4) | (sa[r] == bj ? 128u : 0u);
                dst[r * TP + lane] = lut[idx];
            } else {
                dst[r * TP + lane] = (uint16_t)cell_shifts(sets_from_code(code, CB, w.o), sa[r] == bj);
            }
        }
    }
}

// One-byte traceback words (the common case, gap open < 7): branch-free decode.
// A lane's 64 cells are its four 16-byte words; it folds a_i == b_j into bit 7
// of each word (SWAR zero-byte test on the staged a bytes; words use bits 0-6)
// and decodes through a 256-entry table.
template <bool RC = false>
__device__ inline void load_tile_b1(const WalkArgs& w, int ti, int tj, uint16_t* torus, uint8_t* sa, const uint16_t* lut,
                                    int lane) {
    uint16_t* dst = torus + (ti & (TB4 - 1)) * TT * TP + (tj & (TB4 - 1)) * TT + lane;
    const int i0 = ti * TT + 1;
    const int j = tj * TT + lane + 1;
    sa[lane] = (i0 + lane <= w.m) ? w.a[i0 + lane - 1] : 0xff;
    const bool colok = j <= w.n;
    const unsigned bj = colok ? w.b[j - 1] : 0xfeu;
    const int tic = RC ? ti % RC_CACHE_I : ti, tjc = RC ? ((tj / w.rc_td) % RC_CACHE_S) * w.rc_td + tj % w.rc_td : tj;
    const uint4* base = reinterpret_cast<const uint4*>(w.tb) + ((long long)tjc * w.TC + tic * 4) * 64 + lane;
    const int nq = w.TC - ti * 4;
    unsigned wv[16];
    if constexpr (RC) {
        uint4 c4[4];
        ld4_sc1(base, c4);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            wv[4 * k] = c4[k].x; wv[4 * k + 1] = c4[k].y; wv[4 * k + 2] = c4[k].z; wv[4 * k + 3] = c4[k].w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 c = (colok && k < nq) ? base[(long long)k * 64] : make_uint4(0, 0, 0, 0);
            wv[4 * k] = c.x; wv[4 * k + 1] = c.y; wv[4 * k + 2] = c.z; wv[4 * k + 3] = c.w;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): sa[] visible to this wave
    __builtin_amdgcn_wave_barrier();
    const uint4* sa4 = reinterpret_cast<const uint4*>(sa);
    unsigned av[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint4 x = sa4[k];
        av[4 * k] = x.x; av[4 * k + 1] = x.y; av[4 * k + 2] = x.z; av[4 * k + 3] = x.w;
    }
    const unsigned bj4 = bj * 0x01010101u;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const unsigned x = av[k] ^ bj4;
        const unsigned t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;      // bit 7 of a byte clear <=> byte == 0
        const unsigned cw = (wv[k] & 0x7f7f7f7fu) | (~t & 0x80808080u);
#pragma unroll
        for (int u = 0; u < 4; u++) dst[(4 * k + u) * TP] = lut[(cw >> (8 * u)) & 0xffu];
    }
}

constexpr int RB = 2048;
constexpr int WALK_DBG = 8192;  // tile-need records kept by the diagnostic walk  // LDS rings of tie-break entries / chosen levels (4 blocks of 512 dispatches)

__device__ __forceinline__ int sgpr(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Waves: 0 walker, 4 ring helper, the other fourteen load tiles (WalkArgs::nloaders = 14; with 12,
// wave 8 is an L2 prefetcher and wave 12 idles, the walker's SIMD running nothing busy).
constexpr int WALK_WAVES = 16;
constexpr int NLOAD_MAX = 14;  // loader waves: 12 (default), 13 (+ the idle wave), 14 (+ the prefetcher's)

// The recompute walk's cache slot check (ga::rc_slot_tag): true while block (bi, bs)'s words are in its
// slot.  A loader asks before it copies a tile (pre) and after the copy has landed; it uses the copy only if both
// say so.  Before a copy, a block whose flag says ready although its slot's tag differs (the tag is set before the
// flag, and the second tag read below is issued after the flag read returned) lost its words to another block's
// worker: its flag is reset, so a worker recomputes it.
__device__ inline bool rc_slot_ok(const WalkArgs& w, int bi, int bs, bool pre) {
    unsigned long long* const own = w.rc_own + rc_slot(bi, bs);
    const unsigned long long want = rc_slot_tag(bi, bs, w.rc_nbs, w.rc_ready);
    auto tag = [&]() {
        const unsigned long long t = __hip_atomic_load(own, RLX, AGENT);
        return ((unsigned long long)sgpr_u((unsigned)(t >> 32)) << 32) | sgpr_u((unsigned)t);
    };
    if (!pre) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the copy's loads have returned
    if (tag() == want) return true;
    if (!pre) return false;  // the next poll decides
    unsigned* const fl = w.rc_flags + (long long)bi * w.rc_nbs + bs;
    if (sgpr_u(g_ld(fl)) == w.rc_ready && tag() != want && (threadIdx.x & 63) == 0) {
        unsigned e = w.rc_ready;
        __hip_atomic_compare_exchange_strong(fl, &e, 0u, RLX, RLX, AGENT);
    }
    return false;
}

__device__ __forceinline__ bool in_block(int cur, int ti, int tj) {
    const int dti = (cur >> 16) - ti, dtj = (cur & 0xffff) - tj;
    return cur >= 0 && dti >= 0 && dti < TB4 && dtj >= 0 && dtj < TB4;
}

// One walk by the whole workgroup (every wave returns from here once its role is done): the body of
// walk_kernel, and of walk_chain_kernel once per alignment.  It initialises all of its LDS state.
// torus: TP x TP u16 of LDS (the kernel's).  RC: the recompute walk (ga_rcwalk.hip): a tile
// is loaded only once its block's flag says another workgroup has written its words (sc1 loads), the
// helper publishes the walker's tile for those workgroups, and every tile wait is bounded.
// SLD: the interior walk reads its tie-break entries with scalar loads straight from rng (device memory),
// a group ahead, instead of from the helper's LDS ring (one ds_read and four readfirstlanes per group);
// walk_chain_kernel's entries are in pinned host memory and keep the ring
template <int CB, bool RC = false, bool SLD = true>
__device__ __forceinline__ void walk_body(const WalkArgs& w, const uint32_t* rng, uint16_t* torus) {
    // the thread index through an opaque copy: in walk_chain_kernel nothing derived from it is hoisted
    // out of the loop over walks (it would stay live in VGPRs across every role's code)
    unsigned tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    __shared__ __attribute__((aligned(16))) uint32_t rngbuf[RB];
    __shared__ uint32_t opsbuf[RB / 16];
    __shared__ uint32_t ops_dummy;  // where the walker's deferred level-word store goes when none is pending
    __shared__ uint16_t lut[256];
    __shared__ uint8_t lutF[128];
    __shared__ __attribute__((aligned(16))) uint8_t sa[NLOAD_MAX][TT];
    __shared__ int tag[NSLOT];
    __shared__ int rtag[4];
    __shared__ int cur_tile, walk_done, wD, ops_flushed, rc_timeout;
    __shared__ unsigned long long load_ticks;
    __shared__ int load_count;
    const int lane = tid & 63;
    const int wave = sgpr(tid >> 6);
    const int m = w.m, n = w.n, o = w.o;
    if (tid == 0) { load_ticks = 0; load_count = 0; }
    if (tid < NSLOT) tag[tid] = -1;
    if (tid < 4) rtag[tid] = -1;
    // a slab walk starts at dispatch D0: the rings start at its block
    if (tid == 0) { cur_tile = -1; walk_done = 0; wD = w.D0; ops_flushed = w.D0 >> 9; rc_timeout = 0; }
    if (CB == 1 && tid < 256)
        lut[tid] = (uint16_t)cell_shifts(sets_from_code(tid & 127u, 1, o), (tid >> 7) != 0);
    if (CB == 2 && tid < 128) {
        const int v = (int)tid;
        lutF[v] = (uint8_t)((v == 0) | ((v <= o) << 1) | ((v >= o) << 2));
    }
    if (CB == 2 && tid < 256) {
        // sets_from_code in terms of the flags: bit 0 the raw zM bit, bits 1-3 / 4-6 the (zero, le, ge)
        // flags of the X / Y fields, bit 7 a_i == b_j
        const unsigned x = tid;
        const unsigned zM = (x & 1u) ^ 1u, zX = (x >> 1) & 1u, leX = (x >> 2) & 1u, geX = (x >> 3) & 1u;
        const unsigned zY = (x >> 4) & 1u, leY = (x >> 5) & 1u, geY = (x >> 6) & 1u;
        const unsigned S0 = zM | (zX << 1) | (zY << 2);
        const unsigned S1 = (zM & geX) | (leX << 1) | ((zY & geX) << 2);
        const unsigned S2 = (zM & geY) | ((zX & geY) << 1) | (leY << 2);
        lut[x] = (uint16_t)cell_shifts((int)(S0 | (S1 << 3) | (S2 << 6)), (x >> 7) != 0);
    }
    __syncthreads();

    // loader waves (WalkArgs::nloaders): 12, or 13 with wave 12, or 14 with wave 8 too (no prefetcher)
    const int nload = w.nloaders >= 12 && w.nloaders <= NLOAD_MAX ? w.nloaders : 12;
    const bool prefetch = nload < 14, idle12 = nload < 13;
    if (RC && wave == 8 && prefetch) return;  // the recompute walk's words may not be written yet: no prefetch
    if (wave == 8 && prefetch) {
        // ---------------- L2 prefetcher: touches the ring of tiles just beyond the loaders'
        // 4x4 block (offsets with i+j distance 4..6, each <= 4), so their HBM fetch is
        // done by the time the block reaches them.  Low priority: it shares the walker's SIMD.
        __builtin_amdgcn_s_setprio(0);
        const uint4* tbw = reinterpret_cast<const uint4*>(w.tb);
        const int nti = (w.m + TT - 1) / TT, ntj = (w.n + TT - 1) / TT;
        int last = -2;
        unsigned sink = 0;
        while (!sgpr(__hip_atomic_load(&walk_done, __ATOMIC_ACQUIRE, WGS))) {
            const int cur = sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_ACQUIRE, WGS));
            if (cur < 0 || cur == last) {
                __builtin_amdgcn_s_sleep(4);
                continue;
            }
            last = cur;
            const int ti = cur >> 16, tj = cur & 0xffff;
            for (int d = 4; d <= 6; d++)
                for (int di = max(0, d - 4); di <= min(4, d); di++) {
                    const int pti = ti - di, ptj = tj - (d - di);
                    if (pti < 0 || ptj < 0 || pti >= nti || ptj >= ntj) continue;
                    const uint4* base = tbw + ((long long)ptj * w.TC + pti * (TT * CB / 16)) * 64 + lane;
                    const int nq = min(TT * CB / 16, w.TC - pti * (TT * CB / 16));
                    for (int k = 0; k < nq; k++) sink ^= base[(long long)k * 64].x;
                }
        }
        if (sink == 0x9e3779b9u) w.result[15] = (int)sink;  // keeps the loads
        return;
    }
    if (wave == 4) {
        // ---------------- helper: tie-break table HBM -> LDS ring, levels LDS ring -> HBM ----------------
        const long long nblk = (w.nrng + 511) / 512;
        long long rl = w.D0 >> 9, fl = w.D0 >> 9;
        int pub = -1;  // RC: the walker's tile last published for the recompute workgroups
        for (;;) {
            // done first: the walker stores its final dispatch count before walk_done, so once done is seen
            // d is final (read the other way round, a stale d beside done = 1 dropped the last levels)
            const int done = sgpr(__hip_atomic_load(&walk_done, __ATOMIC_ACQUIRE, WGS));
            const int d = sgpr(__hip_atomic_load(&wD, __ATOMIC_ACQUIRE, WGS));
            bool moved = false;
            if constexpr (RC) {
                const int cur = sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_ACQUIRE, WGS));
                if (cur >= 0 && cur != pub) {
                    if (lane == 0) g_st(w.rc_pos, (unsigned)cur + 1u);  // 0: not yet published
                    pub = cur;
                }
            }
            while (rl < nblk && rl < (d >> 9) + 4) {
                const long long e0 = rl * 512 + lane * 8;
                uint32_t* dst = rngbuf + (rl & 3) * 512 + lane * 8;
#pragma unroll
                for (int k = 0; k < 8; k++) dst[k] = (e0 + k < w.nrng) ? rng[e0 + k] : 0u;
                if (lane == 0) __hip_atomic_store(&rtag[rl & 3], (int)rl, __ATOMIC_RELEASE, WGS);
                rl++;
                moved = true;
            }
            const long long complete = done ? ((long long)d + 511) / 512 : (d >> 9);
            const long long fl0 = fl;
            while (fl < complete) {  // 512 dispatches = 32 words of levels
                if (lane < 32) {
                    const uint32_t v = opsbuf[(fl & 3) * 32 + lane];
                    // host-polled levels (ops_prog): write-through system-scope stores, like a halo's rows
                    if (w.ops_prog != nullptr) __hip_atomic_store(w.ops + fl * 32 + lane, v, RLX, __HIP_MEMORY_SCOPE_SYSTEM);
                    else w.ops[fl * 32 + lane] = v;
                }
                fl++;
                if (lane == 0) __hip_atomic_store(&ops_flushed, (int)fl, __ATOMIC_RELEASE, WGS);
                moved = true;
            }
            if (w.ops_prog != nullptr && fl > fl0) {
                // the host's decode may run up to here: whole blocks while walking, every dispatch at the end.
                // The level stores complete first (a release fence alone left a block stale on the host: its
                // L2 write-back was not awaited before the progress store, tools/exp/r3_dec.sh)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0)
                    __hip_atomic_store(w.ops_prog, done ? (unsigned)d : (unsigned)(fl * 512), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (done && fl >= complete) break;
            if (!moved) __builtin_amdgcn_s_sleep(RC ? 2 : 8);
        }
        if (RC && lane == 0) g_st(w.rc_pos + 1, 1u);  // the recompute workgroups may end
        return;
    }

    if (wave > 0) {
        // ---------------- loader pool: slot ownership ----------------
        // Loader k (k < 12) owns torus slot k, loaders 0..3 also slot k+12: each slot has one
        // writer, so no claim protocol is needed, and the tiles the walker needs next (offsets
        // (1,0), (0,1), (1,1) of its tile) sit in different slots.
        // Before overwriting a slot the owner invalidates its tag and re-reads the current tile:
        // a tile the walker may still read (inside its 4x4 block) is never overwritten, since
        // the walker publishes its tile before it checks a tag.
        if (wave == 12 && idle12) return;
        const int li = wave - 1 - (wave > 4) - (prefetch && wave > 8) - (idle12 && wave > 12);  // 0 .. nload-1
        const int nown = li < NSLOT - nload ? 2 : 1;
        while (!sgpr(__hip_atomic_load(&walk_done, __ATOMIC_ACQUIRE, WGS))) {
            const int cur = sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_ACQUIRE, WGS));
            bool did = false;
            if (cur >= 0) {
                const int ti = cur >> 16, tj = cur & 0xffff;
                // the block tile of each owned slot (the one congruent to it, at offsets 0..3)
                int cand[2] = {-1, -1}, dist[2] = {1 << 20, 1 << 20};
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    if (q >= nown) break;
                    const int sl = li + nload * q, sr = sl >> 2, sc = sl & 3;
                    const int di = (ti - sr) & (TB4 - 1), dj = (tj - sc) & (TB4 - 1);
                    cand[q] = (ti - di < 0 || tj - dj < 0) ? -1 : (((ti - di) << 16) | (tj - dj));
                    {
                        // speculative tiles far off the diagonal are left out (walk paths run near-diagonal):
                        // 1: offsets (3,0) (0,3) (3,1) (1,3); 2: also (2,0) (0,2); 3: also (3,2) (2,3)
                        const int sk = w.skip_corners, ad = abs(di - dj), mx = max(di, dj);
                        if ((sk >= 1 && mx == TB4 - 1 && ad >= 2) || (sk >= 2 && ad >= 2) || (sk >= 3 && mx == TB4 - 1 && ad >= 1))
                            cand[q] = -1;
                    }
                    dist[q] = di + dj;
                }
                const int first_q = dist[1] < dist[0] ? 1 : 0;
                for (int qq = 0; qq < 2 && !did; qq++) {
                    const int q = qq ^ first_q;
                    const int tg = cand[q];
                    if (tg < 0) continue;
                    const int sl = li + nload * q, tti = tg >> 16, ttj = tg & 0xffff;
                    if (sgpr(__hip_atomic_load(&tag[sl], __ATOMIC_RELAXED, WGS)) == tg) continue;
                    // RC: only once the tile's block has been recomputed (its words are then in its cache slot)
                    if (RC && !rc_slot_ok(w, tti, ttj / w.rc_td, true)) continue;
                    if (lane == 0) __hip_atomic_store(&tag[sl], -1, __ATOMIC_SEQ_CST, WGS);
                    if (!in_block(sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_SEQ_CST, WGS)), tti, ttj)) continue;
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    if (CB == 1) load_tile_b1<RC>(w, tti, ttj, torus, sa[li], lut, lane);
                    else load_tile<CB, RC>(w, tti, ttj, torus, sa[li], lut, lutF, lane);
                    if (RC && !rc_slot_ok(w, tti, ttj / w.rc_td, false)) continue;  // its slot changed under the copy
                    if (lane == 0) {
                        atomicAdd(&load_ticks, __builtin_amdgcn_s_memrealtime() - t0);
                        atomicAdd(&load_count, 1);
                    }
                    if (lane == 0 && in_block(sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_SEQ_CST, WGS)), tti, ttj))
                        __hip_atomic_store(&tag[sl], tg, __ATOMIC_RELEASE, WGS);
                    did = true;
                }
            }
            if (!did) __builtin_amdgcn_s_sleep(1);
        }
        return;
    }

    // ---------------- walker wave (its loop touches LDS only) ----------------
    __builtin_amdgcn_s_setprio(3);
    int i = w.i0, j = w.j0, L = w.L0, D = w.D0, h = w.h0, first = w.first0, reason = -1;
    const int jend = w.handoff ? 5 : 2;  // reason when the walk reaches local column 0
    const int iend = w.vhandoff ? 6 : 1;  // ... and local row 0 (a traceback band with rows above it)
    int cti = -1, ctj = -1, nwait = 0, ntiles = 0, ndbg = 0;
    unsigned rc_spins = 0;
    bool rc_degenerate = false;
    const int maxh = w.maxh;
    unsigned long long t_tile = 0, t_ring = 0;  // time spent waiting (s_memrealtime ticks, 100 MHz)
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c_start = __builtin_amdgcn_s_memtime();
    // make tile (ti, tj) current for the loaders (publish) and wait until it is cached
    auto need_tile = [&](int ti, int tj, bool publish) {
        const int tg = (ti << 16) | tj;
        if (publish && lane == 0) __hip_atomic_store(&cur_tile, tg, __ATOMIC_SEQ_CST, WGS);
        const int sl = slot_of(ti, tj);
        if (sgpr(__hip_atomic_load(&tag[sl], __ATOMIC_SEQ_CST, WGS)) == tg) return;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (sgpr(__hip_atomic_load(&tag[sl], __ATOMIC_ACQUIRE, WGS)) != tg) {
            __builtin_amdgcn_s_sleep(1);
            nwait++;
            // RC: a tile that never comes (no recompute workgroup running) ends the walk on garbage with
            // reason 7 instead of hanging; the host reports it
            if (RC && ++rc_spins > (1u << 25)) {
                rc_timeout = 1;
                break;
            }
        }
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
        t_tile += dt;
        if (w.dbg != nullptr && lane == 0 && ndbg < WALK_DBG) {
            w.dbg[4 * ndbg] = (unsigned)ti; w.dbg[4 * ndbg + 1] = (unsigned)tj;
            w.dbg[4 * ndbg + 2] = (unsigned)D; w.dbg[4 * ndbg + 3] = (unsigned)dt;
        }
        ndbg++;
    };
    // a new block of 512 dispatches: the level slot it reuses (block - 4) must be flushed
    auto block_start = [&](int d) {
        const int blk = d >> 9;
        if (lane == 0) __hip_atomic_store(&wD, d, __ATOMIC_RELEASE, WGS);
        if (sgpr(__hip_atomic_load(&ops_flushed, __ATOMIC_ACQUIRE, WGS)) >= blk - 3) return;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (sgpr(__hip_atomic_load(&ops_flushed, __ATOMIC_ACQUIRE, WGS)) < blk - 3) __builtin_amdgcn_s_sleep(1);
        t_ring += __builtin_amdgcn_s_memrealtime() - t0;
    };
    auto rng_ready = [&](int d) {
        const int blk = d >> 9;
        if (sgpr(__hip_atomic_load(&rtag[blk & 3], __ATOMIC_ACQUIRE, WGS)) == blk) return;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (sgpr(__hip_atomic_load(&rtag[blk & 3], __ATOMIC_ACQUIRE, WGS)) != blk) __builtin_amdgcn_s_sleep(1);
        t_ring += __builtin_amdgcn_s_memrealtime() - t0;
    };
    // the byte of the level word that holds dispatches 4*(d/4) .. +3 (little-endian u32 words)
    auto ops_byte = [&](int d) -> uint8_t* {
        return reinterpret_cast<uint8_t*>(opsbuf) + (((d >> 4) & (RB / 16 - 1)) * 4 + 3 - ((d >> 2) & 3));
    };

    // ---- per-step path: the first moves, and degenerate walks, until the walk is in the
    //      interior at a dispatch count that is a multiple of 16 ----
    if (D & 3) *ops_byte(D) = 0;  // a slab walk may start inside a byte
    rng_ready(D);                  // ... and inside a block of entries
    for (;;) {
        if (!first && i >= 1 && j >= 1 && (D & 15) == 0) break;
        if ((D & 511) == 0) {
            block_start(D);
            rng_ready(D);
        }
        const unsigned tab = (unsigned)sgpr((int)rngbuf[D & (RB - 1)]);
        unsigned sh;
        if (i >= 1 && j >= 1) {
            const int nti = (i - 1) >> 6, ntj = (j - 1) >> 6;
            if (nti != cti || ntj != ctj) {
                cti = nti;
                ctj = ntj;
                ntiles++;
                need_tile(cti, ctj, true);
            }
            sh = ((unsigned)sgpr(torus[torus_of(i, j)]) >> (5 * L)) & 31u;
        } else {
            // degenerate walk at row 0 / column 0 with Python index wrapping
            // (RC: these cells' words may never have been recomputed; the host keeps such shapes off it)
            if (RC) rc_degenerate = true;
            const int ri = i < 0 ? i + m + 1 : i, rj = j < 0 ? j + n + 1 : j;
            const int pa = (i - 1) < 0 ? i - 1 + m : i - 1, pb = (j - 1) < 0 ? j - 1 + n : j - 1;
            if (ri < 0 || rj < 0 || pa < 0 || pa >= m || pb < 0 || pb >= n) { reason = 4; break; }  // IndexError
            int S;
            if (ri >= 1 && rj >= 1) {
                S = (sets_from_code(tb_code(w.tb, CB, w.TC, ri, rj), CB, o) >> (3 * L)) & 7;
            } else {
                const int* vv = ri == 0 ? w.bnd_row + 3 * rj : w.bnd_col + 3 * ri;
                const long long M = vv[0], X = vv[1], Y = vv[2];
                S = L == 0 ? argmin3(M, X, Y) : L == 1 ? argmin3(M + o, X, Y + o) : argmin3(M + o, X + o, Y);
            }
            sh = (unsigned)sgpr((int)(2u * S - 2u + (w.a[pa] == w.b[pb] ? 0u : 14u)));
        }
        const int lvl = (int)((tab >> (sh + 3u)) & 3u);
        uint8_t* ob = ops_byte(D);
        *ob = (uint8_t)(((D & 3) ? *ob : 0) | (lvl << (6 - 2 * (D & 3))));
        D++;
        i -= (lvl != 1);
        j -= (lvl != 2);
        L = lvl;
        if (first) {
            first = 0;
            if (i == 0 && j == 0 && !w.vhandoff) { reason = 0; break; }
            continue;
        }
        if (i == 0) { reason = iend; break; }
        if (j == 0) { reason = jend; break; }
        if (++h >= maxh) { reason = 3; break; }
    }

    if (reason < 0) {
        // ---- scalar interior walk (i, j >= 1; every move lowers i + j, so it ends at i == 0 or j == 0) ----
        const int lr = lane >> 3, lc = lane & 7;
        int vlo_i = 1 << 30, vlo_j = 1 << 30;  // lowest row / column of the verified tiles
        // verify the tile of (pi, pj) and its neighbours above / to the left (2x2 tiles): every window
        // anchored at least 20 rows and columns inside them is then cached
        auto verify = [&](int pi, int pj) {
            const int thi = (pi - 1) >> 6, thj = (pj - 1) >> 6;
            const int tli = max(thi - 1, 0), tlj = max(thj - 1, 0);
            const bool moved = thi != cti || thj != ctj;
            if (moved) ntiles++;
            need_tile(thi, thj, moved);
            if (tlj != thj) need_tile(thi, tlj, false);
            if (tli != thi) {
                need_tile(tli, thj, false);
                if (tlj != thj) need_tile(tli, tlj, false);
            }
            cti = thi;
            ctj = thj;
            vlo_i = tli == 0 ? -(1 << 30) : tli * TT + 1;
            vlo_j = tlj == 0 ? -(1 << 30) : tlj * TT + 1;
        };
        // one LDS read per lane: the 8x8 window anchored at (pi, pj)
        // (cells above row 1 / left of column 1 wrap round the torus and are never used)
        auto window = [&](int pi, int pj) -> int {
            const unsigned r = (unsigned)(pi - 1 - lr) & (TP - 1), c = (unsigned)(pj - 1 - lc) & (TP - 1);
            return torus[r * TP + c];
        };
        // widen a window cell (at the last step of the group that issued its read): the empty asm keeps
        // the compiler from pulling the widening (and so the wait for the LDS read) further forward
        auto widen = [](int raw) -> int {
            asm volatile("" : "+v"(raw));
            const unsigned u = (unsigned)raw;
            return (int)((u & 31u) | ((u & 0x3e0u) << 3) | ((u & 0x7c00u) << 6));
        };
        typedef __attribute__((address_space(4))) const uint32_t const_u32;  // scalar (constant) loads
        const unsigned long long rng_u = (unsigned long long)rng;
        const const_u32* rng_s = (const const_u32*)(((unsigned long long)(unsigned)sgpr((int)(rng_u >> 32)) << 32) |
                                                    (unsigned)sgpr((int)rng_u));
        const const_u32* rng_it = rng_s;  // SLD: entries of the current iteration (D .. D+15) and beyond
        int d_it = 0;
        auto tabs = [&](int d) -> uint4 {
            if constexpr (SLD) {
                const const_u32* p = rng_it + (d - d_it);  // a constant offset within an iteration
                return make_uint4(p[0], p[1], p[2], p[3]);
            } else {
                return *reinterpret_cast<const uint4*>(rngbuf + (d & (RB - 1)));
            }
        };

        if ((D & 511) == 0) {
            block_start(D);
            rng_ready(D);
        }
        verify(i, j);
        int wnext = window(i, j);    // anchored at the walk's current cell
        int wcw = widen(wnext);      // the next group's window, widened (off the next group's chain)
        uint4 tnext = tabs(D), tnext2 = tabs(D + 4);  // the entries of the next two groups
        unsigned rel = 0;            // offset of the current cell from wnext's anchor (di*8 + dj)
        unsigned L8 = 8u * L;        // bit offset of the entering level's field in a window cell
        unsigned ops = 0;

        // One group of 4 steps: swap in the prefetched window and entries, prefetch the next ones.
        // CHECK: stop at the matrix edge; returns the steps taken when the walk ended, else 0.
        // hook: work of the iteration's bookkeeping, placed in the group's scheduling region so that it issues in the
        // shadows of the chain's readlanes (in-order issue: at the loop boundary every instruction sat on the chain)
        auto group = [&](auto check_tag, int gd, auto hook) -> int {  // gd: dispatch of the group's first step
            constexpr bool CHECK = decltype(check_tag)::value;
            const int wcur = wcw;
            const uint4 tc = tnext;
            tnext = tnext2;
            // SLD: wait for this group's entries (loaded a group ago) before the new LDS / scalar loads go
            // out, so that the wait does not also cover them
            if constexpr (SLD) asm volatile("" ::"s"(tc.x), "s"(tc.y), "s"(tc.z), "s"(tc.w));
            const unsigned t[4] = {(unsigned)sgpr((int)tc.x), (unsigned)sgpr((int)tc.y), (unsigned)sgpr((int)tc.z),
                                   (unsigned)sgpr((int)tc.w)};
            // ix: the readlane index.  Only its low 6 bits count, so the moves go in unmasked; its low
            // byte is rel + the group's moves (diag 9, left 1, up 8: at most 4 rows and 4 columns).
            // A: the group's levels times 8, base 4.  (The walker is issue-bound: ~7 scalar ops a step.)
            unsigned ix = rel, A = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const unsigned v = (unsigned)__builtin_amdgcn_readlane(wcur, (int)ix);
                if (k == 0) {
                    // the next group's window and entries, issued in the first readlane's shadow (round 5: issued
                    // before it they sat on the chain), not where the next group needs them
                    __builtin_amdgcn_sched_barrier(0);
                    wnext = window(i, j);
                    __builtin_amdgcn_sched_barrier(0);
                    hook();
                }
                // widen the next group's window (read at this group's start) while the last step's
                // scalar chain runs
                if (k == 3) {
                    wcw = widen(wnext);
                    // the entries of the group after next, loaded once the widening's wait is behind (scalar loads
                    // return out of order, so a load in flight there made that wait cover it too)
                    __builtin_amdgcn_sched_barrier(0);
                    tnext2 = tabs(gd + 8);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // the chosen level comes out as the next field's bit offset (lvl * 8): two dependent
                // scalar ops fewer per step than extracting lvl and scaling it
                L8 = (t[k] >> ((v >> L8) & 31u)) & 0x18u;
                // A = A * 4 + L8 as the single fused op (the compiler's reassociated form took 11 ops a group)
                asm volatile("s_lshl2_add_u32 %0, %0, %1" : "+s"(A) : "s"(L8));
                ix += 0x080109u >> L8;
                if (CHECK) {
                    const unsigned mv = (ix - rel) & 0xffu;
                    if ((int)(mv >> 3) == i || (int)(mv & 7u) == j) {
                        i -= (int)(mv >> 3);
                        j -= (int)(mv & 7u);
                        ops = (ops << (2 * (k + 1))) | (A >> 3);
                        return k + 1;
                    }
                }
            }
            ops = (ops << 8) | (A >> 3);
            // the next group starts at this group's net move, unmasked (round 5): its low byte is the moves (no carry out
            // of it: at most 36 + 36), the upper bytes only this group's index-advance carries, which the readlane
            // ignores as it does inside a group; the mask is off the chain, for the bookkeeping
            const unsigned nrel = ix - rel, mv = nrel & 0xffu;
            i -= (int)(mv >> 3);
            j -= (int)(mv & 7u);
            rel = nrel;
            // the widening above stays in this group (scheduled past the boundary it put six VALU ahead of
            // the next group's first readlane)
            __builtin_amdgcn_sched_barrier(0);
            return 0;
        };
        // The iteration boundary, software-pipelined (round 5): an iteration's level word is stored during the next
        // one's first group, and whether the next iteration needs any test (a level block to start, tiles to verify,
        // the matrix edge) is decided during its third group from bounds (two groups move at most 8 rows and 8
        // columns); a fast iteration then follows with one branch.  The pending word goes out before any slow path.
        uint32_t* ops_slot = &ops_dummy;
        unsigned ops_pend = 0;
        bool fast;
        auto no_hook = []() {};
        auto flush_ops = [&]() {
            *ops_slot = ops_pend;
            ops_slot = &ops_dummy;
        };
        for (;;) {
            // iteration of 16 dispatches D .. D+15 (D % 16 == 0)
            if constexpr (SLD) {
                rng_it = rng_s + D;
                asm volatile("" : "+s"(rng_it));  // the address in SGPRs (no vector induction variable)
                d_it = D;
            }
            flush_ops();
            if ((D & 511) == 0) block_start(D);
            if (!SLD && ((D + 16) & 511) == 0) rng_ready(D + 16);
            // every window of this iteration is anchored within 12 steps: rows >= i - 19
            if (__builtin_expect(i - 19 < vlo_i || j - 19 < vlo_j, 0)) verify(i, j);
            if (__builtin_expect(min(i, j) > 16, 1)) {
                // fast iterations back to back: one branch between them
                do {
                    if constexpr (SLD) {
                        rng_it = rng_s + D;
                        asm volatile("" : "+s"(rng_it));
                        d_it = D;
                    }
                    const int dn = D + 16;
                    group(std::false_type{}, D, [&]() { *ops_slot = ops_pend; });
                    group(std::false_type{}, D + 4, no_hook);
                    group(std::false_type{}, D + 8, [&]() {
                        fast = (dn & 511) != 0 && (SLD || ((dn + 16) & 511) != 0) && min(i, j) > 24 &&
                               i - 27 >= vlo_i && j - 27 >= vlo_j;
                    });
                    group(std::false_type{}, D + 12, no_hook);
                    ops_slot = &opsbuf[(D >> 4) & (RB / 16 - 1)];
                    ops_pend = ops;
                    D = dn;
                } while (__builtin_expect(fast, 1));
                continue;
            }
            // near the top / left edge (the verified tiles reach row / column 1 here)
            int g = 0, k = 0;
            for (; g < 4; g++) {
                k = group(std::true_type{}, D + 4 * g, no_hook);
                if (k) break;
            }
            if (g < 4) {
                // ended after k steps of group g: left-align the partial word
                const int nd = 4 * g + k;
                opsbuf[(D >> 4) & (RB / 16 - 1)] = ops << (2 * (16 - nd));
                D += nd;
                reason = i == 0 ? iend : jend;
                break;
            }
            opsbuf[(D >> 4) & (RB / 16 - 1)] = ops;
            D += 16;
        }
    }
    if (lane == 0) {
        if (RC && (rc_timeout || rc_degenerate)) reason = 7;  // the recompute walk failed (host: GA_E_TIMEOUT)
        w.result[0] = D; w.result[1] = i; w.result[2] = j; w.result[3] = reason;
        w.result[4] = nwait; w.result[5] = ntiles;
        w.result[6] = (int)t_tile; w.result[7] = (int)t_ring;
        w.result[8] = (int)(__builtin_amdgcn_s_memrealtime() - t_start);
        w.result[9] = (int)((__builtin_amdgcn_s_memtime() - c_start) >> 4);
        w.result[10] = (int)load_ticks;  // loaders still running only finish tiles nobody waits for
        w.result[11] = load_count;
        __hip_atomic_store(&wD, D, __ATOMIC_RELEASE, WGS);
        __hip_atomic_store(&walk_done, 1, __ATOMIC_RELEASE, WGS);
    }
}

template <int CB>
__global__ void __launch_bounds__(64 * WALK_WAVES) walk_kernel(WalkArgs w) {
    __shared__ uint16_t torus[TP * TP];
    walk_body<CB>(w, w.rng, torus);
}

// A slot's walk arguments, read from the kernel arguments at a run-time index (vector loads), made
// wave-uniform field by field, so that the walk's control and addresses stay in scalar registers as
// in walk_kernel (without it the chain's walks held them in VGPRs and loaded tiles ~2x slower)
template <typename T>
__device__ __forceinline__ T* sgpr_ptr(T* p) {
    const unsigned long long x = (unsigned long long)p;
    return (T*)(((unsigned long long)(unsigned)sgpr((int)(x >> 32)) << 32) | (unsigned)sgpr((int)x));
}
__device__ __forceinline__ WalkArgs uniform_walk_args(const WalkArgs& s) {
    WalkArgs w;
    w.tb = sgpr_ptr(s.tb);
    w.CB = sgpr(s.CB);
    w.TC = sgpr(s.TC);
    w.a = sgpr_ptr(s.a);
    w.b = sgpr_ptr(s.b);
    w.bnd_row = sgpr_ptr(s.bnd_row);
    w.bnd_col = sgpr_ptr(s.bnd_col);
    w.rng = nullptr;
    w.nrng = (long long)(((unsigned long long)(unsigned)sgpr((int)(s.nrng >> 32)) << 32) | (unsigned)sgpr((int)s.nrng));
    w.m = sgpr(s.m);
    w.n = sgpr(s.n);
    w.o = sgpr(s.o);
    w.i0 = sgpr(s.i0);
    w.j0 = sgpr(s.j0);
    w.L0 = sgpr(s.L0);
    w.first0 = sgpr(s.first0);
    w.D0 = sgpr(s.D0);
    w.h0 = sgpr(s.h0);
    w.handoff = sgpr(s.handoff);
    w.vhandoff = sgpr(s.vhandoff);
    w.maxh = sgpr(s.maxh);
    w.ops = sgpr_ptr(s.ops);
    w.result = sgpr_ptr(s.result);
    w.dbg = sgpr_ptr(s.dbg);
    w.skip_corners = sgpr(s.skip_corners);
    w.nloaders = sgpr(s.nloaders);
    w.rc_flags = nullptr;
    w.rc_own = nullptr;
    w.rc_pos = nullptr;
    w.ops_prog = nullptr;
    return w;
}

// The pipelined alignments' walks, one after another in ONE launch: walk k starts as
// soon as walk k-1 has ended, on the CU the walks keep, with no host round trip in between.  Walk k
// reads the tie-break stream from global dispatch G_k = D_0 + ... + D_{k-1}, which only the walks
// know.  The host raises ctl[0] (fills done, in order; every fill has ended and its words are in
// HBM) and tab_ready (entries of the stream written); the kernel raises ctl[1] (walks done, their
// levels and results written back) and, on a wait past wait_limit, ctl[3].  ctl[2] = 1 (host) ends it.
template <int CB>
__global__ void __launch_bounds__(64 * WALK_WAVES) walk_chain_kernel(WalkChainArgs a) {
    __shared__ int go;
    __shared__ long long gnext;
    __shared__ uint16_t torus[TP * TP];
    long long G = 0;
    for (int k = 0; k < a.count; k++) {
        int wait_fill = 0, wait_tab = 0;  // polls that found the fill / the entries not ready (diagnostics)
        unsigned long long t_wait = 0;
        if (threadIdx.x == 0) {
            int ok = 1;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                if (__hip_atomic_load(a.ctl + 2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) { ok = 0; break; }
                const bool fill_ok = (int)__hip_atomic_load(a.ctl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) > k;
                const bool tab_ok = __hip_atomic_load(const_cast<long long*>(a.tab_ready), __ATOMIC_ACQUIRE,
                                                      __HIP_MEMORY_SCOPE_SYSTEM) >= G + a.per;
                if (fill_ok && tab_ok) break;
                wait_fill += !fill_ok;
                wait_tab += !tab_ok;
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.wait_limit) {
                    __hip_atomic_store(a.ctl + 3, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                    ok = 0;
                    break;
                }
                // ~3.4 us between polls: each is a PCIe read, and a walk may wait a whole fill (25 ms)
                __builtin_amdgcn_s_sleep(127);
            }
            go = ok;
            t_wait = __builtin_amdgcn_s_memrealtime() - t0;
        }
        __syncthreads();
        if (!sgpr(go)) return;  // uniform: the walks' control flow and arguments stay scalar
        __threadfence();  // acquire: the slot's traceback words and boundary, written by fill k
        const WalkArgs w = uniform_walk_args(a.w[k % a.S]);
        walk_body<CB, false, false>(w, a.tab + G, torus);
        if (threadIdx.x == 0) {  // result[12..14]: this walk's wait before it started (ticks, polls)
            w.result[12] = (int)t_wait;
            w.result[13] = wait_fill;
            w.result[14] = wait_tab;
        }
        __threadfence_system();  // the levels (and result) reach memory before ctl[1] says so
        __syncthreads();
        if (threadIdx.x == 0) {
            gnext = G + *(volatile int*)w.result;  // result[0] = D_k, written by this lane
            __hip_atomic_store(a.ctl + 1, (unsigned)(k + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        const long long gn = gnext;
        G = (long long)(((unsigned long long)(unsigned)sgpr((int)(gn >> 32)) << 32) | (unsigned)sgpr((int)gn));
    }
}

}  // namespace ga
