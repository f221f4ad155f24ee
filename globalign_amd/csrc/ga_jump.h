// ga_jump.h -- the tie-to-tie walk (dp_array_backward, globaligner.py:395-593): the recompute walk's
// walker advancing one precomputed run of moves per LDS round trip instead of one move per step.
//
// Of the walk's moves only ~6 % meet a tie (a rank set of two or more levels, where cost_ranks_dispatcher's
// random.choice decides, :595-685); every other move is fixed by the cell and the entering level.  The recompute
// workers (ga_rcwalk.hip, JUMP) therefore store per cell and entering level L a 16-bit jump entry:
//   * a tie: bits 1:0 = 0, bits 6:2 = the tie-break table shift sh = 2S - 2 + 14*(a_i != b_j) of ga_walk.h;
//   * otherwise up to 8 moves, move q in bits 2q+1:2q (bit 0: the move lowers j, bit 1: it lowers i; diag 3,
//     left 1, up 2; 0 after the last): the state's own singleton move, then the moves of its successor's entry
//     (the successor entered at that move's level), cut where that successor is a tie or lies outside the block
//     the entry was built in, and after 8 moves.  Every entry is a run of real moves of the deterministic walk.
// The walker stands at a state t (cell (i, j), level L, dispatch D) and per trip issues ONE ds_read: t's three
// level entries (lanes 0..2) and the entries of t's three successors at their levels (lanes 3..5), with the
// table entry of dispatch D beside it.  If t's entry is a run it advances by it; at a tie the table picks the
// level x and it advances by the tie move and the successor's run.  The moves go straight into the walk's
// level stream (2 bits per dispatch, dispatch D at bits 30 - 2*(D & 15) of word D >> 4, as ga_walk.h writes it),
// so the host side is unchanged.  tools/jump_model.py is the CPU model (6.6 moves per trip at C3's shape).
//
// The entries live in a 128 x 128 torus per level (3 x 32 KB of LDS): 4 x 4 tiles of 32 x 32 cells, copied by
// the loader waves from the workers' cache in HBM (6 KB per tile: [level][32 rows][32 columns] u16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ga_device.h"
#include "ga_sync.h"
#include "ga_walk.h"

namespace ga {

constexpr int JT = 32;                        // jump tile edge
constexpr int JB = 4;                         // tiles cached per axis
constexpr int JP = JB * JT;                   // torus pitch (128)
constexpr int JPLANE = JP * JP;               // cells per level plane
constexpr int JTILE_BYTES = 3 * JT * JT * 2;  // one tile in the HBM cache
constexpr int JNSLOT = JB * JB;
constexpr int JM = 10;                        // the trip loop runs while i, j > JM (a trip moves <= 9 rows / columns)
// Waves of the walker's workgroup: 0 walks, 4 is the helper (both on SIMD 0), the other six load tiles.  Eight,
// not walk_body's sixteen: the kernel's workers (one wave per workgroup) need ~200 VGPRs, which 16-wave
// workgroups (128 per lane at most) would spill.  A loader only copies 6 KB per tile (no decode).
constexpr int JWALK_WAVES = 8;
constexpr int JNLOAD = JWALK_WAVES - 2;

__host__ __device__ inline size_t jump_torus_bytes() { return (size_t)3 * JPLANE * sizeof(uint16_t); }
// bytes of one block (64 rows x 64*TD columns: 2 x 2TD tiles) in the HBM cache
__host__ __device__ inline size_t jump_block_bytes(int TD) { return (size_t)4 * TD * JTILE_BYTES; }

__device__ __forceinline__ int jslot_of(int ti, int tj) { return (ti & (JB - 1)) * JB + (tj & (JB - 1)); }
__device__ __forceinline__ int jtorus_of(int i, int j) { return ((i - 1) & (JP - 1)) * JP + ((j - 1) & (JP - 1)); }
__device__ __forceinline__ bool jin_block(int cur, int ti, int tj) {
    const int dti = (cur >> 16) - ti, dtj = (cur & 0xffff) - tj;
    return cur >= 0 && dti >= 0 && dti < JB && dtj >= 0 && dtj < JB;
}
// the level of a move's 2-bit code (diag 3 -> 0, left 1 -> 1, up 2 -> 2) and back
__device__ __forceinline__ unsigned jlevel(unsigned code) { return code == 3u ? 0u : code; }
__device__ __forceinline__ unsigned jcode(unsigned lvl) { return lvl == 0u ? 3u : lvl; }

// One loader wave copies 32-tile (ti, tj) from the cache (block (ti/2, tj/2TD) at slot (bi mod RC_CACHE_I, bs mod
// RC_CACHE_S), written with sc1 stores by the workers of the same launch: sc1 loads) into the torus.
__device__ __forceinline__ void jload_tile(const WalkArgs& w, int ti, int tj, uint16_t* E, int lane) {
    const int bi = ti >> 1, tr = ti & 1, td2 = 2 * w.rc_td, bs = tj / td2, tc = tj - bs * td2;
    const uint8_t* src = w.tb +
                         ((long long)((bi % RC_CACHE_I) * RC_CACHE_S + bs % RC_CACHE_S) * (2 * td2) + tr * td2 + tc) *
                             JTILE_BYTES +
                         lane * 16;
    wk_u4 v0, v1, v2, v3, v4, v5;
    asm volatile(
        "global_load_dwordx4 %0, %6, off sc1\n\t"
        "global_load_dwordx4 %1, %6, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %2, %6, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %3, %6, off offset:3072 sc1\n\t"
        "global_load_dwordx4 %4, %7, off sc1\n\t"
        "global_load_dwordx4 %5, %7, off offset:1024 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(v4), "=&v"(v5)
        : "v"(src), "v"(src + 4096)
        : "memory");
    const wk_u4 v[6] = {v0, v1, v2, v3, v4, v5};
    // 16 bytes q*1024 + lane*16 of the tile: level q >> 1, row (q & 1)*16 + lane/4, columns (lane & 3)*8 ..+7
    const int r0 = (ti & (JB - 1)) * JT + (lane >> 2), c0 = (tj & (JB - 1)) * JT + (lane & 3) * 8;
#pragma unroll
    for (int q = 0; q < 6; q++) {
        uint16_t* d = E + (q >> 1) * JPLANE + (r0 + (q & 1) * 16) * JP + c0;
        *reinterpret_cast<wk_u4*>(d) = v[q];
    }
}

// The tie-to-tie walk of walk_rc_jump_kernel's workgroup 0 (roles as walk_body<CB, RC = true>: wave 0 walks, wave 4
// is the helper, the other six load tiles).  E: the 3 x 128 x 128 torus (dynamic LDS).
__device__ __forceinline__ void walk_jump_body(const WalkArgs& w, const uint32_t* rng, uint16_t* E) {
    unsigned tid = threadIdx.x;
    __shared__ __attribute__((aligned(16))) uint32_t jrngbuf[RB];
    __shared__ uint32_t jopsbuf[RB / 16];
    __shared__ int jtag[JNSLOT];
    __shared__ int jrtag[4];
    __shared__ int jcur_tile, jwalk_done, jwD, jops_flushed, jrc_timeout;
    __shared__ unsigned long long jload_ticks;
    __shared__ int jload_count;
    const int lane = tid & 63;
    const int wave = sgpr(tid >> 6);
    if (tid == 0) {
        jload_ticks = 0;
        jload_count = 0;
        jcur_tile = -1;
        jwalk_done = 0;
        jwD = w.D0;
        jops_flushed = w.D0 >> 9;
        jrc_timeout = 0;
    }
    if (tid < JNSLOT) jtag[tid] = -1;
    if (tid < 4) jrtag[tid] = -1;
    __syncthreads();

    if (wave == 4) {
        // ---------------- helper: tie-break table HBM -> LDS ring, levels LDS ring -> HBM, the walker's block
        // (64-row tiles, the workers' unit) published for the recompute workers ----------------
        const long long nblk = (w.nrng + 511) / 512;
        long long rl = w.D0 >> 9, fl = w.D0 >> 9;
        int pub = -1;
        for (;;) {
            const int done = sgpr(__hip_atomic_load(&jwalk_done, __ATOMIC_ACQUIRE, WGS));
            const int d = sgpr(__hip_atomic_load(&jwD, __ATOMIC_ACQUIRE, WGS));
            bool moved = false;
            const int cur = sgpr(__hip_atomic_load(&jcur_tile, __ATOMIC_ACQUIRE, WGS));
            if (cur >= 0 && cur != pub) {
                const int c64 = ((cur >> 17) << 16) | ((cur & 0xffff) >> 1);  // 32-tiles -> 64-tiles
                if (lane == 0) g_st(w.rc_pos, (unsigned)c64 + 1u);
                pub = cur;
            }
            while (rl < nblk && rl < (d >> 9) + 4) {
                const long long e0 = rl * 512 + lane * 8;
                uint32_t* dst = jrngbuf + (rl & 3) * 512 + lane * 8;
#pragma unroll
                for (int k = 0; k < 8; k++) dst[k] = (e0 + k < w.nrng) ? rng[e0 + k] : 0u;
                if (lane == 0) __hip_atomic_store(&jrtag[rl & 3], (int)rl, __ATOMIC_RELEASE, WGS);
                rl++;
                moved = true;
            }
            const long long complete = done ? ((long long)d + 511) / 512 : (d >> 9);
            const long long fl0 = fl;
            while (fl < complete) {
                if (lane < 32) {
                    const uint32_t v = jopsbuf[(fl & 3) * 32 + lane];
                    if (w.ops_prog != nullptr) __hip_atomic_store(w.ops + fl * 32 + lane, v, RLX, __HIP_MEMORY_SCOPE_SYSTEM);
                    else w.ops[fl * 32 + lane] = v;
                }
                fl++;
                if (lane == 0) __hip_atomic_store(&jops_flushed, (int)fl, __ATOMIC_RELEASE, WGS);
                moved = true;
            }
            if (w.ops_prog != nullptr && fl > fl0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0)
                    __hip_atomic_store(w.ops_prog, done ? (unsigned)d : (unsigned)(fl * 512), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (done && fl >= complete) break;
            if (!moved) __builtin_amdgcn_s_sleep(2);
        }
        if (lane == 0) g_st(w.rc_pos + 1, 1u);  // the recompute workgroups may end
        return;
    }

    if (wave > 0) {
        // ---------------- loaders: loader li owns torus slots li, li + 6, li + 12 (< 16): the walker's next tiles
        // (offsets (1,0), (0,1), (1,1): slots 4, 1, 5 away) belong to different loaders ----------------
        const int li = wave - 1 - (wave > 4);
        constexpr int NQ = (JNSLOT + JNLOAD - 1) / JNLOAD;
        while (!sgpr(__hip_atomic_load(&jwalk_done, __ATOMIC_ACQUIRE, WGS))) {
            const int cur = sgpr(__hip_atomic_load(&jcur_tile, __ATOMIC_ACQUIRE, WGS));
            bool did = false;
            if (cur >= 0) {
                const int ti = cur >> 16, tj = cur & 0xffff;
                int cand[NQ], dist[NQ];
#pragma unroll
                for (int q = 0; q < NQ; q++) {
                    const int sl = li + JNLOAD * q, sr = sl >> 2, sc = sl & 3;
                    const int di = (ti - sr) & (JB - 1), dj = (tj - sc) & (JB - 1);
                    cand[q] = (sl >= JNSLOT || ti - di < 0 || tj - dj < 0) ? -1 : (((ti - di) << 16) | (tj - dj));
                    // the far off-diagonal corners of the block (walk paths run near the diagonal; ga_walk.h)
                    if (max(di, dj) == JB - 1 && abs(di - dj) >= 2) cand[q] = -1;
                    dist[q] = cand[q] < 0 ? (1 << 20) : di + dj;
                }
                // nearest first
                for (int pass = 0; pass < NQ && !did; pass++) {
                    int q = 0;
#pragma unroll
                    for (int x = 1; x < NQ; x++)
                        if (dist[x] < dist[q]) q = x;
                    const int tg = cand[q];
                    dist[q] = 1 << 21;
                    if (tg < 0) continue;
                    const int sl = li + JNLOAD * q, tti = tg >> 16, ttj = tg & 0xffff;
                    if (sgpr(__hip_atomic_load(&jtag[sl], __ATOMIC_RELAXED, WGS)) == tg) continue;
                    // only once the tile's block has been recomputed (its entries are then in the cache)
                    if (!rc_slot_ok(w, tti >> 1, ttj / (2 * w.rc_td), true)) continue;
                    if (lane == 0) __hip_atomic_store(&jtag[sl], -1, __ATOMIC_SEQ_CST, WGS);
                    if (!jin_block(sgpr(__hip_atomic_load(&jcur_tile, __ATOMIC_SEQ_CST, WGS)), tti, ttj)) continue;
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    jload_tile(w, tti, ttj, E, lane);
                    if (!rc_slot_ok(w, tti >> 1, ttj / (2 * w.rc_td), false)) continue;  // its slot changed under the copy
                    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the tile's LDS stores before its tag
                    if (lane == 0) {
                        atomicAdd(&jload_ticks, __builtin_amdgcn_s_memrealtime() - t0);
                        atomicAdd(&jload_count, 1);
                    }
                    if (lane == 0 && jin_block(sgpr(__hip_atomic_load(&jcur_tile, __ATOMIC_SEQ_CST, WGS)), tti, ttj))
                        __hip_atomic_store(&jtag[sl], tg, __ATOMIC_RELEASE, WGS);
                    did = true;
                }
            }
            if (!did) __builtin_amdgcn_s_sleep(1);
        }
        return;
    }

    // ---------------- walker wave ----------------
    __builtin_amdgcn_s_setprio(3);
    int i = w.i0, j = w.j0, L = w.L0, D = w.D0, h = w.h0, first = w.first0, reason = -1;
    const int jend = w.handoff ? 5 : 2;  // reason when the walk reaches local column 0
    const int iend = 1;
    int cti = -1, ctj = -1, nwait = 0, ntiles = 0;
    int ntrips = 0, nverify = 0, nties = 0;  // diagnostics (result[12..14])
    unsigned rc_spins = 0;
    bool rc_degenerate = false;
    const int maxh = w.maxh;
    unsigned long long t_tile = 0, t_ring = 0;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c_start = __builtin_amdgcn_s_memtime();
    auto need_tile = [&](int ti, int tj, bool publish) {
        const int tg = (ti << 16) | tj;
        if (publish && lane == 0) __hip_atomic_store(&jcur_tile, tg, __ATOMIC_SEQ_CST, WGS);
        const int sl = jslot_of(ti, tj);
        if (sgpr(__hip_atomic_load(&jtag[sl], __ATOMIC_SEQ_CST, WGS)) == tg) return;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (sgpr(__hip_atomic_load(&jtag[sl], __ATOMIC_ACQUIRE, WGS)) != tg) {
            __builtin_amdgcn_s_sleep(1);
            nwait++;
            if (++rc_spins > (1u << 25)) {  // a tile that never comes: reason 7 instead of a hang
                jrc_timeout = 1;
                break;
            }
        }
        t_tile += __builtin_amdgcn_s_memrealtime() - t0;
    };
    auto block_start = [&](int d) {
        const int blk = d >> 9;
        if (lane == 0) __hip_atomic_store(&jwD, d, __ATOMIC_RELEASE, WGS);
        if (sgpr(__hip_atomic_load(&jops_flushed, __ATOMIC_ACQUIRE, WGS)) >= blk - 3) return;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (sgpr(__hip_atomic_load(&jops_flushed, __ATOMIC_ACQUIRE, WGS)) < blk - 3) __builtin_amdgcn_s_sleep(1);
        t_ring += __builtin_amdgcn_s_memrealtime() - t0;
    };
    auto rng_ready = [&](int d) {
        const int blk = d >> 9;
        if (sgpr(__hip_atomic_load(&jrtag[blk & 3], __ATOMIC_ACQUIRE, WGS)) == blk) return;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (sgpr(__hip_atomic_load(&jrtag[blk & 3], __ATOMIC_ACQUIRE, WGS)) != blk) __builtin_amdgcn_s_sleep(1);
        t_ring += __builtin_amdgcn_s_memrealtime() - t0;
    };
    // Levels: pend holds the levels of dispatches Dw .. D-1 (Dw = D & ~15), dispatch Dw + q at bits 63 - 2q..62 - 2q.
    // put(lv, k): k levels MSB-aligned in lv, for dispatches D .. D+k-1 (k <= 16); a word completes when D passes
    // Dw + 16 and goes to its ring slot.  A slab walk may start inside a word: the levels before D stay zero.
    unsigned long long pend = 0;
    int Dw = D & ~15;
    auto put = [&](unsigned lv, int k) {
        pend |= ((unsigned long long)lv << 32) >> (2 * (D - Dw));
        D += k;
        if (D - Dw >= 16) {
            jopsbuf[(Dw >> 4) & (RB / 16 - 1)] = (uint32_t)(pend >> 32);
            pend <<= 32;
            Dw += 16;
            if ((Dw & 511) == 0) {
                block_start(Dw);
                rng_ready(Dw);
            }
        }
    };

    // ---- per-step path: the first move, the last moves near row / column 0 (and degenerate walks, which the
    //      recompute walk reports with reason 7) ----
    rng_ready(D);
    auto step = [&]() -> bool {  // one move; true when the walk has ended (reason set)
        unsigned lvl;
        if (i >= 1 && j >= 1) {
            const int nti = (i - 1) >> 5, ntj = (j - 1) >> 5;
            if (nti != cti || ntj != ctj) {
                cti = nti;
                ctj = ntj;
                ntiles++;
                need_tile(cti, ctj, true);
            }
            const unsigned e = (unsigned)sgpr(E[L * JPLANE + jtorus_of(i, j)]);
            if (e & 3u) {
                lvl = jlevel(e & 3u);
            } else {
                const unsigned tab = (unsigned)sgpr((int)jrngbuf[D & (RB - 1)]);
                lvl = (tab >> (((e >> 2) & 31u) + 3u)) & 3u;
            }
        } else {
            rc_degenerate = true;  // (the host keeps such shapes off the recompute walk)
            reason = 4;
            return true;
        }
        put(lvl << 30, 1);
        i -= (lvl != 1);
        j -= (lvl != 2);
        L = (int)lvl;
        if (first) {
            first = 0;
            if (i == 0 && j == 0) { reason = 0; return true; }
            return false;
        }
        if (i == 0) { reason = iend; return true; }
        if (j == 0) { reason = jend; return true; }
        if (++h >= maxh) { reason = 3; return true; }
        return false;
    };
    // the first move(s): until the walk stands inside the trip loop's bounds
    while (reason < 0 && (first || i <= JM || j <= JM)) {
        if (step()) break;
        if (!first && min(i, j) <= JM) {
            // near the top / left edge from the start: per step to the end
            while (reason < 0 && !step()) {}
            break;
        }
    }

    if (reason < 0) {
        // ---- trip loop ----
        // Tiles: the walker verifies the 2 x 2 tiles at its cell's tile (publishing that tile first: the loaders
        // never evict a tile of the 4 x 4 block at the published tile; publish / tag read against the loaders'
        // invalidate / re-check is ga_walk.h's Dekker handshake).  Every trip from a cell >= 10 rows and columns
        // inside the verified region reads and lands inside it, so the walker re-verifies only when it comes within
        // 10 of the region's top or left edge (about once per tile crossed).  One verification is one LDS round
        // trip: lanes 0..3 read the four tags at once (4 dependent reads before: ~0.9 ms of C3's walk); only a
        // missing tile is waited for.  (Verifying the 3 x 3 tiles ahead without blocking, round 5, blocked the walker
        // on tiles two away that the loaders had not reached: slower.)
        int vlo_i = 1 << 30, vlo_j = 1 << 30;
        const unsigned tagbase = lds_addr(jtag);
        auto verify = [&](int pi, int pj) {
            const int thi = (pi - 1) >> 5, thj = (pj - 1) >> 5;
            const int tli = max(thi - 1, 0), tlj = max(thj - 1, 0);
            if (thi != cti || thj != ctj) {
                ntiles++;
                if (lane == 0) __hip_atomic_store(&jcur_tile, (thi << 16) | thj, __ATOMIC_SEQ_CST, WGS);
            }
            const int xi = (lane & 2) ? tli : thi, xj = (lane & 1) ? tlj : thj;
            unsigned tv;
            asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(tv)
                         : "v"(tagbase + 4u * (unsigned)jslot_of(xi, xj)) : "memory");
            if (__builtin_amdgcn_ballot_w64(lane < 4 && tv != (unsigned)((xi << 16) | xj))) {
                need_tile(thi, thj, false);
                if (tlj != thj) need_tile(thi, tlj, false);
                if (tli != thi) {
                    need_tile(tli, thj, false);
                    if (tlj != thj) need_tile(tli, tlj, false);
                }
            }
            cti = thi;
            ctj = thj;
            vlo_i = tli * JT + 1;
            vlo_j = tlj * JT + 1;
        };
        // per-lane fetch offsets: lanes 0..2 t's level planes, 3..5 the successors (diag / left / up) at their
        // level; rows of JP cells (2*JP bytes), planes of JPLANE cells
        const unsigned drow = (lane == 3 || lane == 5) ? 2u * JP : 0u;
        const unsigned dcol = (lane == 3 || lane == 4) ? 2u : 0u;
        const unsigned plane = 2u * JPLANE * (unsigned)(lane < 3 ? lane : lane < 6 ? lane - 3 : 0);
        const unsigned ebase = lds_addr(E) + plane;
        // the table: lanes 8..17 read dispatches d .. d+9 (a trip moves <= 9), so the next state's entry (dispatch
        // d + k) is already in a register when its trip begins: lane 8 + k.  (The ring holds 4 blocks of 512
        // dispatches; d+9 past a block boundary may read an older block: such an entry is only used after
        // rng_ready, below.)
        const unsigned tbase = lds_addr(jrngbuf) + 4u * (unsigned)(lane >= 8 && lane < 18 ? lane - 8 : 0);
        // One trip: t's entries and its successors' (lanes 0..5), one LDS round trip.  The loop is software-
        // pipelined so that only the chain sits between a fetch landing and the next fetch going out: the entry
        // taken (readlane), the advance (i, j: a mask and a bit count each), the next fetch's addresses; the table
        // read, the level record (put), the move count and the region check run while it is in flight.  A fetch
        // whose cell has left the verified tiles reads harmless torus cells (the addresses are masked): the check
        // after it then re-verifies and fetches again.
        auto fetch_e = [&](unsigned& v) {  // the entries: needs only (i, j)
            const unsigned roff = ((unsigned)(i - 1) & (JP - 1)) << 8, coff = ((unsigned)(j - 1) & (JP - 1)) << 1;
            const unsigned addr = ebase + (((roff - drow) & (2u * JP * (JP - 1))) | ((coff - dcol) & (2u * (JP - 1))));
            asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(addr));
            __builtin_amdgcn_sched_barrier(0);
        };
        auto fetch_t = [&](unsigned& tb, int d) {  // the table entries of dispatches d .. d+9
            asm volatile("ds_read_b32 %0, %1" : "=v"(tb) : "v"(tbase + (((unsigned)d << 2) & (4u * (RB - 1)))));
        };
        auto outside = [&]() { return ((i - 10 - vlo_i) | (j - 10 - vlo_j)) < 0; };
        verify(i, j);
        if (!outside()) {
            unsigned v, tb;
            int kprev = 0;
            fetch_e(v);
            fetch_t(tb, D);
            for (;;) {
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v), "+v"(tb));
                const unsigned e = (unsigned)__builtin_amdgcn_readlane((int)v, L);
                unsigned W;
                ntrips++;
                if (__builtin_expect(e & 3u, 1)) {
                    W = e;
                } else {
                    nties++;
                    // a tie: the table picks the level x; W = the tie move, then x's successor's run (none if a tie)
                    const unsigned t = (unsigned)__builtin_amdgcn_readlane((int)tb, 8 + kprev);
                    const unsigned x = (t >> (((e >> 2) & 31u) + 3u)) & 3u;
                    const unsigned sx = (unsigned)__builtin_amdgcn_readlane((int)v, (int)(3u + x));
                    W = (((sx & 3u) ? sx : 0u) << 2) | jcode(x);
                }
                i -= __builtin_popcount(W & 0xaaaaau);
                j -= __builtin_popcount(W & 0x55555u);
                fetch_e(v);  // speculative while the region check below is pending
                const int k = __builtin_popcount((W | (W >> 1)) & 0x55555u);
                fetch_t(tb, D);
                kprev = k;
                if (__builtin_expect(((D + k) ^ D) >> 9, 0)) {
                    // a new block of table entries: the helper keeps the ring 3 blocks ahead, but make sure (and read
                    // the entries again once they are there)
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v), "+v"(tb));
                    rng_ready(D + k);
                    fetch_t(tb, D + k);
                    kprev = 0;
                }
                L = (int)jlevel((W >> (2 * k - 2)) & 3u);
                // the moves as levels, MSB first: bit-reversing W swaps each field's two bits, and xor 3 maps the
                // swapped codes (diag 3, left 2, up 1) to the levels 0, 1, 2
                put(__builtin_bitreverse32(W) ^ ~(0xffffffffu >> (2 * k)), k);
                h += k;
                if (__builtin_expect(outside(), 0)) {
                    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v), "+v"(tb));
                    nverify++;
                    verify(i, j);
                    if (outside()) break;
                    fetch_e(v);
                    fetch_t(tb, D);
                    kprev = 0;
                }
            }
        }
        first = 0;
        // the last moves, per step, near row / column 0
        while (reason < 0 && !step()) {}
    }
    // the partial last word of levels
    jopsbuf[(Dw >> 4) & (RB / 16 - 1)] = (uint32_t)(pend >> 32);
    if (lane == 0) {
        if (jrc_timeout || rc_degenerate) reason = 7;  // the recompute walk failed (host: GA_E_TIMEOUT)
        w.result[0] = D; w.result[1] = i; w.result[2] = j; w.result[3] = reason;
        w.result[4] = nwait; w.result[5] = ntiles;
        w.result[6] = (int)t_tile; w.result[7] = (int)t_ring;
        w.result[8] = (int)(__builtin_amdgcn_s_memrealtime() - t_start);
        w.result[9] = (int)((__builtin_amdgcn_s_memtime() - c_start) >> 4);
        w.result[10] = (int)jload_ticks;
        w.result[11] = jload_count;
        w.result[12] = ntrips;
        w.result[13] = nverify;
        w.result[14] = nties;
        __hip_atomic_store(&jwD, D, __ATOMIC_RELEASE, WGS);
        __hip_atomic_store(&jwalk_done, 1, __ATOMIC_RELEASE, WGS);
    }
}

}  // namespace ga
