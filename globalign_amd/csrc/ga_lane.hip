// ga_lane.hip -- the lane-skewed anti-diagonal score fill (dp_array_forward, globaligner.py:366-392;
// get_next_best_costs :317-363), score only.  DESIGN.md 5.6.
//
// A stripe is 64*TD columns; lane l owns the TD adjacent columns j0+l*TD+1 .. j0+l*TD+TD and at step
// t works on row i = t - l + 1 of all of them.  So a lane's TD columns are one in-register row
// segment (h1' chained through them, 5 VALU per cell) and only the lane-to-lane hand-over is skewed:
// lane l takes h1'(i, left) from lane l-1's step t-1 and H'(i-1, left) from its step t-2 through
// two DPP lane shifts per step.  Compared with the per-column skew of fill_diag_kernel the skew
// across a stripe is 64 steps instead of 64*TD, and compared with the row scan (fill_kernel) no
// step pays a 64-lane scan: tools/micro/lane_bench.hip puts the TD = 8 step at 0.41 SIMD cycles
// per cell with every per-step overhead of this kernel (the blocked row scan runs C4 at 0.77).
//
// Per 8-step sub-chunk a compute wave
//   * reads the next sub-chunk's 8 left-edge rows (H', h1') from its input ring (LDS, broadcast),
//   * reads its lanes' profile windows: sub' bytes of 8 consecutive rows per column from a table
//     whose dword r holds rows r..r+3 of one code (any start row is dword aligned), so a step's
//     profile value is an SDWA byte select folded into M' = H'(diag) + sub',
//   * writes lane 63's 8 outputs: each step shifts lane 63's (H', h1') into a DPP shift register
//     (wave_shl:1), whose lanes 56..63 then hold the sub-chunk's rows; one 8-lane store.
// The IO wave feeds ring 0 from HBM (the slab's left edge, the previous workgroup's hand-off rows
// or another GPU's halo), drains the last wave's ring to HBM and fills the profile table, exactly
// as the row-scan and per-column anti-diagonal kernels do (ga_kernels.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ga_device.h"
#include "ga_lane.h"
#include "ga_lane_asm.h"
#include "ga_sync.h"

#ifndef GA_LANE_LE
#define GA_LANE_LE 13
#endif

namespace ga {

// The slab (chain position) of this workgroup; thread 0 only.  Ticket order by default: a later slab never
// waits on one whose workgroup is not yet running.  p.xcd_map (one round of workgroups, every stripe resident):
// the hardware dispatches workgroup h to XCD h mod 8, so consecutive tickets sit on different XCDs and every
// cross-workgroup hand-off crossed the non-coherent L2 boundary (540 against 385 ns one way,
// profiles/r04/micro_handoff_lat.txt).  Instead the slabs are cut into one contiguous run per XCD, in XCD
// order, each run as long as the number of workgroups that XCD received: 7 links cross XCDs instead of
// nslabs - 1.  That order is safe only with every workgroup resident, so it is used only once all have
// arrived (the last to arrive says so); if they have not within ~40 us (the device busy with other work),
// the first to give up switches every workgroup to ticket order (one CAS decides).
// Flags: [0] arrivals (the ticket), [2] mode (0 pending, 1 per XCD, 2 tickets), [4 + x] arrivals on XCD x.
__device__ unsigned lane_slab(const FillArgs& p) {
    unsigned* F = p.ticket;
    if (!p.xcd_map) return atomicAdd(F, 1u);
    const unsigned x = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20) & 7u;  // HW_REG_XCC_ID bits 3:0
    const unsigned rk = __hip_atomic_fetch_add(F + 4 + x, 1u, __ATOMIC_RELAXED, AGENT);
    // the per-XCD count first: once the last arrival is seen every count is final
    const unsigned arr = __hip_atomic_fetch_add(F, 1u, __ATOMIC_ACQ_REL, AGENT);
    unsigned mode = 0;
    if (arr == (unsigned)p.nslabs - 1u) {
        unsigned exp = 0;
        mode = __hip_atomic_compare_exchange_strong(F + 2, &exp, 1u, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE, AGENT) ? 1u : exp;
    } else {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while ((mode = __hip_atomic_load(F + 2, __ATOMIC_ACQUIRE, AGENT)) == 0u) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 4000) {  // 40 us (100 MHz)
                unsigned exp = 0;
                mode = __hip_atomic_compare_exchange_strong(F + 2, &exp, 2u, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE, AGENT)
                           ? 2u : exp;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    if (mode != 1u) return arr;
    unsigned start = 0;
    for (unsigned y = 0; y < x; y++) start += __hip_atomic_load(F + 4 + y, __ATOMIC_RELAXED, AGENT);
    return start + rk;
}

// The query profile of a lane fill's rows (FillArgs::qprof): dword r + 2 of code c (r = -2 .. m + 1) holds sub'(a_r .. a_r+3, c)
// as int8 bytes, rows outside 1..m zero -- the dwords the profile wave used to build per row from a and sub' (for a
// 24-code alphabet 96 LDS byte reads and 24 writes per lane per 64 rows: at C5 it fell behind the chain's head, which
// then waited on it for 32 % of its steps, round 5, profiles/r05/c5_stamps.txt); one thread per dword
__global__ void __launch_bounds__(256) lane_qprof_kernel(const uint8_t* __restrict__ a, int m, const int* __restrict__ subp,
                                                         int K, uint32_t* __restrict__ out) {
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int pitch = m + 4;
    if (q >= (long long)K * pitch) return;
    const int c = (int)(q / pitch), r = (int)(q % pitch) - 2;
    uint32_t v = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int row = r + u;
        if (row >= 1 && row <= m) v |= (uint32_t)(uint8_t)(int8_t)subp[a[row - 1] * K + c] << (8 * u);
    }
    out[q] = v;
}

void launch_lane_qprof(hipStream_t s, const uint8_t* a, int m, const int* subp, int K, uint32_t* out) {
    const long long nq = (long long)K * (m + 4);
    lane_qprof_kernel<<<dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s>>>(a, m, subp, K, out);
}

size_t fill_lane_lds_bytes(int nwc, int K, int qrows) {
    return (size_t)LK_HEAD_BYTES + (size_t)(nwc + 1) * RING * sizeof(int2) + (size_t)K * (qrows + LK_QMIRROR) * 4 +
           (size_t)K * 32;  // + the K x K int8 sub' table (K <= 32)
}

// DBG: per stripe {start, end (s_memrealtime), cycles waiting for edges / profile / ring space,
// total cycles, HW_ID} into p.dbg (tools/lane_stamps.py)
// CB > 0: traceback words (CB bytes per cell) into p.tb in fill_kernel's aligned layout; SUB: steps per
// sub-chunk (8 or 16: the edge / profile reads, the publish and the waits are paid once per SUB steps)
// CKP: the banded traceback's score pass, storing the checkpoint rows (a variant of its own: the extra
// paths cost the plain score fill registers)
// RC: the recompute checkpoints (score only): every stripe's right edge to p.colck (lanes
// 64-SUB..63's shift registers after each sub-chunk, 128 B per store) and, every p.stck_every steps, each
// lane's whole state (its columns' H' and h2', the h1' it hands right, the diagonal H' it took from the
// left) to p.stck: a staircase (lane l at row k*stck_every - l) from which any 64-row tile of the stripe
// is recomputed with the same steps (ga_rcwalk.hip)
// LATE: score-only waves await and read the next sub-chunk's edges GA_LANE_LE steps into a sub-chunk
// instead of after its first step (a stripe then trails its left neighbour by that many steps less, at ~3 %
// more cycles per step): for one-round chains (C3, slabs), whose time is m steps plus every stripe's lag;
// fills in rounds (C4 on one GPU) run uncoupled and keep the early reads
template <int NWC, int TD, int CB, int SUB, bool DBG, bool CKP = false, bool RC = false, bool LATE = false>
__global__ void __launch_bounds__(lane_block_threads(NWC)) fill_lane_kernel(FillArgs p) {
    constexpr bool OUTW = lane_out_wave(NWC);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    unsigned* cnt = reinterpret_cast<unsigned*>(smem);
    int2* ring = reinterpret_cast<int2*>(smem + LK_HEAD_BYTES);
    uint32_t* pq = reinterpret_cast<uint32_t*>(ring + (NWC + 1) * RING);
    const int QR = p.qrows;  // profile ring rows (power of two)
    const int QS = QR + LK_QMIRROR;
    const unsigned qmask = (unsigned)QR - 1u;
    const int K = p.K;
    int8_t* stab = reinterpret_cast<int8_t*>(pq + (size_t)K * QS);  // [K][32]: sub'(x, c) at x*32 + c
    unsigned* abort_sh = cnt + LK_ABORT;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
    if (threadIdx.x < 32) reinterpret_cast<unsigned*>(smem + LK_ZERO_OFF)[threadIdx.x] = 0u;  // the zero block
    for (int q = threadIdx.x; q < K * K; q += blockDim.x) stab[(q / K) * 32 + q % K] = (int8_t)p.subp[q];
    __syncthreads();
    if (threadIdx.x == 0) cnt[LK_SLAB] = lane_slab(p);
    __syncthreads();
    const int g = __builtin_amdgcn_readfirstlane((int)cnt[LK_SLAB]);
    const int m = p.m, o = p.o;
    const int nsteps = m + 63;  // lane 63 reaches row m at step m + 62
    // 16-step windows (pairs of sub-chunks); with traceback words the last aligned word
    // (ceil(m/16) - 1) leaves lanes 48..63 at window ceil(m/16) + 3 (LkRot)
    const int tca = (m + 15) / 16;
    const int nwin = CB > 0 ? tca + 4 : (nsteps + 15) / 16;
    const int nlive = min(NWC, p.nstripes - g * NWC);

    // the IO and profile waves share SIMDs with compute waves (priority 2): at a lower priority they issue only
    // when their compute wave stalls, which delays hand-offs and profile rows (GA_LANE_IOPRIO, experiments)
    auto io_prio = [&]() {
        if (p.io_prio >= 3) __builtin_amdgcn_s_setprio(3);
        else if (p.io_prio == 2) __builtin_amdgcn_s_setprio(2);
        else if (p.io_prio == 1) __builtin_amdgcn_s_setprio(1);
    };
    // the out-path (the last compute wave's ring -> HBM) runs in a wave of its own when the workgroup has one
    // (OUTW, p.out_wave): in the IO wave a pass waited behind every in-path poll's round trip
    const bool own_out = OUTW && p.out_wave;
    const bool last_slab = g == p.nslabs - 1;
    const bool out_sent = !(last_slab && p.edge_out != nullptr);
    // one out-path pass: up to 192 rows from the last compute wave's ring to HBM; true if it moved any
    auto out_pass = [&](unsigned& out_next) -> bool {
        int2* dst = out_sent ? p.hand + (long long)g * (m + 1) : p.edge_out;
        const int2* rout = ring + nlive * RING;
        if (out_sent && p.hand_direct) {
            // the last compute wave stores its right edge to the hand-off rows itself (sub_chunk): only
            // its ring slots are freed here
            const unsigned P = lds_ld(&cnt[2 * nlive - 1]);
            if (P > out_next) {
                lds_st(&cnt[2 * nlive], P);
                out_next = min(P, (unsigned)m);
                return true;
            }
            return false;
        }
        const unsigned P = lds_ld(&cnt[2 * nlive - 1]);
        // up to 192 rows a pass
        const unsigned hi = min(min(P, (unsigned)m), out_next + 192);
        if (hi > out_next && (hi - out_next >= GOUT || hi == (unsigned)m)) {
#pragma unroll
            for (int h = 0; h < 3; h++) {
                const unsigned r = out_next + 1 + lane + 64 * h;
                if (r <= hi) {
                    const int2 e = rout[(r - 1) & RMASK];
                    if (out_sent && p.hand_scope < 2) g_st64(dst + r, e);
                    else s_st64(dst + r, e);  // another GPU's halo
                    if (last_slab && r == (unsigned)m && p.n % (64 * TD) == 0) p.out_last[0] = e.x;
                }
            }
            if (!out_sent) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(p.edge_prog, hi, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (lane == 0) lds_st(&cnt[2 * nlive], hi);
            if (DBG && lane == 0 && out_next < (unsigned)(m / 2) && hi >= (unsigned)(m / 2))
                p.dbg[LK_DBG_WORDS * (g * NWC + nlive - 1) + 11] = __builtin_amdgcn_s_memrealtime();
            out_next = hi;
            return true;
        }
        return false;
    };
    if (OUTW && w == NWC + 2) {
        // ---------------- out wave ----------------
        if (!own_out) return;
        io_prio();
        unsigned out_next = 0, spins = 0;
        while (out_next < (unsigned)m) {
            if (out_pass(out_next)) {
                spins = 0;
            } else {
                if (__hip_atomic_load(abort_sh, RLX, WGS)) {
                    g_st(p.abort_word, 1u);
                    break;
                }
                if (!spin_ok(spins, p.spin_limit, p.abort_word)) {
                    __hip_atomic_store(abort_sh, 1u, RLX, WGS);
                    break;
                }
            }
        }
        // gave up before the right edge was complete: tell the reader of the edge (the next slab's fill)
        if (!out_sent && out_next < (unsigned)m && p.edge_prog != nullptr && lane == 0) s_prog_abort(p.edge_prog);
        return;
    }
    if (w == NWC) {
        // ---------------- IO wave: edges HBM -> LDS ring (and LDS ring -> HBM without an out wave) ----------------
        io_prio();
        const int2* src = g == 0 ? p.left : p.hand + (long long)(g - 1) * (m + 1);
        const unsigned* src_prog = g == 0 ? p.left_prog : nullptr;
        const unsigned limit = (g == 0 && p.left_prog != nullptr) ? p.halo_spin_limit : p.spin_limit;
        const bool src_sc1 = p.left_prog != nullptr;
        int2* rin0 = ring;
        const bool in_sent = g > 0;
        unsigned in_next = 0, out_next = own_out ? (unsigned)m : 0u, spins = 0, in_win = 192;
        while (in_next < (unsigned)m || out_next < (unsigned)m) {
            bool moved = false;
            if (in_next < (unsigned)m && in_sent) {
                const unsigned cap = min(min(lds_ld(&cnt[0]) + RING, (unsigned)m), in_next + in_win);
                if (cap > in_next) {
                    // one sc1 round trip per poll; while the writer is behind, its next 16 rows (the writer's
                    // last compute wave stores a 16-step sub-chunk's rows at a time), else up to 192 (three loads
                    // per lane in flight together): the chain writes a row every ~40 ns and a round trip under load
                    // takes 1-3 us, so a 64-row poll fell behind on some links and their lag grew over the whole
                    // fill (lane stamps: end lags up to 128 us at workgroup boundaries)
                    const unsigned r = in_next + 1 + lane;
                    // (GA_LANE_HANDSCOPE >= 1: system-scope loads, past every cache, for the experiments)
                    auto hld = [&](const int2* a) { return unpack64(p.hand_scope ? s_ld64(a) : g_ld64(a)); };
                    const int2 e1 = r <= cap ? hld(src + r) : make_int2(HAND_SENT, 0);
                    const int2 e2 = r + 64 <= cap ? hld(src + r + 64) : make_int2(HAND_SENT, 0);
                    const int2 e3 = r + 128 <= cap ? hld(src + r + 128) : make_int2(HAND_SENT, 0);
                    const unsigned long long ok1 = __ballot(e1.x != HAND_SENT), ok2 = __ballot(e2.x != HAND_SENT),
                                             ok3 = __ballot(e3.x != HAND_SENT);
                    unsigned k = ~ok1 ? (unsigned)__builtin_ctzll(~ok1) : 64u;
                    if (k == 64u) k += ~ok2 ? (unsigned)__builtin_ctzll(~ok2) : 64u;
                    if (k == 128u) k += ~ok3 ? (unsigned)__builtin_ctzll(~ok3) : 64u;
                    in_win = p.poll_win > 0 ? (unsigned)p.poll_win : k >= cap - in_next ? 192u : 16u;
                    if (k > 0) {
                        if (lane < (int)k) rin0[(r - 1) & RMASK] = e1;
                        if (lane + 64 < (int)k) rin0[(r + 63) & RMASK] = e2;
                        if (lane + 128 < (int)k) rin0[(r + 127) & RMASK] = e3;
                        const unsigned hi = in_next + k;
                        if (lane == 0) lds_st(&cnt[LK_PROD0], hi == (unsigned)m ? LK_DONE : hi);
                        if (DBG && lane == 0 && in_next < (unsigned)(m / 2) && hi >= (unsigned)(m / 2))
                            p.dbg[LK_DBG_WORDS * (g * NWC) + 10] = __builtin_amdgcn_s_memrealtime();
                        in_next = hi;
                        moved = true;
                    }
                }
            } else if (in_next < (unsigned)m) {
                const unsigned space = lds_ld(&cnt[0]) + RING;
                const unsigned pv = src_prog ? s_ld(src_prog) : (unsigned)m;
                if (pv == PROG_ABORT) {  // the left neighbour's fill gave up
                    __hip_atomic_store(abort_sh, 1u, RLX, WGS);
                    g_st(p.abort_word, 1u);
                    break;
                }
                const unsigned avail = min(pv, (unsigned)m);
                const unsigned hi = min(min(space, avail), in_next + 64);
                if (hi > in_next && (hi - in_next >= 16 || hi == avail)) {
                    const unsigned r = in_next + 1 + lane;
                    if (r <= hi) rin0[(r - 1) & RMASK] = src_sc1 ? unpack64(s_ld64(src + r)) : src[r];
                    if (lane == 0) lds_st(&cnt[LK_PROD0], hi == (unsigned)m ? LK_DONE : hi);
                    in_next = hi;
                    moved = true;
                }
            }
            // (a pass here waits for the in-path's poll round trip too)
            if (out_next < (unsigned)m && out_pass(out_next)) moved = true;
            if (!moved) {
                if (__hip_atomic_load(abort_sh, RLX, WGS)) {
                    g_st(p.abort_word, 1u);
                    break;
                }
                if (!spin_ok(spins, limit, p.abort_word)) {
                    __hip_atomic_store(abort_sh, 1u, RLX, WGS);
                    break;
                }
            } else {
                spins = 0;
            }
        }
        // gave up before the right edge was complete: tell the reader of the edge (the next slab's fill)
        if (!own_out && !out_sent && out_next < (unsigned)m && p.edge_prog != nullptr && lane == 0)
            s_prog_abort(p.edge_prog);
        return;
    }
    if (w == NWC + 1) {
        // ---------------- profile wave: the LDS query-profile table, ahead of the slowest compute wave.  A wave
        // of its own (round 3: the IO wave's), so that the hand-off rows never wait behind it: for a 24-code
        // alphabet the table's 64-row batches held the IO wave long enough to triple the cross-workgroup lag
        // (28 us against 8.5 for DNA, profiles/r03/lane_stamps_c5_shape.jsonl)
        io_prio();
        // dword row r of code c: sub'(a_r .. a_r+3, c), rows outside 1..m zero.  A lane's window
        // may start up to 3 rows above row 1 (its first sub-chunk), so rows -2..0 are written too.
        auto put_dword = [&](int r) {
            int x[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                ok[u] = r + u >= 1 && r + u <= m;
                x[u] = ok[u] ? p.a[r + u - 1] : 0;
            }
            const unsigned slot = (unsigned)(r - 1) & qmask;
            for (int c = 0; c < K; c++) {
                uint32_t v = 0;
#pragma unroll
                for (int u = 0; u < 4; u++) v |= ok[u] ? (uint32_t)(uint8_t)stab[x[u] * 32 + c] << (8 * u) : 0u;
                pq[c * QS + slot] = v;
                if (slot < (unsigned)LK_QMIRROR) pq[c * QS + QR + slot] = v;
            }
        };
        // the precomputed profile (p.qprof): K dword loads and LDS stores per lane per 64 rows, loads in flight together
        const int qpitch = m + 4;
        auto copy_dword = [&](int r) {
            const unsigned slot = (unsigned)(r - 1) & qmask;
            const uint32_t* src = p.qprof + (r + 2);
            for (int c0 = 0; c0 < K; c0 += 8) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = c0 + u < K ? src[(long long)(c0 + u) * qpitch] : 0u;
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    if (c0 + u < K) {
                        pq[(c0 + u) * QS + slot] = v[u];
                        if (slot < (unsigned)LK_QMIRROR) pq[(c0 + u) * QS + QR + slot] = v[u];
                    }
                }
            }
        };
        if (lane < 3) {
            if (p.qprof) copy_dword(lane - 2);
            else put_dword(lane - 2);
        } else if (p.lean0) {
            // the lean ramp (lean0): lanes still above row 1 read the dwords of rows -63 .. -3 too (lane L writes dword
            // L - 66), all zero bytes, so that their steps keep row 0's values; with dwords -2 .. 0 they fill the ring's
            // last 64 slots, which rows QR - 63 .. QR reuse only once every wave is past its first 64 steps (below)
            const unsigned slot = (unsigned)(lane - 67) & qmask;
            for (int c = 0; c < K; c++) pq[c * QS + slot] = 0u;
        }
        unsigned q_next = 0, spins = 0;
        while (q_next < (unsigned)m) {
            // the slowest wave reads rows above (its output rows) - 16, so slots of rows below that + QR are free;
            // lean0: until it has published a row (its lanes all past row 0) the ring's last 64 slots hold the zero rows
            const unsigned pl = lds_ld(&cnt[2 * nlive - 1]);
            const unsigned space = p.lean0 && pl == 0u ? (unsigned)QR - 64u : (pl > 32u ? pl - 32u : 0u) + (unsigned)QR;
            const unsigned hi = min(min(space, (unsigned)m), q_next + 64);
            if (hi > q_next && (hi - q_next >= 64 || hi == (unsigned)m)) {
                const unsigned r = q_next + 1 + lane;
                if (r <= hi) {
                    if (p.qprof) copy_dword((int)r);
                    else put_dword((int)r);
                }
                if (lane == 0) lds_st(&cnt[LK_PRODQ], hi == (unsigned)m ? LK_DONE : hi);
                q_next = hi;
                spins = 0;
            } else {
                if (__hip_atomic_load(abort_sh, RLX, WGS)) break;
                if (!spin_ok(spins, p.spin_limit, p.abort_word)) {
                    __hip_atomic_store(abort_sh, 1u, RLX, WGS);
                    break;
                }
            }
        }
        return;
    }
    if (w >= nlive) return;

    // ---------------- compute wave w: stripe s, columns j0+1 .. j0+64*TD ----------------
    __builtin_amdgcn_s_setprio(2);
    const int s = g * NWC + w;
    const int j0 = s * 64 * TD;
    const int jl = j0 + lane * TD;  // this lane: columns jl+1 .. jl+TD
    const bool partial = j0 + 64 * TD > p.n;
    const int cn = p.n - 1 - j0;    // column n's offset in a partial stripe
    const int tm = partial ? m - 1 + cn / TD : -1;  // the step at which its lane reaches row m
    const int ck = cn % TD;
    int Hm = 0;
    int H[TD], Y[TD];
    unsigned qb[TD];  // dword index of each column's code row in the profile table
#pragma unroll
    for (int k = 0; k < TD; k++) {
        const int jc = jl + k + 1;
        const bool ok = jc <= p.n;
        const int2 t = p.top[ok ? jc : p.n];
        H[k] = t.x;  // H'(0, j) until the lane reaches row 1
        Y[k] = t.y;  // h2'(0, j)
        qb[k] = (unsigned)((ok ? p.b[jc - 1] : 0) * QS);
    }
    // traceback words: column (lane, k) is lane p = (lane*TD + k) mod 64 of 64-column stripe
    // TD*s + (lane*TD + k) / 64 (as for fill_kernel's blocked stripes)
    constexpr int CBX = CB > 0 ? CB : 1;
    uint32_t acc[TD][4 * CBX], prevw[TD][4 * CBX];
    uint4* colw[TD];
    LkRot<TD, CBX> rot;
    const unsigned op1 = (unsigned)o + 1u;
    if constexpr (CB > 0) {
        rot.init(lane & 15);
#pragma unroll
        for (int k = 0; k < TD; k++) {
            const int c = lane * TD + k;
            colw[k] = reinterpret_cast<uint4*>(p.tb) + ((long long)(TD * s + c / 64) * p.TC) * 64 + (c & 63);
#pragma unroll
            for (int d = 0; d < 4 * CBX; d++) prevw[k][d] = 0;
        }
    }
    int HLp = p.top[min(jl, p.n)].x;  // lane 0: H'(0, j0), the diagonal of row 1
    // (lean0: the h1' a lane above row 1 hands right must not undercut row 0's H' = o, so it starts at 2o)
    int Hl = H[TD - 1], Xl = p.lean0 ? 2 * o : 0, RH = 0, RX = 0;
    const int2* rin = ring + w * RING;
    int2* rout = ring + (w + 1) * RING;
    // the hand-scheduled asm step (ga_lane_asm.h) for the unmasked sub-chunks of the score-only fills
    // (not at 8 waves per workgroup with TD >= 4: the register budget of 640-thread workgroups cannot hold the
    // lean sub-chunk, and register allocation then runs for tens of minutes)
    constexpr bool ASMOK = CB == 0 && !CKP && SUB == 16 && (NWC == 4 || TD <= 2);
    const bool use_asm = ASMOK && p.asm_step;
    unsigned* prod_in = w == 0 ? &cnt[LK_PROD0] : &cnt[2 * w - 1];
    // the workgroup's last compute wave writes the hand-off rows (not a slab's halo to another GPU, which
    // the IO wave streams with its progress word)
    const bool last_slab_w = g == p.nslabs - 1;
    const bool hand_direct = p.hand_direct && w == nlive - 1 && !(last_slab_w && p.edge_out != nullptr);
    int2* hand_out = p.hand + (long long)g * (m + 1);
    const bool last_full = last_slab_w && p.n % (64 * TD) == 0;
    unsigned* cons_out = &cnt[2 * w + 2];
    unsigned pc_lds = lds_addr(&cnt[2 * w]);  // {cons(w), prod(w + 1)}: one 8-byte store
    const unsigned rout_lds = lds_addr(rout);
    // the recompute checkpoints' right edge of this stripe, and a scratch slot per lane past all of them
    int2* const colck_s = RC && p.colck != nullptr ? p.colck + (long long)s * (m + 1 + COLCK_PAD) : nullptr;
    int2* const colck_x = RC && p.colck != nullptr ? colck_s + (m + 1 + lane) : nullptr;
    // the lean steady state's checkpoint store: a raw buffer over the stripe's rows (base and size in SGPRs) and a
    // 32-bit offset per lane, rows rlo + lane - 48 for lanes 48..63 (LEAN sub-chunks hold no row past m), off the
    // buffer's end for the others, whose stores the buffer's range check then drops: no exec change, and no scratch
    // writes (they were three quarters of the store's bytes); off = cb + 8 rlo for every lane, one v_add with an
    // SGPR (a per-lane multiplier took a 64-bit v_mad_u64_u32): the other lanes' 0x7ffffff0 + 8 rlo stays past
    // the buffer's (m + 1) * 8 bytes and below 2^32 while rc_rows_fit(m) (ga_check.h), which the host requires
    const unsigned ck_cb = lane >= 48 ? (unsigned)(lane - 48) * 8u : 0x7ffffff0u;
    lk_v4i ck_rsrc = {0, 0, 0, 0};
    if (RC && p.colck != nullptr) {
        const unsigned long long cbase = reinterpret_cast<unsigned long long>(colck_s);
        ck_rsrc = lk_v4i{(int)sgpr_u((unsigned)cbase), (int)(sgpr_u((unsigned)(cbase >> 32)) & 0xffffu),
                         (int)sgpr_u((unsigned)(m + 1) * 8u), 0x00020000};  // stride 0, num_records, gfx9 dword 3
    }
    unsigned avail = 0, outfree = 0, qavail = 0;
    bool aborted = false;
    unsigned long long wcyc[3] = {0, 0, 0}, t_start = 0, c_start = 0;
    // DBG probe (row m/2): when this wave knew its edge row m/2 had landed, when it published its own row m/2
    unsigned long long t_avail = 0, t_pub = 0;
    if (DBG) {
        t_start = __builtin_amdgcn_s_memrealtime();
        c_start = __builtin_amdgcn_s_memtime();
    }
    // DBG: when the wave started the sub-chunks of rows 256, 1024, 4096 and 16384 (how the lag between two stripes
    // grows along the rows: tools/lane_stamps.py "lag_by_row")
    unsigned long long t_rows[6] = {0, 0, 0, 0, 0, 0};
    auto dbg_rows = [&](int r0) {
        if (r0 == 64) t_rows[4] = __builtin_amdgcn_s_memrealtime();
        if (r0 == 128) t_rows[5] = __builtin_amdgcn_s_memrealtime();
        if (r0 == 256) t_rows[0] = __builtin_amdgcn_s_memrealtime();
        if (r0 == 1024) t_rows[1] = __builtin_amdgcn_s_memrealtime();
        if (r0 == 4096) t_rows[2] = __builtin_amdgcn_s_memrealtime();
        if (r0 == 16384) t_rows[3] = __builtin_amdgcn_s_memrealtime();
    };
    auto wait_ge = [&](unsigned* ctr, unsigned add, unsigned& cached, int target, int kind) {
        unsigned spins = 0;
        cached = sgpr_u(cached);
        unsigned long long t0 = 0;
        if (DBG && (int)cached < target) t0 = __builtin_amdgcn_s_memtime();
        while ((int)cached < target && !aborted) {
            cached = lds_ldu(ctr) + add;
            if ((int)cached >= target) break;
            if (!spin_ok_lds(spins, p.spin_limit, abort_sh)) aborted = true;
        }
        if (DBG && t0) wcyc[kind] += __builtin_amdgcn_s_memtime() - t0;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    };
    // sub-chunk 0: lane 0's rows 1..SUB (slots 0..SUB-1), the lanes' profile windows
    constexpr int NE = SUB / 2;  // int4 edge registers per sub-chunk: (H', h1') of two rows each
    constexpr int NQ = SUB / 4;  // profile dwords per column per sub-chunk: four rows each
    int4 A[NE], B[NE];
    uint32_t qA[TD][NQ], qB[TD][NQ];
    wait_ge(prod_in, 0, avail, SUB, 0);
    // DBG: the first wait is the chain's ramp (a stripe's left neighbour has not reached row SUB yet), not a stall
    // of the steady state
    unsigned long long w_first = 0, t_first = 0;
    if (DBG) {
        w_first = wcyc[0];
        t_first = __builtin_amdgcn_s_memrealtime();
    }
    // the edge rows: lane 0 reads them from the ring, lanes 1..63 read the zero block (the asm step adds the
    // edge register to the zero-filled DPP shift; the compiler's step takes lane 0's value only)
    const int4* const ezero = reinterpret_cast<const int4*>(smem + LK_ZERO_OFF);
    // the lean sub-chunk's LDS addresses: the producer's counter, the profile table, a scratch slot per lane (the
    // all-lane row stores of lanes that carry no row)
    const unsigned ca_lds = lds_addr(prod_in);
    const unsigned pq_lds = lds_addr(pq);
    const unsigned scr_lds = lds_addr(smem + LK_SCR_OFF);
    // ... and their loop-invariant per-lane parts, so that a sub-chunk's addresses cost one op each (round 5: the
    // compiler's forms took 27 instructions between two lean statements): the profile rows q4[k] + ((4 r - 4 lane) &
    // 4 qmask); the edge rows (ea_s & ea_m) | ea_b (lane 0 the ring's rows, the others the zero block); the row stores
    // ((8 x + 8 lane) & w?_m) + w?_b (lanes 48..63 their ring slot, the others a scratch slot of their own)
    unsigned q4[TD], ea_m, ea_b, wa_m, wa_b, wb_m, wb_b;
    {
#pragma unroll
        for (int k = 0; k < TD; k++) q4[k] = pq_lds + 4u * qb[k];
        const unsigned scr = scr_lds + 8u * (unsigned)lane, rout_l = lds_addr(rin + RING);
        const bool hi = lane >= 48;
        ea_m = lane == 0 ? ~0u : 0u;
        ea_b = lane == 0 ? 0u : lds_addr(ezero);
        wa_m = hi && (lane & 4) ? 8u * RMASK : 0u;
        wa_b = hi && (lane & 4) ? rout_l : scr;
        wb_m = hi && !(lane & 4) ? 8u * RMASK : 0u;
        wb_b = hi && !(lane & 4) ? rout_l : scr;
    }
    {
        const int4* src = lane == 0 ? reinterpret_cast<const int4*>(rin) : ezero;
#pragma unroll
        for (int k = 0; k < NE; k++) A[k] = src[k];
    }
    wait_ge(&cnt[LK_PRODQ], 0, qavail, SUB, 1);
    {
        const unsigned idx = (unsigned)(-lane) & qmask;
#pragma unroll
        for (int k = 0; k < TD; k++)
#pragma unroll
            for (int d = 0; d < NQ; d++) qA[k][d] = pq[qb[k] + idx + 4 * d];
    }
    unsigned pnext = *prod_in;  // the producer's counter, read a sub-chunk before it is needed
    // the banded traceback's score pass: the next checkpoint row any lane may still reach
    int next_ck = CKP ? p.ckpt_rows : 0x7fffffff;
    // the step of a sub-chunk at which score-only waves await and read the next sub-chunk's edges
    // (0: after the first step, as the traceback variants do)
    constexpr int LE = (CB == 0 && !CKP && SUB == 16 && LATE) ? GA_LANE_LE : 0;

    // one SUB-step sub-chunk: steps r0 .. r0+SUB-1 from C / qc; after its first step the next
    // sub-chunk's edges, profile windows and the producer's counter are read into Nx / qx / pnext (they
    // land while the other steps run); then lanes 64-SUB..63 store lane 63's SUB rows and lane 0
    // publishes {cons(w) = r0 + 2 SUB, prod(w + 1)} in one 8-byte store
    // LEAN (the steady state of the lean sub-chunk, see the main loop): the sub-chunk is known unmasked and lean, so no
    // per-sub-chunk test of r0 / tm / the knobs sits between the statements
    auto sub_chunk = [&](int r0, int4 (&C)[NE], int4 (&Nx)[NE], uint32_t (&qc)[TD][NQ], uint32_t (&qx)[TD][NQ],
                         auto HALF, auto LEANT) {
        constexpr int HB = decltype(HALF)::value * SUB;  // the sub-chunk's first step in its 16-step window
        constexpr bool LEAN = decltype(LEANT)::value;
        if (!LE) {
            avail = sgpr_u(max(avail, pnext));
            if ((int)avail < r0 + 2 * SUB) wait_ge(prod_in, 0, avail, r0 + 2 * SUB, 0);
        }
        if ((int)qavail < r0 + 2 * SUB) wait_ge(&cnt[LK_PRODQ], 0, qavail, r0 + 2 * SUB, 1);
        int eh[SUB], ex[SUB];
#pragma unroll
        for (int k = 0; k < NE; k++) {
            eh[2 * k] = C[k].x; ex[2 * k] = C[k].y; eh[2 * k + 1] = C[k].z; ex[2 * k + 1] = C[k].w;
        }
        // the next sub-chunk's profile windows (the IO wave fills them far ahead) after the first step
        auto qloads = [&]() {
            asm volatile("" ::: "memory");
            const unsigned idx = (unsigned)(r0 + SUB - lane) & qmask;
#pragma unroll
            for (int k = 0; k < TD; k++)
#pragma unroll
                for (int d = 0; d < NQ; d++) qx[k][d] = pq[qb[k] + idx + 4 * d];
            asm volatile("" ::: "memory");
        };
        // its left-edge rows and the producer's counter: after the first step, or (LE) only LE steps into
        // the sub-chunk, awaiting them there -- the stripe then trails its left neighbour by SUB - LE
        // steps less (the LDS read still lands SUB - LE steps before its first use)
        auto eloads = [&]() {
            asm volatile("" ::: "memory");
            if (LE) {
                avail = sgpr_u(max(avail, pnext));
                if ((int)avail < r0 + 2 * SUB) wait_ge(prod_in, 0, avail, r0 + 2 * SUB, 0);
            }
            {
                const int4* src = lane == 0 ? reinterpret_cast<const int4*>(rin + ((r0 + SUB) & RMASK)) : ezero;
#pragma unroll
                for (int k = 0; k < NE; k++) Nx[k] = src[k];
            }
            pnext = __hip_atomic_load(prod_in, RLX, WGS);
            asm volatile("" ::: "memory");
        };
        const int row0 = r0 - lane + 1;
        const bool capl = lane == cn / TD;
        // checkpoint row (banded traceback's score pass): the multiple of ckpt_rows
        // (>= 16 = SUB, so at most one) among this lane's rows of the sub-chunk, and the step it falls on
        int cku = -1;
        int2* ckr = nullptr;
        auto ck_find = [&]() {
            const int top = row0 + SUB - 1, ckrow = top >= p.ckpt_rows ? top - top % p.ckpt_rows : 0;
            if (ckrow >= row0 && ckrow >= p.ckpt_rows && ckrow < m) {
                cku = ckrow - row0;
                ckr = p.ckpt + (long long)(ckrow / p.ckpt_rows - 1) * (p.n + 1);
            }
        };
        auto steps = [&](auto MK, auto CKV) {
            constexpr bool MASKED = decltype(MK)::value;
            constexpr bool CKS = decltype(CKV)::value;
            auto one = [&](auto UC) {
                constexpr int u = decltype(UC)::value;
                uint32_t qq[TD];
#pragma unroll
                for (int k = 0; k < TD; k++) qq[k] = qc[k][u >> 2];
                lane_step<TD, u & 3, CB, (HB + u) & 15, MASKED>(H, Y, Xl, Hl, HLp, RH, RX, eh[u], ex[u], qq, o, acc,
                                                               op1, row0 + u, capl && r0 + u == tm, ck, Hm);
                if constexpr (CKS) {
                    if (cku == u) {
#pragma unroll
                        for (int k = 0; k < TD; k++)
                            if (jl + k + 1 <= p.n) ckr[jl + k + 1] = make_int2(H[k], Y[k]);
                    }
                }
            };
            one(std::integral_constant<int, 0>{});
            qloads();
            if constexpr (LE > 0) {
                LkUnroll<1, LE>::run(one);
                eloads();
                LkUnroll<LE, SUB>::run(one);
            } else {
                eloads();
                LkUnroll<1, SUB>::run(one);
            }
        };
        // wave-uniform: does any lane's window hold the next checkpoint row (lanes hold rows r0-62 .. r0+SUB)?
        const bool ckw = CKP && next_ck <= r0 + SUB;
        if (ckw) ck_find();
        // once lane 63's next window starts past it, the following multiple
        if (CKP && next_ck < r0 + SUB - 62) next_ck += p.ckpt_rows;
        if constexpr (CKP) {
            if (r0 < 64 || (unsigned)(tm - r0) < (unsigned)SUB) {
                if (ckw) steps(std::true_type{}, std::true_type{});
                else steps(std::true_type{}, std::false_type{});
            } else if (ckw) {
                steps(std::false_type{}, std::true_type{});
            } else {
                steps(std::false_type{}, std::false_type{});
            }
        } else {
            // (lean0, a uniform row 0: the first 64 steps need no mask either, for the asm statement; see it_lo below)
            const bool masked = !LEAN && ((r0 < 64 && !(p.lean0 && use_asm)) || (unsigned)(tm - r0) < (unsigned)SUB);
            if constexpr (ASMOK) {
                if (LEAN || (use_asm && !masked && !hand_direct)) {
                    // The lean sub-chunk: the 16 steps, the next sub-chunk's profile and edge reads
                    // and lane 63's rows out as ONE asm statement (LaneSub, ga_lane_asm.h), so that no compiler code,
                    // copy or conservative wait sits between the steps.  Lane 63's rows go out by DPP moves into
                    // lanes 48..63 and two all-lane ds_write2_b32 (1 + 2 LDS writes instead of 17); the producer's
                    // counter is read just before the edge rows, so a counter that covers them proves them (LDS
                    // executes a wave's operations in order, the producer writes rows before its counter) and only a
                    // producer that really is behind costs a poll and a re-read.
                    const int rlo = r0 - 62;
                    // (a wave-uniform test: compared in a VGPR, the compiler masked exec around the wait, twice a sub-chunk)
                    outfree = sgpr_u(outfree);
                    if ((int)outfree < rlo + SUB - 1) wait_ge(cons_out, RING, outfree, rlo + SUB - 1, 2);
                    lk_v4i Ev[NE];
#pragma unroll
                    for (int k = 0; k < NE; k++) Ev[k] = lk_v4i{C[k].x, C[k].y, C[k].z, C[k].w};
                    // (the invariant parts above; the asm forms keep the compiler from re-deriving them)
                    unsigned ea, qi4, wt, wa, wb, qbv[TD];
                    const unsigned ea_s = lds_addr(rin) + 8u * ((unsigned)(r0 + SUB) & RMASK);
                    asm volatile("v_and_or_b32 %0, %1, %2, %3" : "=v"(ea) : "s"(ea_s), "v"(ea_m), "v"(ea_b));
                    asm volatile("v_sub_u32 %0, %1, %2" : "=v"(qi4) : "s"(4u * (unsigned)(r0 + SUB)), "v"(4u * (unsigned)lane));
                    qi4 &= 4u * qmask;
#pragma unroll
                    for (int k = 0; k < TD; k++) asm volatile("v_add_u32 %0, %1, %2" : "=v"(qbv[k]) : "v"(q4[k]), "v"(qi4));
                    asm volatile("v_add_u32 %0, %1, %2" : "=v"(wt) : "s"(8u * (unsigned)(rlo - 49)), "v"(8u * (unsigned)lane));
                    wa = (wt & wa_m) + wa_b;
                    wb = (wt & wb_m) + wb_b;
                    const unsigned wc = lane == 0 ? pc_lds : scr_lds + 8u * (unsigned)lane;
                    const bool hi = lane >= 48;
                    const lk_v2u cp = {(unsigned)(r0 + 2 * SUB), (unsigned)max(rlo + SUB - 1, 0)};
                    unsigned cv;
                    lk_v4i En[NE];
                    lk_v2u qn[TD][2];
                    int R[4];
                    LaneSub<TD, LE ? 12 : 0>::run(H, Y, Xl, HLp, Ev, qc, o, ca_lds, ea, qbv, wa, wb, wc, cp, cv, En, qn, R);
                    Hl = H[TD - 1];
                    if (DBG && rlo <= m / 2 && m / 2 < rlo + SUB) t_pub = __builtin_amdgcn_s_memrealtime();
                    const int need = min(r0 + 2 * SUB, m);
                    if ((int)sgpr_u(cv) < need) {
                        wait_ge(prod_in, 0, avail, need, 0);
                        asm volatile("" ::: "memory");
                        const int4* src = lane == 0 ? reinterpret_cast<const int4*>(rin + ((r0 + SUB) & RMASK)) : ezero;
#pragma unroll
                        for (int k = 0; k < NE; k++) Nx[k] = src[k];
                        // landed inside this branch, so that the compiler's wait is not at the merge (where it would
                        // also wait for the lean statement's row stores on every sub-chunk)
#pragma unroll
                        for (int k = 0; k < NE; k++) asm volatile("" ::"v"(Nx[k].x), "v"(Nx[k].y), "v"(Nx[k].z), "v"(Nx[k].w));
                    } else {
#pragma unroll
                        for (int k = 0; k < NE; k++) Nx[k] = make_int4(En[k].x, En[k].y, En[k].z, En[k].w);
                    }
                    if (DBG && r0 + SUB < m / 2 && m / 2 <= r0 + 2 * SUB) t_avail = __builtin_amdgcn_s_memrealtime();
#pragma unroll
                    for (int k = 0; k < TD; k++) {
                        qx[k][0] = qn[k][0].x;
                        qx[k][1] = qn[k][0].y;
                        qx[k][2] = qn[k][1].x;
                        qx[k][3] = qn[k][1].y;
                    }
                    if (RC && LEAN) {
                        // (colck is set whenever the RC variant runs, enqueue_fill) one offset and one store
                        const lk_v2u vv = (lane & 4) ? lk_v2u{(unsigned)R[0], (unsigned)R[1]} : lk_v2u{(unsigned)R[2], (unsigned)R[3]};
                        const unsigned off = ck_cb + sgpr_u(8u * (unsigned)rlo);
                        asm volatile("buffer_store_dwordx2 %1, %0, %2, 0 offen" ::"v"(off), "v"(vv), "s"(ck_rsrc) : "memory");
                    } else if (RC && p.colck != nullptr) {
                        // lanes 48..63 hold rows rlo .. rlo+15 of the stripe's right edge; every lane stores (lanes
                        // without a row into the scratch slots past the checkpoints): no exec change, which would
                        // drain the VALU pipeline on every sub-chunk (the direct hand-off takes the compiler's steps)
                        const int row = rlo + lane - 48;
                        const int2 v = (lane & 4) ? make_int2(R[0], R[1]) : make_int2(R[2], R[3]);
                        // one 8-byte store in asm: the compiler split `*p = v` into two dword stores and put the second
                        // under an exec mask
                        int2* const cdst = hi && row <= m ? colck_s + row : colck_x;
                        const lk_v2u vv = {(unsigned)v.x, (unsigned)v.y};
                        asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(cdst), "v"(vv) : "memory");
                    }
                    return;
                }
            }
            if constexpr (!LEAN) {
                if (masked) steps(std::true_type{}, std::false_type{});
                else steps(std::false_type{}, std::false_type{});
            }
        }
        if constexpr (!LEAN) {
        // lane 63 computed rows r0-62 .. r0-63+SUB; lanes 64-SUB..63 of the shift registers hold them
        const int rlo = r0 - 62;
        if ((int)outfree < rlo + SUB - 1) wait_ge(cons_out, RING, outfree, rlo + SUB - 1, 2);
        const unsigned oaddr = rout_lds + (unsigned)((rlo - 1 - (64 - SUB) + lane) & RMASK) * 8u;
        typedef int v2i_t __attribute__((ext_vector_type(2)));
        const v2i_t hx = {RH, RX};
        const lk_v2u cp = {(unsigned)(r0 + 2 * SUB), (unsigned)max(rlo + SUB - 1, 0)};
        unsigned long long saved;
        const unsigned pcl = pc_lds;            // (a generic lambda's asm operands must be its own locals)
        // exec = lanes 64-SUB .. 63 as literals (an SGPR operand for the mask was given a VGPR pair in the TD 8 variant
        // once the lean steady state doubled the loop body)
        asm volatile(
            "s_mov_b64 %0, exec\n\t"
            "s_mov_b32 exec_lo, 0\n\t"
            "s_mov_b32 exec_hi, %4\n\t"
            "ds_write_b64 %1, %2\n\t"
            "s_mov_b64 exec, 1\n\t"
            "ds_write_b64 %3, %5\n\t"
            "s_mov_b64 exec, %0\n\t"
            "s_nop 4"
            : "=&s"(saved)
            : "v"(oaddr), "v"(hx), "v"(pcl), "n"(SUB == 16 ? (int)0xffff0000u : (int)0xff000000u), "v"(cp)
            : "memory");
        if (hand_direct) {
            // the workgroup's right edge straight to its hand-off rows (agent-scope 8-byte stores, each row
            // one untorn granule the next workgroup's IO wave polls for), 16 rows per sub-chunk
            const int row = rlo + lane - (64 - SUB);
            if (lane >= 64 - SUB && row >= 1 && row <= m) {
                g_st64(hand_out + row, make_int2(RH, RX));
                if (row == m && last_full) p.out_last[0] = RH;  // H'(m, n): the cost
            }
        }
        if constexpr (RC) {
            // lane 64-SUB+u holds row rlo+u of this stripe's right edge
            const int row = rlo + lane - (64 - SUB);
            if (p.colck != nullptr && lane >= 64 - SUB && row >= 1 && row <= m)
                colck_s[row] = make_int2(RH, RX);
        }
        }  // !LEAN
    };
    // traceback words: window w of 16 steps done -> aligned word w - 1 - lane/16 of every column (LkRot)
    auto emit = [&](int win) {
        if constexpr (CB > 0) {
            const int a = win - 1 - (lane >> 4);
            const bool st = a >= 0 && a < tca;
#pragma unroll
            for (int k = 0; k < TD; k++) {
                uint32_t r[4 * CBX];
                rot.rotate(acc[k], r);
                uint32_t wd[4 * CBX];
#pragma unroll
                for (int d = 0; d < 4 * CBX; d++) {
                    wd[d] = (prevw[k][d] & rot.mask[d]) | (r[d] & ~rot.mask[d]);
                    prevw[k][d] = r[d];
                }
                if (st) {
#pragma unroll
                    for (int d = 0; d < CBX; d++)
                        colw[k][(long long)(a * CBX + d) * 64] =
                            make_uint4(wd[4 * d], wd[4 * d + 1], wd[4 * d + 2], wd[4 * d + 3]);
                }
            }
        }
    };
    // whole pairs of sub-chunks (steps past row m compute garbage nobody reads); with traceback
    // words a 16-step window is a pair of 8-step sub-chunks or one 16-step sub-chunk
    static_assert(CB == 0 || SUB == 8 || SUB == 16, "traceback windows are 16 steps");
    const int nit = (16 * nwin + 2 * SUB - 1) / (2 * SUB);
    // The lean sub-chunk's steady state: iterations [it_lo, it_hi) run it with no per-sub-chunk test (from row 64 on, every
    // lane is inside the matrix; a partial stripe's last lane reaches row m at step tm, and the sub-chunks near it are
    // masked); the iterations before and after take the tested path
    // (not at TD 8: the second copy of the loop body pushed the C4 variant past 256 VGPRs into scratch, 6x slower)
    constexpr bool LEANOK = ASMOK && TD <= 4;
    int it_lo = nit, it_hi = nit;
    if constexpr (LEANOK) {
        if (use_asm && !hand_direct) {
            // lean0 (a uniform row 0): from the first iteration.  A lane above row 1 steps on zero profile bytes, so
            // M' = H'(diag) = o, X' >= o (its left lane's h1', which starts at 2o), Y' = 2o: H' = o, h2' = 2o, h1' in
            // [o, 2o] -- row 0's values, unchanged, until the lane reaches row 1.  Otherwise the masked ramp first (the
            // generic path; the first 64 steps of every stripe, on the chain's critical path: round 6)
            it_lo = p.lean0 ? 0 : min(64 / (2 * SUB), nit);
            // every sub-chunk x of [it_lo, it_hi) has x <= tm - SUB: (unsigned)(tm - x) >= SUB
            it_hi = !partial ? nit : tm - 3 * SUB + 1 >= 0 ? min(nit, (tm - 3 * SUB + 1) / (2 * SUB) + 1) : 0;
            // RC: and no row past m in a lean sub-chunk (its checkpoint store does not test): r0 + SUB - 62 + 15 <= m
            if (RC) it_hi = min(it_hi, (m + 31) / (2 * SUB) + 1);
            it_hi = max(it_hi, it_lo);
        }
    }
    if constexpr (LEANOK) {
        // every global load of the prologue (p.top, p.b, ...) landed: said once here, with the intrinsic the compiler's
        // wait insertion understands, since the path around an empty first loop otherwise left them "pending" into the
        // lean loop, whose statements then each waited for every outstanding memory operation (s_waitcnt vmcnt(0))
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        auto iteration = [&](int it, auto LEANT) {
            const int r0 = __builtin_amdgcn_readfirstlane(it * 2 * SUB);
            if (DBG) dbg_rows(r0);
            if (CB > 0 && SUB == 16) {
                sub_chunk(r0, A, B, qA, qB, std::integral_constant<int, 0>{}, LEANT);
                emit(2 * it);
                sub_chunk(r0 + SUB, B, A, qB, qA, std::integral_constant<int, 0>{}, LEANT);
                emit(2 * it + 1);
            } else {
                sub_chunk(r0, A, B, qA, qB, std::integral_constant<int, 0>{}, LEANT);
                sub_chunk(r0 + SUB, B, A, qB, qA, std::integral_constant<int, 1>{}, LEANT);
                emit(it);
            }
            if constexpr (RC) {
                // staircase checkpoint k after step k*E - 1: lane 0 has finished row k*E, lane l row k*E - l
                // (the spacing is a power of two: a mask and a shift, not a division per iteration).  The stores are
                // asm with the checkpoint's base in SGPRs: as compiler stores they made it wait for every outstanding
                // store (s_waitcnt vmcnt(0)) before the next lean statement, i.e. for the checkpoint stores' round trip
                // to memory on every iteration (the recompute fill 0.7 ms slower than the plain one at C3)
                const int done = r0 + 2 * SUB;
                if (p.stck_every > 0 && (done & (p.stck_every - 1)) == 0 && done < m) {
                    const int2* ck = p.stck + ((long long)((done >> p.stck_shift) - 1) * p.nstripes + s) * (TD + 1) * 64;
                    const unsigned loff = (unsigned)lane * 8u;
#pragma unroll
                    for (int k = 0; k <= TD; k++) {
                        const lk_v2u vv = k < TD ? lk_v2u{(unsigned)H[k], (unsigned)Y[k]} : lk_v2u{(unsigned)Xl, (unsigned)HLp};
                        asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3" ::"v"(loff), "v"(vv), "s"(ck), "n"(k * 512)
                                     : "memory");
                    }
                }
            }
        };
        int it = 0;
        for (; it < it_lo; it++) iteration(it, std::false_type{});
        for (; it < it_hi; it++) iteration(it, std::true_type{});
        for (; it < nit; it++) iteration(it, std::false_type{});
    } else {
        // the loop body written out (an extra lambda layer kept the traceback variants' sub-chunks out of line and
        // their register arrays in scratch)
        for (int it = 0; it < nit; it++) {
            const int r0 = __builtin_amdgcn_readfirstlane(it * 2 * SUB);
            if (DBG) dbg_rows(r0);
            if (CB > 0 && SUB == 16) {
                sub_chunk(r0, A, B, qA, qB, std::integral_constant<int, 0>{}, std::false_type{});
                emit(2 * it);
                sub_chunk(r0 + SUB, B, A, qB, qA, std::integral_constant<int, 0>{}, std::false_type{});
                emit(2 * it + 1);
            } else {
                sub_chunk(r0, A, B, qA, qB, std::integral_constant<int, 0>{}, std::false_type{});
                sub_chunk(r0 + SUB, B, A, qB, qA, std::integral_constant<int, 1>{}, std::false_type{});
                emit(it);
            }
            if constexpr (RC) {
                // staircase checkpoint k after step k*E - 1: lane 0 has finished row k*E, lane l row k*E - l
                const int done = r0 + 2 * SUB;
                if (p.stck_every > 0 && (done & (p.stck_every - 1)) == 0 && done < m) {
                    int2* ck = p.stck + ((long long)((done >> p.stck_shift) - 1) * p.nstripes + s) * (TD + 1) * 64 + lane;
#pragma unroll
                    for (int k = 0; k < TD; k++) ck[k * 64] = make_int2(H[k], Y[k]);
                    ck[TD * 64] = make_int2(Xl, HLp);
                }
            }
        }
    }
    unsigned* prod_out = &cnt[2 * w + 1];
    if (lane == 0) __hip_atomic_store(prod_out, LK_DONE, RLX, WGS);
    if (partial && lane == cn / TD) p.out_last[0] = Hm;
    if (DBG && lane == 0) {
        unsigned long long* d = p.dbg + LK_DBG_WORDS * s;
        d[8] = t_avail;
        d[9] = t_pub;
        d[0] = t_start;
        d[1] = __builtin_amdgcn_s_memrealtime();
        d[2] = wcyc[0];
        d[3] = wcyc[1];
        d[4] = wcyc[2];
        d[5] = __builtin_amdgcn_s_memtime() - c_start;
        d[6] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID: wave, SIMD, CU, SE
        d[7] = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID: the XCD (bits 3:0)
        d[12] = w_first;
        d[13] = t_first;
#pragma unroll
        for (int k = 0; k < 6; k++) d[14 + k] = t_rows[k];
    }
}

#ifndef GA_LANE_KERNEL_ONLY  // (a test unit compiles one kernel variant alone)
template <int NWC, int TD, int CB, int SUB, bool DBG = false>
static void launch_lane_one(hipStream_t s, const FillArgs& p) {
    // the recompute checkpoints exist in one variant only (no timestamps, 16-step sub-chunks): enqueue_fill
    // asks for nothing else with them, and any other variant would leave them unwritten
    if constexpr (CB == 0 && SUB != 16)
        if (p.stck != nullptr) return launch_lane_one<NWC, TD, CB, 16, false>(s, p);
    if constexpr (!DBG && CB == 0)
        if (p.dbg != nullptr && p.stck == nullptr) return launch_lane_one<NWC, TD, CB, SUB, true>(s, p);
    // the LDS floor sets how many workgroups share a CU (GA_FILL_LDS_FLOOR overrides it, for tuning)
    const size_t floor_b = p.lds_floor >= 0 ? (size_t)p.lds_floor : (size_t)FILL_LDS_MIN;
    const size_t lds = std::max<size_t>(fill_lane_lds_bytes(NWC, p.K, p.qrows), floor_b);
    if constexpr (CB == 0 && !DBG && SUB == 16) {
        if (p.stck != nullptr) {
            auto* fc = fill_lane_kernel<NWC, TD, 0, 16, false, false, true, true>;
            (void)hipFuncSetAttribute((const void*)fc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            fc<<<dim3(p.nslabs), dim3(lane_block_threads(NWC)), lds, s>>>(p);
            return;
        }
    }
    if constexpr (CB == 0 && !DBG) {
        if (p.ckpt != nullptr) {  // 8-step sub-chunks: with 16 the checkpoint stores spill at TD >= 4
            auto* fc = fill_lane_kernel<NWC, TD, CB, 8, false, true>;
            (void)hipFuncSetAttribute((const void*)fc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            fc<<<dim3(p.nslabs), dim3(lane_block_threads(NWC)), lds, s>>>(p);
            return;
        }
    }
    if constexpr (CB == 0 && SUB == 16) {
        if (p.late) {
            auto* fl = fill_lane_kernel<NWC, TD, 0, 16, DBG, false, false, true>;
            (void)hipFuncSetAttribute((const void*)fl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            fl<<<dim3(p.nslabs), dim3(lane_block_threads(NWC)), lds, s>>>(p);
            return;
        }
    }
    auto* fn = fill_lane_kernel<NWC, TD, CB, SUB, DBG>;
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fn<<<dim3(p.nslabs), dim3(lane_block_threads(NWC)), lds, s>>>(p);
}

// variants without spills (vgpr_spill_count of the code object; lane_geometry keeps to them): score
// only TD <= 8; one-byte words TD <= 4; two-byte words TD <= 2; four-byte words TD <= 2 at NWC = 4
template <int NWC, int TD, int CB>
constexpr bool lane_variant_ok() {
    return CB == 0 || (CB == 1 && TD <= 4) || (CB == 2 && TD <= 2) || (CB == 4 && TD <= 2 && NWC == 4);
}

template <int TD, int CB>
static void launch_lane_td(hipStream_t s, const FillArgs& p) {
    // score only: 16-step sub-chunks (GA_LANE_SUB=8 selects 8, for tuning); traceback words: 16-step
    // sub-chunks for one-byte words at TD <= 4 with 4 waves (202 VGPRs, no spills; the pipelined C3 fill
    // 26.2 -> 24.9 ms, 8.85 -> 8.34 ms per alignment in steady state; GA_LANE_TB_SUB=8 selects 8), else 8
    const int sub_env = p.lane_sub > 0 ? p.lane_sub : 16;
    const int tb_sub_env = p.lane_tb_sub > 0 ? p.lane_tb_sub : 16;
    // (TD = 8 at 8 waves per workgroup spills with 16-step sub-chunks: 8)
    constexpr bool tb16 = CB == 1 && TD <= 4;
    if constexpr (tb16) {
        if (p.nwc == 4 && tb_sub_env == 16) return launch_lane_one<4, TD, CB, 16>(s, p);
    }
    constexpr bool sub16_ok4 = CB == 0, sub16_ok8 = CB == 0 && TD < 8;
    if (p.nwc == 4) {
        if constexpr (lane_variant_ok<4, TD, CB>()) {
            if (sub16_ok4 && sub_env != 8) launch_lane_one<4, TD, CB, sub16_ok4 ? 16 : 8>(s, p);
            else launch_lane_one<4, TD, CB, 8>(s, p);
        }
    } else {
        if constexpr (lane_variant_ok<8, TD, CB>()) {
            if (sub16_ok8 && sub_env != 8) launch_lane_one<8, TD, CB, sub16_ok8 ? 16 : 8>(s, p);
            else launch_lane_one<8, TD, CB, 8>(s, p);
        }
    }
}

template <int CB>
static void launch_lane_cb(hipStream_t s, const FillArgs& p) {
    switch (p.cols_per_lane) {
        case 1: launch_lane_td<1, CB>(s, p); break;
        case 2: launch_lane_td<2, CB>(s, p); break;
        case 4: launch_lane_td<4, CB>(s, p); break;
        default: launch_lane_td<8, CB>(s, p); break;
    }
}

void launch_fill_lane(hipStream_t s, const FillArgs& p, int CB) {
    if (p.tb == nullptr) launch_lane_cb<0>(s, p);
    else if (CB == 1) launch_lane_cb<1>(s, p);
    else if (CB == 2) launch_lane_cb<2>(s, p);
    else launch_lane_cb<4>(s, p);
}
#endif  // GA_LANE_KERNEL_ONLY

}  // namespace ga
