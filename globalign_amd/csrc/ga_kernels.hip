// ga_kernels.hip -- CDNA4 (gfx950) kernels of the affine-gap global-alignment engine.
//
// Hot path of globalign (globaligner.py in iamgiddyaboutgit/globalign):
//   make_dp_array (:756-821)          -> qp_kernel + boundary_kernel
//   dp_array_forward (:366-392)       -> fill_kernel
//     get_next_best_costs (:317-363)  -> dp_step (one cell per lane per step)
//   dp_array_backward (:395-593)      -> walk_kernel
//     cost_ranks_dispatcher (:595-685)   (tie-break bits precomputed on the host)
//
// Arithmetic.  With the potential phi(i,j) = GV(i) + GH(j)
// (prefix sums of the vertical / horizontal gap costs) every value is stored
// shifted, V' = V - phi.  Because the gap-open cost o >= 0 the reference's
// three minima collapse to
//     M' = H'(i-1,j-1) + sub'(a_i,b_j)        sub' = sub - gV(a_i) - gH(b_j)
//     X' = h1'(i,j-1)   h1' = min(X', H'+o)  (carried to the right)
//     Y' = h2'(i-1,j)   h2' = min(Y', H'+o)  (carried downwards)
//     H' = min3(M', X', Y')
// which is exact integer arithmetic (no rounding), so results are bit-exact.
//
// Layout (HBM): one wave owns a 64-column stripe; lane l owns column
// 64*s + l + 1 and processes row t - l + 1 at step t (anti-diagonal skew), so a
// row's left neighbour is lane l-1's previous step: moved with DPP wave_shr:1.
// Seven compute waves per workgroup are chained through LDS rings; an eighth
// (IO) wave moves the slab's left/right edges to/from HBM with write-through
// (sc1) stores and a progress word (cdna_hip_programming.md Guideline 16, R1).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ga_device.h"

namespace ga {

#define RLX __ATOMIC_RELAXED
#define AGENT __HIP_MEMORY_SCOPE_AGENT
#define WGS __HIP_MEMORY_SCOPE_WORKGROUP

__device__ __forceinline__ unsigned lds_ld(unsigned* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, WGS); }
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) { __hip_atomic_store(p, v, __ATOMIC_RELEASE, WGS); }
__device__ __forceinline__ unsigned g_ld(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), RLX, AGENT);
}
__device__ __forceinline__ void g_st(unsigned* p, unsigned v) { __hip_atomic_store(p, v, RLX, AGENT); }
__device__ __forceinline__ unsigned long long g_ld64(const int2* p) {
    return __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<int2*>(p)), RLX, AGENT);
}
__device__ __forceinline__ void g_st64(int2* p, int2 v) {
    unsigned long long x = (unsigned long long)(unsigned)v.x | ((unsigned long long)(unsigned)v.y << 32);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), x, RLX, AGENT);
}
__device__ __forceinline__ int2 unpack64(unsigned long long x) { return make_int2((int)(unsigned)x, (int)(x >> 32)); }

// Bounded spin: returns false (and raises the abort word) after `limit` sleeps.
__device__ __forceinline__ bool spin_ok(unsigned& spins, unsigned limit, unsigned* abort_word) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins >= limit) {
        g_st(abort_word, 1u);
        return false;
    }
    if ((spins & 1023u) == 0 && g_ld(abort_word)) return false;
    return true;
}

// Bounded spin for compute waves: LDS-only (no global memory op may appear in their
// loop, or the compiler's vmcnt bookkeeping turns the prefetch waits into vmcnt(0)).
__device__ __forceinline__ bool spin_ok_lds(unsigned& spins, unsigned limit, unsigned* abort_sh) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins >= limit) {
        __hip_atomic_store(abort_sh, 1u, __ATOMIC_RELAXED, WGS);
        return false;
    }
    if ((spins & 255u) == 0 && __hip_atomic_load(abort_sh, __ATOMIC_RELAXED, WGS)) return false;
    return true;
}

// ----------------------------------------------------------------------------------
// Boundary (make_dp_array, globaligner.py:756-821) in the shifted space, plus the
// prefix sums GV/GH and the original boundary triples the traceback needs at
// row 0 / column 0.  One workgroup of 1024 threads; a chunked scan.
__device__ void block_scan_gaps(const uint8_t* __restrict__ s, int len, const int* __restrict__ g, int* __restrict__ pre,
                                int* sh) {
    // pre[0] = 0, pre[k] = sum_{q<k} g[s[q]] for k in [0, len]
    const int T = blockDim.x, tid = threadIdx.x;
    const int chunk = (len + T - 1) / T;
    const int lo = min(len, tid * chunk), hi = min(len, lo + chunk);
    int acc = 0;
    for (int q = lo; q < hi; q++) acc += g[s[q]];
    sh[tid] = acc;
    __syncthreads();
    for (int off = 1; off < T; off <<= 1) {
        int v = tid >= off ? sh[tid - off] : 0;
        __syncthreads();
        sh[tid] += v;
        __syncthreads();
    }
    int run = sh[tid] - acc;  // exclusive prefix of this chunk
    for (int q = lo; q < hi; q++) {
        pre[q] = run;
        run += g[s[q]];
    }
    if (tid == T - 1) pre[len] = sh[T - 1];
    __syncthreads();
}

__global__ void __launch_bounds__(1024) boundary_kernel(const uint8_t* __restrict__ a, int m, const uint8_t* __restrict__ b,
                                                        int n, const int* __restrict__ gh, const int* __restrict__ gv, int o,
                                                        int big, int* __restrict__ GVp, int* __restrict__ GHp,
                                                        int2* __restrict__ top, int2* __restrict__ left,
                                                        int* __restrict__ bnd_row, int* __restrict__ bnd_col,
                                                        int* __restrict__ meta) {
    __shared__ int sh[1024];
    block_scan_gaps(a, m, gv, GVp, sh);
    block_scan_gaps(b, n, gh, GHp, sh);
    for (int j = threadIdx.x; j <= n; j += blockDim.x) {
        int M, X, Y;
        if (j == 0) { M = X = Y = 0; }                        // :778
        else { M = big; X = o + GHp[j]; Y = big; }            // :780-784, :802-809
        bnd_row[3 * j] = M; bnd_row[3 * j + 1] = X; bnd_row[3 * j + 2] = Y;
        int H = min(min(M, X), Y);
        int h2 = min(Y, H + o);
        top[j] = make_int2(H - GHp[j], h2 - GHp[j]);
    }
    for (int i = threadIdx.x; i <= m; i += blockDim.x) {
        int M, X, Y;
        if (i == 0) { M = X = Y = 0; }
        else { M = big; X = big; Y = o + GVp[i]; }            // :789-793, :812-819
        bnd_col[3 * i] = M; bnd_col[3 * i + 1] = X; bnd_col[3 * i + 2] = Y;
        int H = min(min(M, X), Y);
        int h1 = min(X, H + o);
        left[i] = make_int2(H - GVp[i], h1 - GVp[i]);
    }
    if (threadIdx.x == 0) { meta[0] = GVp[m]; meta[1] = GHp[n]; }
}

// Custom boundary triples (host supplied, original space) -> shifted edges.
__global__ void custom_boundary_kernel(const uint8_t* __restrict__ a, int m, const uint8_t* __restrict__ b, int n,
                                       const int* __restrict__ gh, const int* __restrict__ gv, int o,
                                       int* __restrict__ GVp, int* __restrict__ GHp, int2* __restrict__ top,
                                       int2* __restrict__ left, const int* __restrict__ bnd_row,
                                       const int* __restrict__ bnd_col, int* __restrict__ meta) {
    __shared__ int sh[1024];
    block_scan_gaps(a, m, gv, GVp, sh);
    block_scan_gaps(b, n, gh, GHp, sh);
    for (int j = threadIdx.x; j <= n; j += blockDim.x) {
        int M = bnd_row[3 * j], X = bnd_row[3 * j + 1], Y = bnd_row[3 * j + 2];
        int H = min(min(M, X), Y);
        top[j] = make_int2(H - GHp[j], min(Y, H + o) - GHp[j]);
    }
    for (int i = threadIdx.x; i <= m; i += blockDim.x) {
        int M = bnd_col[3 * i], X = bnd_col[3 * i + 1], Y = bnd_col[3 * i + 2];
        int H = min(min(M, X), Y);
        left[i] = make_int2(H - GVp[i], min(X, H + o) - GVp[i]);
    }
    if (threadIdx.x == 0) { meta[0] = GVp[m]; meta[1] = GHp[n]; }
}

// ----------------------------------------------------------------------------------
// The wavefront fill.
//
// Traceback word of a cell (CB bytes, W = (8*CB-1)/2 bits per field):
//   bits [0,W)   : min(X - H, o+1)     X in S1 <=> <= o ; M,Y may be in S1 <=> >= o
//   bits [W,2W)  : min(Y - H, o+1)
//   bit  2W      : M != H
// which is all dp_array_backward's rank test needs at this cell.
template <int CB>
struct TbFmt {
    static constexpr int W = (8 * CB - 1) / 2;
    static constexpr int SPC = 16 / CB;  // steps per 16-byte lane chunk
};

struct StepState {
    int Yc;    // h2' carried from the row above (Y' of this lane's next cell)
    int HLp;   // H' of the left column one row up (the next cell's diagonal)
    int Hout;  // this lane's H' of the current row   (to lane l+1)
    int Xout;  // this lane's h1' of the current row  (to lane l+1)
};

// BYTES of query profile (one chunk's sub' values for one lane), as raw dwords.
template <int BYTES>
struct QPack {
    static constexpr int NWD = (BYTES + 3) / 4;
    uint32_t w[NWD];
    template <typename T>
    __device__ static QPack load(const T* p) {
        QPack r;
        __builtin_memcpy(r.w, p, sizeof(r.w));
        return r;
    }
    template <typename QT>
    __device__ __forceinline__ int get(int u) const {
        if (sizeof(QT) == 1) return (int)(int8_t)(w[u >> 2] >> (8 * (u & 3)));
        return (int)(int16_t)(w[u >> 1] >> (16 * (u & 1)));
    }
};

// ABL: diagnostic ablations (0 in the product): 2 = no DPP (timing only)
template <int CB, bool MASK, bool FULL, int ABL = 0>
__device__ __forceinline__ void dp_step(StepState& s, int2 lin, int sub, int o, unsigned op1, int t, int lane, int m,
                                        bool colok, uint32_t& accw, int sh, int* full, int fullW, int jcol) {
    constexpr int W = TbFmt<CB>::W;
    // left neighbour (lane l-1, previous step); lane 0 takes the slab edge from the ring
    const int HL = (ABL & 2) ? (lin.x ^ s.Hout) : __builtin_amdgcn_update_dpp(lin.x, s.Hout, 0x138, 0xf, 0xf, false);  // wave_shr:1
    const int XL = (ABL & 2) ? (lin.y ^ s.Xout) : __builtin_amdgcn_update_dpp(lin.y, s.Xout, 0x138, 0xf, 0xf, false);
    const int Hd = s.HLp;
    s.HLp = HL;
    bool act = true;
    if (MASK) {
        const int i = t - lane + 1;
        act = (i >= 1) & (i <= m) & colok;
    }
    if (act) {
        const int M = Hd + sub;
        const int H = min(min(M, XL), s.Yc);
        const int Ho = H + o;
        const unsigned code = min((unsigned)(XL - H), op1) | (min((unsigned)(s.Yc - H), op1) << W) |
                              (min((unsigned)(M - H), 1u) << (2 * W));
        if (FULL) {
            const int i = t - lane + 1;
            int* f = full + 3 * ((long long)i * fullW + jcol);
            f[0] = M; f[1] = XL; f[2] = s.Yc;
        }
        accw = sh == 0 ? code : (accw | (code << sh));
        s.Xout = min(XL, Ho);
        s.Yc = min(s.Yc, Ho);
        s.Hout = H;
    } else if (MASK && !colok) {
        s.Hout = HL;  // columns beyond n forward their left input unchanged
        s.Xout = XL;
    }
}



// ABL (diagnostic ablations, 0 in the product): 1 = no ring write, 2 = no DPP, 4 = no ring
// read, 8 = no query-profile reads, 16 = no inter-wave waits.
//
// Workgroup = NW compute waves + 2 IO waves, all communication through LDS.
// Compute waves issue no HBM operation at all (their steady loop is VALU + LDS):
//   * IO-A (wave NW) moves the slab's left edge in (HBM -> ring 0), the right edge
//     out (ring NW -> HBM, write-through + progress word) and fills the query
//     profile ring qring[code][row] from seq_1 (sub' = sub - gV - gH);
//   * IO-B (wave NW+1) streams the compute waves' traceback words from LDS
//     staging slots to HBM.
// LDS layout (dynamic, byte offsets from FillLds::*).
struct FillLds {
    static constexpr int CNT = 0;                                  // u32 counters (see CI_*)
    static constexpr int RINGS = 256;                              // (NW+1) x RING x int2
    static constexpr int DUMMY = RINGS + (NW + 1) * RING * 8;      // 64 x 17 x int2 sink for lanes 0..62
    static constexpr int TBST = DUMMY + 64 * 17 * 8;               // NW x TBS x 64 x 16 B
    static constexpr int QRING_TB = TBST + NW * TBS * 1024;
    static constexpr int QRING_NOTB = TBST;
};
enum { CI_PROD = 0, CI_CONS = 8, CI_TBPROD = 16, CI_TBCONS = 24, CI_ABORT = 32, CI_SLAB = 33 };

template <int CB, typename QT, bool TB, bool FULL, int ABL = 0>
__global__ void __launch_bounds__(64 * (NW + 2)) fill_kernel(FillArgs p) {
    constexpr int SPC = TbFmt<CB>::SPC;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    unsigned* cnt = reinterpret_cast<unsigned*>(smem + FillLds::CNT);
    int2* rings = reinterpret_cast<int2*>(smem + FillLds::RINGS);
    int2* dummy = reinterpret_cast<int2*>(smem + FillLds::DUMMY);
    uint4* tbst = reinterpret_cast<uint4*>(smem + FillLds::TBST);
    QT* qring = reinterpret_cast<QT*>(smem + (TB ? FillLds::QRING_TB : FillLds::QRING_NOTB));
    unsigned* prod = cnt + CI_PROD;
    unsigned* cons = cnt + CI_CONS;
    unsigned* tbprod = cnt + CI_TBPROD;
    unsigned* tbcons = cnt + CI_TBCONS;
    unsigned* abort_sh = cnt + CI_ABORT;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave index: uniform
    if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x == 0) cnt[CI_SLAB] = atomicAdd(p.ticket, 1u);
    __syncthreads();
    const int g = __builtin_amdgcn_readfirstlane((int)cnt[CI_SLAB]);  // uniform: scalar branches below
    const unsigned m = (unsigned)p.m;
    const int QSTRIDE = QROWS + SPC;  // per code: QROWS slots + SPC mirrored rows (no wrap inside a chunk)
    const int T = (int)m + 63;
    const int nchunks = (T + SPC - 1) / SPC;

    if (w == NW) {
        // ---------------- IO-A: slab edges HBM <-> LDS rings, query profile ----------------
        const int2* src = g == 0 ? p.left : p.hand + (long long)(g - 1) * (m + 1);
        const unsigned* src_prog = g == 0 ? p.left_prog : p.hand_prog + (g - 1);
        const unsigned limit = (g == 0 && p.left_prog != nullptr) ? p.halo_spin_limit : p.spin_limit;
        const bool src_sc1 = g != 0 || p.left_prog != nullptr;
        int2* dst = (g == p.nslabs - 1 && p.edge_out != nullptr) ? p.edge_out : p.hand + (long long)g * (m + 1);
        const int K = p.K;
        unsigned in_next = 0, out_next = 0, spins = 0;
        while (in_next < m || out_next < m) {
            bool moved = false;
            if (in_next < m) {
                // ring 0 slots are reused after wave 0 read them; query-profile rows after
                // the last compute wave's lanes all passed them (its output count)
                const unsigned space = min(lds_ld(&cons[0]) + RING, lds_ld(&prod[NW]) + QROWS - 2 * SPC);
                const unsigned avail = src_prog ? min(g_ld(src_prog), m) : m;
                const unsigned hi = min(min(space, avail), in_next + 64);
                if (hi > in_next && (hi - in_next >= 16 || hi == avail)) {
                    const unsigned r = in_next + 1 + lane;
                    if (r <= hi) {
                        rings[(r + 62) & RMASK] = src_sc1 ? unpack64(g_ld64(src + r)) : src[r];
                        const int x = p.a[r - 1];
                        const int slot = r & QMASK;
                        const int* sp = p.subp + x * K;
                        for (int c = 0; c < K; c++) {
                            const QT v = (QT)sp[c];
                            qring[c * QSTRIDE + slot] = v;
                            if (slot < SPC) qring[c * QSTRIDE + QROWS + slot] = v;
                        }
                    }
                    if (lane == 0) lds_st(&prod[0], hi);
                    in_next = hi;
                    moved = true;
                }
            }
            if (out_next < m) {
                const unsigned avail = lds_ld(&prod[NW]);
                const unsigned hi = min(avail, out_next + 64);
                if (hi > out_next && (hi - out_next >= GOUT || hi == m)) {
                    const unsigned r = out_next + 1 + lane;
                    if (r <= hi) g_st64(dst + r, rings[NW * RING + ((r + 62) & RMASK)]);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0) {
                        g_st(p.hand_prog + g, hi);
                        if (p.edge_prog != nullptr && g == p.nslabs - 1)
                            __hip_atomic_store(p.edge_prog, hi, RLX, __HIP_MEMORY_SCOPE_SYSTEM);
                        lds_st(&cons[NW], hi);
                    }
                    out_next = hi;
                    moved = true;
                }
            }
            if (!moved) {
                if (__hip_atomic_load(abort_sh, RLX, WGS)) {  // a compute wave gave up
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
        return;
    }

    if (w == NW + 1) {
        // ---------------- IO-B: traceback words LDS staging -> HBM ----------------
        if (!TB) return;
        unsigned done[NW];
        int nlive = 0;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            done[k] = 0;
            nlive += (g * NW + k) < p.nstripes;
        }
        unsigned spins = 0;
        for (;;) {
            bool moved = false, all = true;
#pragma unroll
            for (int k = 0; k < NW; k++) {
                if (k >= nlive) continue;
                const unsigned avail = lds_ld(&tbprod[k]);
                if (avail > done[k]) {
                    const long long s = (long long)g * NW + k;
                    uint4* dstp = reinterpret_cast<uint4*>(p.tb) + (s * p.TC) * 64 + lane;
                    for (unsigned cc = done[k]; cc < avail; cc++)
                        dstp[(long long)cc * 64] = tbst[(k * TBS + (cc % TBS)) * 64 + lane];
                    done[k] = avail;
                    if (lane == 0) lds_st(&tbcons[k], avail);  // the LDS reads above are complete
                    moved = true;
                }
                all &= done[k] >= (unsigned)nchunks;
            }
            if (all) break;
            if (!moved) {
                if (__hip_atomic_load(abort_sh, RLX, WGS)) break;
                if (!spin_ok(spins, p.spin_limit, p.abort_word)) {
                    __hip_atomic_store(abort_sh, 1u, RLX, WGS);
                    break;
                }
            } else {
                spins = 0;
            }
        }
        return;
    }

    // ---------------- compute wave w: stripe s ----------------
    const int s = g * NW + w;
    const bool live = s < p.nstripes;
    const int jcol = s * 64 + lane + 1;               // 1-based column of this lane
    const bool colok = live && jcol <= p.n;
    const bool full_stripe = live && (s * 64 + 64 <= p.n);
    const int bcode = colok ? p.b[jcol - 1] : 0;
    const QT* qcol = qring + bcode * QSTRIDE;
    StepState st;
    {
        const int jt = colok ? jcol : 0;
        st.Hout = p.top[jt].x;                       // H'(0, j)
        st.Yc = p.top[jt].y;                         // h2'(0, j)
        st.HLp = p.top[colok ? jcol - 1 : 0].x;      // H'(0, j-1): diagonal of row 1
        st.Xout = 0;
    }
    const int o = p.o;
    const unsigned op1 = (unsigned)o + 1u;
    const int2* rin = rings + w * RING;
    // lanes 0..62 write into their own sink rows, 17 int2 apart: the per-lane stride of 34
    // dwords spreads a 16-lane ds_write_b64 group over all 32 banks (no conflicts)
    int2* const aout = lane == 63 ? rings + (w + 1) * RING : dummy + lane * 17;
    const unsigned aout_mask = lane == 63 ? (unsigned)RMASK : 0u;
    unsigned spins = 0, avail = 0, outfree = RING, tbfree = TBS;
    unsigned long long stamp0 = 0, stamp1 = 0;
    bool ok = true;

    for (int c = 0; c < nchunks && ok; c++) {
        const int t0 = c * SPC;
        if (p.dbg != nullptr && c == 1) stamp0 = __builtin_amdgcn_s_memrealtime();
        if (p.dbg != nullptr && c == nchunks / 2) stamp1 = __builtin_amdgcn_s_memrealtime();
        // inputs: rows t0+1 .. t0+SPC in ring w (counter read only when needed)
        const unsigned need = min((unsigned)(t0 + SPC), m);
        while (!(ABL & 16) && avail < need) {
            avail = lds_ld(&prod[w]);
            if (avail >= need) break;
            if (!spin_ok_lds(spins, p.spin_limit, abort_sh)) { ok = false; break; }
        }
        // outputs: rows t0-62 .. t0+SPC-63; a ring slot is reused RING rows later
        const int hi_out = t0 + SPC - 63;
        while (!(ABL & 16) && (int)outfree < hi_out) {
            outfree = lds_ld(&cons[w + 1]) + RING;
            if ((int)outfree >= hi_out) break;
            if (!spin_ok_lds(spins, p.spin_limit, abort_sh)) { ok = false; break; }
        }
        // traceback staging slot c % TBS must have been drained (chunk c - TBS)
        while (TB && live && !(ABL & 16) && tbfree < (unsigned)c + 1u) {
            tbfree = lds_ld(&tbcons[w]) + TBS;
            if (tbfree >= (unsigned)c + 1u) break;
            if (!spin_ok_lds(spins, p.spin_limit, abort_sh)) { ok = false; break; }
        }
        if (!ok) break;
        spins = 0;
        if (lane == 0) __hip_atomic_store(&cons[w], min((unsigned)t0, m), RLX, WGS);
        // this chunk's left-edge rows (broadcast) and substitution values (per lane)
        int2 lin[SPC];
        int qv[SPC];
        const QT* qa = qcol + ((t0 + 1 - lane) & QMASK);
#pragma unroll
        for (int u = 0; u < SPC; u++) {
            lin[u] = (ABL & 4) ? make_int2(t0 + u, u) : rin[(t0 + 63 + u) & RMASK];
            qv[u] = (ABL & 8) ? (u - 3) : (int)qa[u];
        }
        int2* ao = aout + ((unsigned)t0 & aout_mask);
        uint32_t acc[4] = {0, 0, 0, 0};
        const bool steady = full_stripe && t0 >= 63 && t0 + SPC - 1 <= (int)m - 1;
        if (steady) {
#pragma unroll
            for (int u = 0; u < SPC; u++) {
                dp_step<CB, false, FULL, ABL>(st, lin[u], qv[u], o, op1, t0 + u, lane, m, true, acc[(u * CB) >> 2],
                                              (u * CB * 8) & 31, p.full, p.n + 1, jcol);
                if (!(ABL & 1)) ao[u] = make_int2(st.Hout, st.Xout);
            }
        } else {
#pragma unroll
            for (int u = 0; u < SPC; u++) {
                dp_step<CB, true, FULL, ABL>(st, lin[u], qv[u], o, op1, t0 + u, lane, m, colok, acc[(u * CB) >> 2],
                                             (u * CB * 8) & 31, p.full, p.n + 1, jcol);
                if (!(ABL & 1)) ao[u] = make_int2(st.Hout, st.Xout);
            }
        }
        if (TB && live) tbst[(w * TBS + (c % TBS)) * 64 + lane] = make_uint4(acc[0], acc[1], acc[2], acc[3]);
        if (lane == 0) {
            // one release (lgkmcnt(0)) covers the ring rows and the staged words
            if (TB && live) lds_st(&tbprod[w], (unsigned)c + 1u);
            if (hi_out >= 1) lds_st(&prod[w + 1], min((unsigned)hi_out, m));
        }
    }
    if (p.dbg != nullptr && lane == 0 && live) {
        p.dbg[4 * s] = stamp0;
        p.dbg[4 * s + 1] = stamp1;
        p.dbg[4 * s + 2] = __builtin_amdgcn_s_memrealtime();
    }
    // the lane owning column n writes the final H' (cost = H' + phi(m, n))
    if (ok && colok && jcol == p.n) p.out_last[0] = st.Hout;
}

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
// sh_L = 2*S_L + 16*(a_i != b_j), S_L the rank set of sets_from_code.  The
// host table entry of dispatch D holds, at bits sh..sh+1, the level the
// reference's random.choice picks for that set (match half at 2S, mismatch
// half at 16+2S), so a step is lvl = (tab >> sh_L) & 3.
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
__device__ __forceinline__ unsigned cell_shifts(int sets, bool am) {
    const unsigned mm = am ? 0u : 16u;
    const unsigned f0 = 2u * (sets & 7) + mm, f1 = 2u * ((sets >> 3) & 7) + mm, f2 = 2u * ((sets >> 6) & 7) + mm;
    return f0 | (f1 << 5) | (f2 << 10);
}

__device__ __forceinline__ unsigned tb_code(const uint8_t* tb, int CB, int TC, int i, int j) {
    const int s = (j - 1) >> 6, l = (j - 1) & 63, t = i - 1 + l;
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

// One loader wave decodes tile (ti, tj) into the torus: lane = column; each lane
// walks the 16-byte chunks of its column's traceback stream that cover the
// tile's 64 rows (the general path; one-byte words use load_tile_b1).
template <int CB>
__device__ void load_tile(const WalkArgs& w, int ti, int tj, uint16_t* torus, uint8_t* sa, const uint16_t* lut,
                          int lane) {
    uint16_t* dst = torus + (ti & (TB4 - 1)) * TT * TP + (tj & (TB4 - 1)) * TT;
    constexpr int SPC = 16 / CB;
    constexpr int KMAX = TT / SPC + 1;
    const int i0 = ti * TT + 1;                       // first row of the tile
    const int j = tj * TT + lane + 1;                 // this lane's column
    sa[lane] = (i0 + lane <= w.m) ? w.a[i0 + lane - 1] : 0xff;
    const bool colok = j <= w.n;
    const int bj = colok ? w.b[j - 1] : 0xfe;
    const int tfirst = i0 - 1 + lane;                 // t of row i0 in this column
    const int q0 = tfirst / SPC;
    const uint4* base = reinterpret_cast<const uint4*>(w.tb) + ((long long)tj * w.TC) * 64 + lane;
    uint4 ch[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
        const int q = q0 + k;
        ch[k] = (colok && q < w.TC) ? base[(long long)q * 64] : make_uint4(0, 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): sa[] visible to this wave
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
        const unsigned wd[4] = {ch[k].x, ch[k].y, ch[k].z, ch[k].w};
#pragma unroll
        for (int u = 0; u < SPC; u++) {
            const int r = (q0 + k) * SPC + u - tfirst;   // tile row
            if (r >= 0 && r < TT) {
                unsigned code = wd[(u * CB) >> 2] >> ((u * CB * 8) & 31);
                if (CB == 1) code &= 0xffu;
                else if (CB == 2) code &= 0xffffu;
                dst[r * TP + lane] = (uint16_t)cell_shifts(sets_from_code(code, CB, w.o), sa[r] == bj);
            }
        }
    }
}

// One-byte traceback words (the common case, gap open < 7): branch-free decode.
// A lane's 64 cells sit at byte offset (tfirst mod 16) of the five 16-byte
// chunks it loads; the lane realigns them (dword select + v_alignbyte), folds
// a_i == b_j into bit 7 of each word (SWAR zero-byte test on the staged a
// bytes; words use bits 0-6) and decodes through a 256-entry table.
__device__ void load_tile_b1(const WalkArgs& w, int ti, int tj, uint16_t* torus, uint8_t* sa, const uint16_t* lut,
                             int lane) {
    uint16_t* dst = torus + (ti & (TB4 - 1)) * TT * TP + (tj & (TB4 - 1)) * TT + lane;
    const int i0 = ti * TT + 1;
    const int j = tj * TT + lane + 1;
    sa[lane] = (i0 + lane <= w.m) ? w.a[i0 + lane - 1] : 0xff;
    const bool colok = j <= w.n;
    const unsigned bj = colok ? w.b[j - 1] : 0xfeu;
    const int tfirst = i0 - 1 + lane;
    const int q0 = tfirst >> 4, off = tfirst & 15;
    const uint4* base = reinterpret_cast<const uint4*>(w.tb) + ((long long)tj * w.TC) * 64 + lane;
    unsigned wv[20];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const int q = q0 + k;
        const uint4 c = (colok && q < w.TC) ? base[(long long)q * 64] : make_uint4(0, 0, 0, 0);
        wv[4 * k] = c.x; wv[4 * k + 1] = c.y; wv[4 * k + 2] = c.z; wv[4 * k + 3] = c.w;
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
    const int dw = off >> 2;
    const unsigned sb = (unsigned)(off & 3);
    unsigned al[17];
#pragma unroll
    for (int k = 0; k < 17; k++) al[k] = dw == 0 ? wv[k] : dw == 1 ? wv[k + 1] : dw == 2 ? wv[k + 2] : wv[k + 3];
    const unsigned bj4 = bj * 0x01010101u;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        unsigned cw = __builtin_amdgcn_alignbyte(al[k + 1], al[k], sb);  // rows 4k .. 4k+3
        const unsigned x = av[k] ^ bj4;
        const unsigned t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;      // bit 7 of a byte clear <=> byte == 0
        cw = (cw & 0x7f7f7f7fu) | (~t & 0x80808080u);
#pragma unroll
        for (int u = 0; u < 4; u++) dst[(4 * k + u) * TP] = lut[(cw >> (8 * u)) & 0xffu];
    }
}

constexpr int RB = 2048;  // LDS rings of tie-break entries / chosen levels (4 blocks of 512 dispatches)

__device__ __forceinline__ int sgpr(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Waves: 0 walker, 4 ring helper, 8 idle (so the walker's SIMD runs nothing
// else), the other nine load tiles.
constexpr int WALK_WAVES = 12;
constexpr int NLOAD = 9;
// loader claim order over the 4x4 block: nearest tiles first (row offset, column offset)
__constant__ int8_t LOAD_ORDER[NSLOT][2] = {{0, 0}, {1, 0}, {0, 1}, {1, 1}, {2, 0}, {0, 2}, {2, 1}, {1, 2},
                                           {2, 2}, {3, 0}, {0, 3}, {3, 1}, {1, 3}, {3, 2}, {2, 3}, {3, 3}};

__device__ __forceinline__ bool in_block(int cur, int ti, int tj) {
    const int dti = (cur >> 16) - ti, dtj = (cur & 0xffff) - tj;
    return cur >= 0 && dti >= 0 && dti < TB4 && dtj >= 0 && dtj < TB4;
}

template <int CB>
__global__ void __launch_bounds__(64 * WALK_WAVES) walk_kernel(WalkArgs w) {
    __shared__ uint16_t torus[TP * TP];
    __shared__ __attribute__((aligned(16))) uint32_t rngbuf[RB];
    __shared__ uint32_t opsbuf[RB / 16];
    __shared__ uint16_t lut[256];
    __shared__ __attribute__((aligned(16))) uint8_t sa[NLOAD][TT];
    __shared__ int tag[NSLOT], busy[NSLOT];
    __shared__ int rtag[4];
    __shared__ int cur_tile, walk_done, wD, ops_flushed;
    __shared__ unsigned long long load_ticks;
    __shared__ int load_count;
    const int lane = threadIdx.x & 63;
    const int wave = sgpr(threadIdx.x >> 6);
    const int m = w.m, n = w.n, o = w.o;
    if (threadIdx.x == 0) { load_ticks = 0; load_count = 0; }
    if (threadIdx.x < NSLOT) { tag[threadIdx.x] = -1; busy[threadIdx.x] = 0; }
    if (threadIdx.x < 4) rtag[threadIdx.x] = -1;
    // a slab walk starts at dispatch D0: the rings start at its block
    if (threadIdx.x == 0) { cur_tile = -1; walk_done = 0; wD = w.D0; ops_flushed = w.D0 >> 9; }
    if (CB == 1 && threadIdx.x < 256)
        lut[threadIdx.x] = (uint16_t)cell_shifts(sets_from_code(threadIdx.x & 127u, 1, o), (threadIdx.x >> 7) != 0);
    __syncthreads();

    if (wave == 8) return;
    if (wave == 4) {
        // ---------------- helper: tie-break table HBM -> LDS ring, levels LDS ring -> HBM ----------------
        const long long nblk = (w.nrng + 511) / 512;
        long long rl = w.D0 >> 9, fl = w.D0 >> 9;
        for (;;) {
            const int d = sgpr(__hip_atomic_load(&wD, __ATOMIC_ACQUIRE, WGS));
            const int done = sgpr(__hip_atomic_load(&walk_done, __ATOMIC_ACQUIRE, WGS));
            bool moved = false;
            while (rl < nblk && rl < (d >> 9) + 4) {
                const long long e0 = rl * 512 + lane * 8;
                uint32_t* dst = rngbuf + (rl & 3) * 512 + lane * 8;
#pragma unroll
                for (int k = 0; k < 8; k++) dst[k] = (e0 + k < w.nrng) ? w.rng[e0 + k] : 0u;
                if (lane == 0) __hip_atomic_store(&rtag[rl & 3], (int)rl, __ATOMIC_RELEASE, WGS);
                rl++;
                moved = true;
            }
            const long long complete = done ? ((long long)d + 511) / 512 : (d >> 9);
            while (fl < complete) {  // 512 dispatches = 32 words of levels
                if (lane < 32) w.ops[fl * 32 + lane] = opsbuf[(fl & 3) * 32 + lane];
                fl++;
                if (lane == 0) __hip_atomic_store(&ops_flushed, (int)fl, __ATOMIC_RELEASE, WGS);
                moved = true;
            }
            if (done && fl >= complete) break;
            if (!moved) __builtin_amdgcn_s_sleep(8);
        }
        return;
    }

    if (wave > 0) {
        // ---------------- loader pool: claim the nearest uncached tile of the walker's 4x4 block ----------------
        // A slot is written only by the loader holding busy[slot].  The claim re-reads the current tile
        // after invalidating the slot's tag, so a tile the walker may still read is never overwritten:
        // the walker publishes its tile before it checks a tag.
        const int li = wave - 1 - (wave > 4) - (wave > 8);
        while (!sgpr(__hip_atomic_load(&walk_done, __ATOMIC_ACQUIRE, WGS))) {
            const int cur = sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_ACQUIRE, WGS));
            bool did = false;
            if (cur >= 0) {
                const int ti = cur >> 16, tj = cur & 0xffff;
                for (int pidx = 0; pidx < NSLOT && !did; pidx++) {
                    const int tti = ti - LOAD_ORDER[pidx][0], ttj = tj - LOAD_ORDER[pidx][1];
                    if (tti < 0 || ttj < 0) continue;
                    const int tg = (tti << 16) | ttj, sl = slot_of(tti, ttj);
                    if (sgpr(__hip_atomic_load(&tag[sl], __ATOMIC_RELAXED, WGS)) == tg) continue;
                    if (sgpr(__hip_atomic_load(&busy[sl], __ATOMIC_RELAXED, WGS)) != 0) continue;
                    int got = 0;
                    if (lane == 0) {
                        int expect = 0;
                        got = __hip_atomic_compare_exchange_strong(&busy[sl], &expect, 1, __ATOMIC_SEQ_CST,
                                                                   __ATOMIC_RELAXED, WGS);
                    }
                    if (!sgpr(got)) continue;
                    bool ok = sgpr(__hip_atomic_load(&tag[sl], __ATOMIC_SEQ_CST, WGS)) != tg;
                    if (ok) {
                        if (lane == 0) __hip_atomic_store(&tag[sl], -1, __ATOMIC_SEQ_CST, WGS);
                        ok = in_block(sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_SEQ_CST, WGS)), tti, ttj);
                    }
                    if (ok) {
                        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                        if (CB == 1) load_tile_b1(w, tti, ttj, torus, sa[li], lut, lane);
                        else load_tile<CB>(w, tti, ttj, torus, sa[li], lut, lane);
                        if (lane == 0) {
                            atomicAdd(&load_ticks, __builtin_amdgcn_s_memrealtime() - t0);
                            atomicAdd(&load_count, 1);
                        }
                        if (lane == 0 && in_block(sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_SEQ_CST, WGS)), tti, ttj))
                            __hip_atomic_store(&tag[sl], tg, __ATOMIC_RELEASE, WGS);
                        did = true;
                    }
                    if (lane == 0) __hip_atomic_store(&busy[sl], 0, __ATOMIC_RELEASE, WGS);
                }
            }
            if (!did) __builtin_amdgcn_s_sleep(2);
        }
        return;
    }

    // ---------------- walker wave (its loop touches LDS only) ----------------
    int i = w.i0, j = w.j0, L = w.L0, D = w.D0, h = w.h0, first = w.first0, reason = -1;
    const int jend = w.handoff ? 5 : 2;  // reason when the walk reaches local column 0
    int cti = -1, ctj = -1, nwait = 0, ntiles = 0;
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
        }
        t_tile += __builtin_amdgcn_s_memrealtime() - t0;
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
            sh = (unsigned)sgpr((int)(2u * S + (w.a[pa] == w.b[pb] ? 0u : 16u)));
        }
        const int lvl = (int)((tab >> sh) & 3u);
        uint8_t* ob = ops_byte(D);
        *ob = (uint8_t)(((D & 3) ? *ob : 0) | (lvl << (6 - 2 * (D & 3))));
        D++;
        i -= (lvl != 1);
        j -= (lvl != 2);
        L = lvl;
        if (first) {
            first = 0;
            if (i == 0 && j == 0) { reason = 0; break; }
            continue;
        }
        if (i == 0) { reason = 1; break; }
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
        // widen a window cell when its group starts: the empty asm keeps the compiler from pulling the
        // widening (and so the wait for the LDS read) back into the group that issued the read
        auto widen = [](int raw) -> int {
            asm volatile("" : "+v"(raw));
            const unsigned u = (unsigned)raw;
            return (int)((u & 31u) | ((u & 0x3e0u) << 3) | ((u & 0x7c00u) << 6));
        };
        auto tabs = [&](int d) { return *reinterpret_cast<const uint4*>(rngbuf + (d & (RB - 1))); };

        if ((D & 511) == 0) {
            block_start(D);
            rng_ready(D);
        }
        verify(i, j);
        int wnext = window(i, j);    // anchored at the walk's current cell
        uint4 tnext = tabs(D);
        unsigned rel = 0;            // offset of the current cell from wnext's anchor (di*8 + dj)
        unsigned L8 = 8u * L;        // bit offset of the entering level's field in a window cell
        unsigned ops = 0;

        // One group of 4 steps: swap in the prefetched window and entries, prefetch the next ones.
        // CHECK: stop at the matrix edge; returns the steps taken when the walk ended, else 0.
        auto group = [&](auto check_tag, int gd) -> int {  // gd: dispatch of the group's first step
            constexpr bool CHECK = decltype(check_tag)::value;
            const int wcur = widen(wnext);
            const uint4 tc = tnext;
            wnext = window(i, j);
            tnext = tabs(gd + 4);
            __builtin_amdgcn_sched_barrier(0);  // issue the prefetch here, not where the next group needs it
            const unsigned t[4] = {(unsigned)sgpr((int)tc.x), (unsigned)sgpr((int)tc.y), (unsigned)sgpr((int)tc.z),
                                   (unsigned)sgpr((int)tc.w)};
            unsigned idx = rel, mv = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const unsigned v = (unsigned)__builtin_amdgcn_readlane(wcur, (int)(idx + mv));
                const unsigned lvl = (t[k] >> ((v >> L8) & 31u)) & 3u;
                ops = ops * 4u + lvl;
                L8 = lvl << 3;
                mv += (0x080109u >> L8) & 0xffu;  // diag 9, left 1, up 8
                if (CHECK) {
                    if ((int)(mv >> 3) == i || (int)(mv & 7u) == j) {
                        i -= (int)(mv >> 3);
                        j -= (int)(mv & 7u);
                        return k + 1;
                    }
                }
            }
            i -= (int)(mv >> 3);
            j -= (int)(mv & 7u);
            rel = mv;
            return 0;
        };
        for (;;) {
            // iteration of 16 dispatches D .. D+15 (D % 16 == 0)
            if ((D & 511) == 0) block_start(D);
            if (((D + 16) & 511) == 0) rng_ready(D + 16);
            // every window of this iteration is anchored within 12 steps: rows >= i - 19
            if (__builtin_expect(i - 19 < vlo_i || j - 19 < vlo_j, 0)) verify(i, j);
            if (__builtin_expect(min(i, j) > 16, 1)) {
                group(std::false_type{}, D);
                group(std::false_type{}, D + 4);
                group(std::false_type{}, D + 8);
                group(std::false_type{}, D + 12);
                opsbuf[(D >> 4) & (RB / 16 - 1)] = ops;
                D += 16;
                continue;
            }
            // near the top / left edge (the verified tiles reach row / column 1 here)
            int g = 0, k = 0;
            for (; g < 4; g++) {
                k = group(std::true_type{}, D + 4 * g);
                if (k) break;
            }
            if (g < 4) {
                // ended after k steps of group g: left-align the partial word
                const int nd = 4 * g + k;
                opsbuf[(D >> 4) & (RB / 16 - 1)] = ops << (2 * (16 - nd));
                D += nd;
                reason = i == 0 ? 1 : jend;
                break;
            }
            opsbuf[(D >> 4) & (RB / 16 - 1)] = ops;
            D += 16;
        }
    }
    if (lane == 0) {
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

// ----------------------------------------------------------------------------------
// host-side launchers (called from ga_host.cpp)
void launch_boundary(hipStream_t s, const uint8_t* a, int m, const uint8_t* b, int n, const int* gh, const int* gv,
                     int o, int big, int* GVp, int* GHp, int2* top, int2* left, int* bnd_row, int* bnd_col, int* meta,
                     bool custom) {
    if (custom)
        custom_boundary_kernel<<<1, 1024, 0, s>>>(a, m, b, n, gh, gv, o, GVp, GHp, top, left, bnd_row, bnd_col, meta);
    else
        boundary_kernel<<<1, 1024, 0, s>>>(a, m, b, n, gh, gv, o, big, GVp, GHp, top, left, bnd_row, bnd_col, meta);
}

size_t fill_lds_bytes(int CB, int qbytes, bool tb, int K) {
    const int spc = 16 / CB;
    return (size_t)(tb ? FillLds::QRING_TB : FillLds::QRING_NOTB) + (size_t)K * (QROWS + spc) * qbytes;
}

template <int CB, typename QT, bool TB, bool FULL, int ABL>
static void launch_one(hipStream_t s, const FillArgs& p) {
    const size_t lds = fill_lds_bytes(CB, (int)sizeof(QT), TB, p.K);
    auto* fn = fill_kernel<CB, QT, TB, FULL, ABL>;
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fn<<<dim3(p.nslabs), dim3(64 * (NW + 2)), lds, s>>>(p);
}

template <int CB, typename QT>
static void launch_fill_t(hipStream_t s, const FillArgs& p, bool tb, bool full) {
    if (full) launch_one<CB, QT, true, true, 0>(s, p);
    else if (tb) launch_one<CB, QT, true, false, 0>(s, p);
    else launch_one<CB, QT, false, false, 0>(s, p);
}

void launch_fill(hipStream_t s, const FillArgs& p, int CB, int qbytes, bool tb, bool full) {
    if (qbytes == 1) {
        if (CB == 1) launch_fill_t<1, int8_t>(s, p, tb, full);
        else if (CB == 2) launch_fill_t<2, int8_t>(s, p, tb, full);
        else launch_fill_t<4, int8_t>(s, p, tb, full);
    } else {
        if (CB == 1) launch_fill_t<1, int16_t>(s, p, tb, full);
        else if (CB == 2) launch_fill_t<2, int16_t>(s, p, tb, full);
        else launch_fill_t<4, int16_t>(s, p, tb, full);
    }
}

// diagnostic ablation launcher (CB=1, int8 profile only)
void launch_fill_ablation(hipStream_t s, const FillArgs& p, bool tb, int abl) {
#define GA_ABL_CASE(A)                                          \
    case A:                                                     \
        if (tb) launch_one<1, int8_t, true, false, A>(s, p);    \
        else launch_one<1, int8_t, false, false, A>(s, p);      \
        break;
    switch (abl) {
        GA_ABL_CASE(0) GA_ABL_CASE(1) GA_ABL_CASE(2) GA_ABL_CASE(4) GA_ABL_CASE(8) GA_ABL_CASE(16) GA_ABL_CASE(17)
        GA_ABL_CASE(21) GA_ABL_CASE(29) GA_ABL_CASE(31)
        default: break;
    }
#undef GA_ABL_CASE
}

void launch_walk(hipStream_t s, const WalkArgs& w) {
    if (w.CB == 1) walk_kernel<1><<<1, 64 * WALK_WAVES, 0, s>>>(w);
    else if (w.CB == 2) walk_kernel<2><<<1, 64 * WALK_WAVES, 0, s>>>(w);
    else walk_kernel<4><<<1, 64 * WALK_WAVES, 0, s>>>(w);
}

}  // namespace ga
