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

// ----------------------------------------------------------------------------------
// Query profile: qp[c][QPAD + i] = sub(a_i, c) - gV(a_i) - gH(c)  (i in [0,m)).
// A lane owning column code c reads its row's sub' with one byte/short load whose
// address is (uniform step) + (lane constant): no VALU work for the lookup.
template <typename QT>
__global__ void qp_kernel(const uint8_t* __restrict__ a, int m, const int* __restrict__ sub,
                          const int* __restrict__ gh, const int* __restrict__ gv, int K, QT* __restrict__ qp,
                          long long stride) {
    long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long total = stride * K;
    for (; idx < total; idx += (long long)gridDim.x * blockDim.x) {
        int c = (int)(idx / stride);
        long long p = idx - (long long)c * stride;
        long long i = p - QPAD;
        QT v = 0;
        if (i >= 0 && i < m) {
            int x = a[i];
            v = (QT)(sub[x * K + c] - gv[x] - gh[c]);
        }
        qp[idx] = v;
    }
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

template <int CB, bool MASK, bool FULL>
__device__ __forceinline__ void dp_step(StepState& s, int2 lin, int sub, int o, unsigned op1, int t, int lane, int m,
                                        bool colok, uint32_t& accw, int sh, int* full, int fullW, int jcol) {
    constexpr int W = TbFmt<CB>::W;
    // left neighbour (lane l-1, previous step); lane 0 takes the slab edge from the ring
    const int HL = __builtin_amdgcn_update_dpp(lin.x, s.Hout, 0x138, 0xf, 0xf, false);  // wave_shr:1
    const int XL = __builtin_amdgcn_update_dpp(lin.y, s.Xout, 0x138, 0xf, 0xf, false);
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



template <int CB, typename QT, bool TB, bool FULL>
__global__ void __launch_bounds__(64 * (NW + 1)) fill_kernel(FillArgs p) {
    constexpr int SPC = TbFmt<CB>::SPC;
    __shared__ int2 ring[NW + 1][RING];
    __shared__ unsigned prod[NW + 1], cons[NW + 1];
    __shared__ int slab_sh;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    if (threadIdx.x == 0) slab_sh = (int)atomicAdd(p.ticket, 1u);
    if (threadIdx.x <= NW) { prod[threadIdx.x] = 0; cons[threadIdx.x] = 0; }
    __syncthreads();
    const int g = slab_sh;
    const unsigned m = (unsigned)p.m;

    if (w == NW) {
        // ---------------- IO wave: slab edges HBM <-> LDS rings ----------------
        const int2* src = g == 0 ? p.left : p.hand + (long long)(g - 1) * (m + 1);
        const unsigned* src_prog = g == 0 ? p.left_prog : p.hand_prog + (g - 1);
        const unsigned limit = (g == 0 && p.left_prog != nullptr) ? p.halo_spin_limit : p.spin_limit;
        const bool src_sc1 = g != 0 || p.left_prog != nullptr;
        int2* dst = p.hand + (long long)g * (m + 1);
        unsigned in_next = 0, out_next = 0, spins = 0;
        while (in_next < m || out_next < m) {
            bool moved = false;
            if (in_next < m) {
                const unsigned space = lds_ld(&cons[0]) + RING;
                const unsigned avail = src_prog ? min(g_ld(src_prog), m) : m;
                const unsigned hi = min(min(space, avail), in_next + 64);
                if (hi > in_next && (hi - in_next >= 16 || hi == avail)) {
                    const unsigned r = in_next + 1 + lane;
                    if (r <= hi) ring[0][r & RMASK] = src_sc1 ? unpack64(g_ld64(src + r)) : src[r];
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
                    if (r <= hi) g_st64(dst + r, ring[NW][r & RMASK]);
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
                if (!spin_ok(spins, limit, p.abort_word)) break;
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
    const QT* qpl = reinterpret_cast<const QT*>(p.qp) + (long long)bcode * p.qp_stride + QPAD - lane;
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
    const int T = (int)m + 63;
    const int nchunks = (T + SPC - 1) / SPC;
    int2* rin = ring[w];
    int2* rout = ring[w + 1];
    unsigned spins = 0;
    int q[SPC], qn[SPC];
#pragma unroll
    for (int u = 0; u < SPC; u++) q[u] = qpl[u];
    uint8_t* tbl = TB ? p.tb + ((long long)s * p.TC * 64 + lane) * 16 : nullptr;
    bool ok = true;

    for (int c = 0; c < nchunks && ok; c++) {
        const int t0 = c * SPC;
        // inputs: rows t0+1 .. t0+SPC must be in the ring
        const unsigned need = min((unsigned)(t0 + SPC), m);
        while (lds_ld(&prod[w]) < need) {
            if (!spin_ok(spins, p.spin_limit, p.abort_word)) { ok = false; break; }
        }
        // outputs: rows t0-62 .. t0+SPC-63 will be written; keep RING rows of slack
        const int hi_out = t0 + SPC - 63;
        if (hi_out - RING > 0) {
            while ((int)lds_ld(&cons[w + 1]) < hi_out - RING) {
                if (!spin_ok(spins, p.spin_limit, p.abort_word)) { ok = false; break; }
            }
        }
        if (!ok) break;
        spins = 0;
        if (lane == 0) lds_st(&cons[w], min((unsigned)t0, m));
        // prefetch next chunk's substitution values
#pragma unroll
        for (int u = 0; u < SPC; u++) qn[u] = qpl[t0 + SPC + u];
        uint32_t acc[4] = {0, 0, 0, 0};
        const bool steady = full_stripe && t0 >= 63 && t0 + SPC - 1 <= (int)m - 1;
        if (steady) {
#pragma unroll
            for (int u = 0; u < SPC; u++) {
                const int t = t0 + u;
                const int2 lin = rin[(t + 1) & RMASK];
                dp_step<CB, false, FULL>(st, lin, q[u], o, op1, t, lane, m, true, acc[(u * CB) >> 2],
                                         (u * CB * 8) & 31, p.full, p.n + 1, jcol);
                if (lane == 63) rout[(t - 62) & RMASK] = make_int2(st.Hout, st.Xout);
            }
        } else {
#pragma unroll
            for (int u = 0; u < SPC; u++) {
                const int t = t0 + u;
                const int2 lin = rin[(t + 1) & RMASK];
                dp_step<CB, true, FULL>(st, lin, q[u], o, op1, t, lane, m, colok, acc[(u * CB) >> 2],
                                        (u * CB * 8) & 31, p.full, p.n + 1, jcol);
                const int r = t - 62;
                if (r >= 1 && r <= (int)m && lane == 63) rout[r & RMASK] = make_int2(st.Hout, st.Xout);
            }
        }
        if (TB && live) *reinterpret_cast<uint4*>(tbl + (long long)c * 1024) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
        if (hi_out >= 1 && lane == 0) lds_st(&prod[w + 1], min((unsigned)hi_out, m));
#pragma unroll
        for (int u = 0; u < SPC; u++) q[u] = qn[u];
    }
    // the lane owning column n writes the final H' (cost = H' + phi(m, n))
    if (ok && colok && jcol == p.n) p.out_last[0] = st.Hout;
}

// ----------------------------------------------------------------------------------
// Traceback walk (dp_array_backward, globaligner.py:395-593).
//
// One workgroup.  A WR x WC window of decoded rank sets (S0|S1<<3|S2<<6 per cell)
// is staged in LDS around the walker; thread 0 walks, every thread restages the
// window when the walk leaves it.  Degenerate inputs (the walk
// visits row 0 / column 0 and wraps with Python negative indexing) are
// reproduced cell by cell from HBM.


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

__device__ __forceinline__ unsigned tb_code(const uint8_t* tb, int CB, int TC, int i, int j) {
    const int s = (j - 1) >> 6, l = (j - 1) & 63, t = i - 1 + l;
    const int spc = 16 / CB;
    const uint8_t* p = tb + (((long long)s * TC + t / spc) * 64 + l) * 16 + (t % spc) * CB;
    unsigned v = p[0];
    if (CB >= 2) v |= (unsigned)p[1] << 8;
    if (CB == 4) v |= ((unsigned)p[2] << 16) | ((unsigned)p[3] << 24);
    return v;
}

// choose a level from the candidate set using the step's tie-break bits
// (dispatcher entries :599-671: 3-way (0,0,0)-type uses draw 0/9, pairs use 1-3/10-12)
__device__ __forceinline__ int choose(int S, unsigned bits) {
    switch (S) {
        case 1: return 0;
        case 2: return 1;
        case 4: return 2;
        case 7: return (int)(bits & 3u);
        case 3: return (int)((bits >> 2) & 1u);          // (match, gap1)
        case 5: return 2 * (int)((bits >> 3) & 1u);      // (match, gap2)
        default: return 1 + (int)((bits >> 4) & 1u);    // 6: (gap1, gap2)
    }
}

__global__ void __launch_bounds__(256) walk_kernel(WalkArgs w) {
    __shared__ uint16_t win[WR * WC];
    __shared__ uint8_t wa[WR], wb[WC];
    __shared__ uint16_t wr[RW];
    __shared__ int st[8];  // i, j, L, D, h, first, done, reason
    const int tid = threadIdx.x;
    const int m = w.m, n = w.n, o = w.o;
    if (tid == 0) {
        st[0] = m; st[1] = n; st[2] = 0; st[3] = 0; st[4] = 0; st[5] = 1; st[6] = 0; st[7] = 0;
    }
    __syncthreads();
    for (;;) {
        if (st[6]) break;
        const int ci = st[0], cj = st[1], k0 = st[3];
        const int i0 = max(1, ci - WR + 1), j0 = max(1, cj - WC + 1);
        __syncthreads();
        // ---- stage the window: cells [i0, i0+WR) x [j0, j0+WC) ----
        if (ci >= 1 && cj >= 1) {
            for (int e = tid; e < WR * WC; e += blockDim.x) {
                const int r = e / WC, cc = e - r * WC;
                const int ii = i0 + r, jj = j0 + cc;
                uint16_t v = 0;
                if (ii <= m && jj <= n) v = (uint16_t)sets_from_code(tb_code(w.tb, w.CB, w.TC, ii, jj), w.CB, o);
                win[e] = v;
            }
            for (int e = tid; e < WR; e += blockDim.x) wa[e] = (i0 + e <= m) ? w.a[i0 + e - 1] : 0;
            for (int e = tid; e < WC; e += blockDim.x) wb[e] = (j0 + e <= n) ? w.b[j0 + e - 1] : 0;
        }
        for (int e = tid; e < RW; e += blockDim.x) wr[e] = (k0 + e < w.nrng) ? w.rng[k0 + e] : 0;
        __syncthreads();
        if (tid == 0) {
            int i = st[0], j = st[1], L = st[2], D = st[3], h = st[4], first = st[5];
            int done = 0, reason = 0;
            const int maxh = m + n;
            for (;;) {
                if (D - k0 >= RW) break;  // restage the tie-break window
                int S, am;
                const bool inwin = i >= i0 && j >= j0 && i < i0 + WR && j < j0 + WC && ci >= 1 && cj >= 1;
                if (inwin) {
                    S = (win[(i - i0) * WC + (j - j0)] >> (3 * L)) & 7;
                    am = wa[i - i0] == wb[j - j0];
                } else if (i >= 1 && j >= 1) {
                    break;  // interior cell outside the window: restage around it
                } else {
                    // degenerate walk at row 0 / column 0 with Python index wrapping
                    const int ri = i < 0 ? i + m + 1 : i, rj = j < 0 ? j + n + 1 : j;
                    const int pa = (i - 1) < 0 ? i - 1 + m : i - 1, pb = (j - 1) < 0 ? j - 1 + n : j - 1;
                    if (ri < 0 || rj < 0 || pa < 0 || pa >= m || pb < 0 || pb >= n) {
                        done = 1; reason = 4;  // IndexError
                        break;
                    }
                    if (ri >= 1 && rj >= 1) {
                        S = (sets_from_code(tb_code(w.tb, w.CB, w.TC, ri, rj), w.CB, o) >> (3 * L)) & 7;
                    } else {
                        const int* v = ri == 0 ? w.bnd_row + 3 * rj : w.bnd_col + 3 * ri;
                        const long long M = v[0], X = v[1], Y = v[2];
                        S = L == 0 ? argmin3(M, X, Y) : L == 1 ? argmin3(M + o, X, Y + o) : argmin3(M + o, X + o, Y);
                    }
                    am = w.a[pa] == w.b[pb];
                }
                const unsigned rb = wr[D - k0];
                const int lvl = choose(S, am ? (rb & 31u) : (rb >> 5));
                w.ops[D] = (uint8_t)lvl;
                D++;
                if (lvl == 0) { i--; j--; } else if (lvl == 1) { j--; } else { i--; }
                L = lvl;
                if (first) {
                    first = 0;
                    if (i == 0 && j == 0) { done = 1; reason = 0; break; }
                    continue;
                }
                if (i == 0) { done = 1; reason = 1; break; }
                if (j == 0) { done = 1; reason = 2; break; }
                if (++h >= maxh) { done = 1; reason = 3; break; }
            }
            st[0] = i; st[1] = j; st[2] = L; st[3] = D; st[4] = h; st[5] = first; st[6] = done; st[7] = reason;
            if (done) { w.result[0] = D; w.result[1] = i; w.result[2] = j; w.result[3] = reason; }
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------------------------
// host-side launchers (called from ga_host.cpp)
void launch_qp(hipStream_t s, const uint8_t* a, int m, const int* sub, const int* gh, const int* gv, int K, void* qp,
               long long stride, int qbytes) {
    const long long total = stride * K;
    int blocks = (int)min((total + 255) / 256, 4096LL);
    if (qbytes == 1)
        qp_kernel<int8_t><<<blocks, 256, 0, s>>>(a, m, sub, gh, gv, K, (int8_t*)qp, stride);
    else
        qp_kernel<int16_t><<<blocks, 256, 0, s>>>(a, m, sub, gh, gv, K, (int16_t*)qp, stride);
}

void launch_boundary(hipStream_t s, const uint8_t* a, int m, const uint8_t* b, int n, const int* gh, const int* gv,
                     int o, int big, int* GVp, int* GHp, int2* top, int2* left, int* bnd_row, int* bnd_col, int* meta,
                     bool custom) {
    if (custom)
        custom_boundary_kernel<<<1, 1024, 0, s>>>(a, m, b, n, gh, gv, o, GVp, GHp, top, left, bnd_row, bnd_col, meta);
    else
        boundary_kernel<<<1, 1024, 0, s>>>(a, m, b, n, gh, gv, o, big, GVp, GHp, top, left, bnd_row, bnd_col, meta);
}

template <int CB, typename QT>
static void launch_fill_t(hipStream_t s, const FillArgs& p, bool tb, bool full) {
    dim3 grid(p.nslabs), block(64 * (NW + 1));
    if (full) fill_kernel<CB, QT, true, true><<<grid, block, 0, s>>>(p);
    else if (tb) fill_kernel<CB, QT, true, false><<<grid, block, 0, s>>>(p);
    else fill_kernel<CB, QT, false, false><<<grid, block, 0, s>>>(p);
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

void launch_walk(hipStream_t s, const WalkArgs& w) { walk_kernel<<<1, 256, 0, s>>>(w); }

}  // namespace ga
