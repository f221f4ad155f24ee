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
// Layout (HBM): one wave owns a 64-column stripe and steps down its rows; the
// horizontal dependence within a row is a prefix-min scan across the lanes
// (DPP).  NWC compute waves per workgroup are chained through LDS rings; an
// IO wave moves the slab's left/right edges to/from HBM with write-through
// (sc1) stores and a progress word (cdna_hip_programming.md Guideline 16, R1).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ga_device.h"
#include "ga_row.h"
#include "ga_sync.h"
#include "ga_walk.h"

namespace ga {

// row of a 4-row sub-chunk after which the row-scan waves await and read the next sub-chunk's
// edges (0..3; tools/sweep14.sh: 2 is 2 % faster than 0 at C3, 1 % at C4)
#ifndef GA_EDGE_U
#define GA_EDGE_U 2
#endif

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

// The same boundary with the prefix sums spread over the chip (the single-workgroup scan
// above is latency-bound: ~5 ms at 10^6 columns).  Segments of BSEG codes per workgroup:
// bnd_sums (segment sums) -> bnd_scan (one workgroup scans the segment sums) -> bnd_apply
// (each segment rescans itself from its base) -> bnd_edges (elementwise boundary values).
constexpr int BSEG = 4096;  // 256 threads x 16 consecutive codes
__global__ void __launch_bounds__(256) bnd_sums_kernel(const uint8_t* __restrict__ a, int m, const uint8_t* __restrict__ b,
                                                       int n, const int* __restrict__ gh, const int* __restrict__ gv,
                                                       int nba, int* __restrict__ bs) {
    __shared__ int red[256];
    const int k = blockIdx.x;
    const bool isa = k < nba;
    const uint8_t* sq = isa ? a : b;
    const int* g = isa ? gv : gh;
    const int len = isa ? m : n;
    const int lo = (isa ? k : k - nba) * BSEG;
    int acc = 0;
    for (int q = lo + threadIdx.x; q < min(len, lo + BSEG); q += 256) acc += g[sq[q]];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) bs[k] = red[0];
}

// exclusive scan, in place, of bs[0, nba) and of bs[nba, nba + nbb) (one workgroup)
__global__ void __launch_bounds__(1024) bnd_scan_kernel(int* __restrict__ bs, int nba, int nbb) {
    __shared__ int sh[1024];
    for (int part = 0; part < 2; part++) {
        int* v = part == 0 ? bs : bs + nba;
        const int len = part == 0 ? nba : nbb;
        int carry = 0;
        for (int base = 0; base < len; base += 1024) {
            const int q = base + (int)threadIdx.x;
            const int x = q < len ? v[q] : 0;
            sh[threadIdx.x] = x;
            __syncthreads();
            for (int off = 1; off < 1024; off <<= 1) {
                const int y = (int)threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
                __syncthreads();
                sh[threadIdx.x] += y;
                __syncthreads();
            }
            if (q < len) v[q] = carry + sh[threadIdx.x] - x;
            carry += sh[1023];
            __syncthreads();
        }
    }
}

// pre[q] = sum of g over codes < q, for the segment's q; the last segment also writes pre[len]
__global__ void __launch_bounds__(256) bnd_apply_kernel(const uint8_t* __restrict__ a, int m, const uint8_t* __restrict__ b,
                                                        int n, const int* __restrict__ gh, const int* __restrict__ gv,
                                                        int nba, const int* __restrict__ bs, int* __restrict__ GVp,
                                                        int* __restrict__ GHp) {
    __shared__ int sh[256];
    const int k = blockIdx.x;
    const bool isa = k < nba;
    const uint8_t* sq = isa ? a : b;
    const int* g = isa ? gv : gh;
    int* pre = isa ? GVp : GHp;
    const int len = isa ? m : n;
    const int lo = (isa ? k : k - nba) * BSEG + 16 * (int)threadIdx.x;
    int v[16];
    int acc = 0;
#pragma unroll
    for (int u = 0; u < 16; u++) {
        v[u] = lo + u < len ? g[sq[lo + u]] : 0;
        acc += v[u];
    }
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const int y = (int)threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
        __syncthreads();
        sh[threadIdx.x] += y;
        __syncthreads();
    }
    int run = bs[k] + sh[threadIdx.x] - acc;
#pragma unroll
    for (int u = 0; u < 16; u++) {
        if (lo + u < len) pre[lo + u] = run;
        run += v[u];
        if (lo + u == len - 1) pre[len] = run;
    }
}

__global__ void __launch_bounds__(256) bnd_edges_kernel(int m, int n, int o, int big, const int* __restrict__ GVp,
                                                        const int* __restrict__ GHp, int2* __restrict__ top,
                                                        int2* __restrict__ left, int* __restrict__ bnd_row,
                                                        int* __restrict__ bnd_col, int* __restrict__ meta) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t <= n) {
        const int j = t;
        int M, X, Y;
        if (j == 0) { M = X = Y = 0; }                        // :778
        else { M = big; X = o + GHp[j]; Y = big; }            // :780-784, :802-809
        bnd_row[3 * j] = M; bnd_row[3 * j + 1] = X; bnd_row[3 * j + 2] = Y;
        const int H = min(min(M, X), Y);
        top[j] = make_int2(H - GHp[j], min(Y, H + o) - GHp[j]);
    }
    if (t <= m) {
        const int i = t;
        int M, X, Y;
        if (i == 0) { M = X = Y = 0; }
        else { M = big; X = big; Y = o + GVp[i]; }            // :789-793, :812-819
        bnd_col[3 * i] = M; bnd_col[3 * i + 1] = X; bnd_col[3 * i + 2] = Y;
        const int H = min(min(M, X), Y);
        left[i] = make_int2(H - GVp[i], min(X, H + o) - GVp[i]);
    }
    if (t == 0) { meta[0] = GVp[m]; meta[1] = GHp[n]; }
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
// The row-scan fill (dp_array_forward :366-392, get_next_best_costs :317-363).
//
// One wave owns a 64-column stripe; lane l owns column 64s+l+1 and the wave
// steps down the rows.  Within a row, M' and Y' need only the row above, and
// the horizontal chain is a prefix minimum:
//     h1'(i,j) = min(h1'(i,j-1), min(M',Y')(i,j) + o)
// so with V~ = h1' - o and U = min(M', Y') the whole row's V~ is one inclusive
// prefix-min scan of U across the 64 lanes (six DPP steps), seeded with the
// stripe's left edge, and X'(i,j) = V~(i,j-1) + o is a one-lane DPP shift.
// A wave therefore hands its right edge to the next stripe's wave after a few
// rows (FROWS-row chunks, published every 4 rows), not after 64 skewed steps:
// the wavefront ramp across the matrix shrinks from ~nstripes*100 steps to
// ~nstripes*5 rows.
//
// Traceback word of a cell (CB bytes, W = (8*CB-1)/2 bits per field):
//   bits [0,W)   : min(X - H, o+1)     X in S1 <=> <= o ; M,Y may be in S1 <=> >= o
//   bits [W,2W)  : min(Y - H, o+1)
//   bit  2W      : M != H
// which is all dp_array_backward's rank test needs at this cell.
template <int CB>
struct TbFmt {
    static constexpr int W = (8 * CB - 1) / 2;
    static constexpr int SPC = 16 / CB;  // rows per 16-byte word
};

// FROWS query-profile values (sub' of one lane's column for 16 rows), raw dwords.
template <typename QT>
struct QPack {
    static constexpr int NWD = FROWS * (int)sizeof(QT) / 4;
    uint32_t w[NWD];
    __device__ __forceinline__ void load(const QT* p) {
        const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
        for (int k = 0; k < NWD / 4; k++) {
            const uint4 v = q[k];
            w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
        }
    }
    // a lane's rows at any byte offset (the anti-diagonal fill's profile; LDS allows unaligned reads)
    __device__ __forceinline__ void load_unaligned(const QT* p) { __builtin_memcpy(w, p, sizeof(w)); }
    __device__ __forceinline__ int get(int u) const {
        if (sizeof(QT) == 1) return (int)(int8_t)(w[u >> 2] >> (8 * (u & 3)));
        return (int)(int16_t)(w[u >> 1] >> (16 * (u & 1)));
    }
};

// A compute wave's publication of four rows, one lane with a narrowed exec mask (no branch:
// the compute loop keeps scalar control flow; a structured `if (lane == k)` turns uniform
// values into VGPR phis): the lane owning the stripe's right edge writes the ring rows,
// then {cons, prod} in one 8-byte store.  LDS executes one wave's operations in order,
// so the rows land before the counters.
typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void lds_publish(unsigned ring_addr, unsigned pc_addr, unsigned long long lanemask, v4i a,
                                            v4i b, unsigned cons, unsigned prod) {
    unsigned long long saved;
    const v2u cp = {cons, prod};
    asm volatile(
        "s_mov_b64 %0, exec\n\ts_mov_b64 exec, %3\n\t"
        "ds_write_b128 %1, %4\n\tds_write_b128 %1, %5 offset:16\n\tds_write_b64 %2, %6\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "v"(ring_addr), "v"(pc_addr), "s"(lanemask), "v"(a), "v"(b), "v"(cp)
        : "memory");
}

// LDS: counters | ring[NWC+1][RING] (int2) | qring[K][qrows] (QT)
//   ring k feeds compute wave k (ring 0 from the IO wave, ring k+1 from wave k; the IO
//   wave drains ring nlive).  Slot (i-1) & RMASK of a ring holds what row i of the
//   next stripe needs from its left edge: (H'(i-1, edge), V~(i, edge)) with
//   V~ = h1' - o, one broadcast 8-byte read per row.
//   prod[k] = P: slots of rows <= P are written (the H' of row P itself lands with row P+1);
//   cons[k] = C: the reader of ring k no longer needs slots < C;
//   both live in one array, prodcons[2k] = cons[k], prodcons[2k+1] = prod[k+1], so compute
//   wave k publishes both with one 8-byte store (prod[0] is written by the IO wave);
//   prodq = Q: query-profile rows <= Q are written (the IO wave runs it ahead of the edges).
enum { CI_PC = 0, CI_PROD0 = 31, CI_ABORT = 32, CI_SLAB = 33, CI_PRODQ = 34 };
constexpr int FILL_CNT_BYTES = 256;

template <int CB, typename QT, bool TB, int T, bool DBG>
__device__ void fill_blocked(FillArgs& p, unsigned* cnt, int2* ring, QT* qring, uint4* tbstage, int w, int g, int lane);

// LDS staging of a blocked wave's traceback words (T > 1): 16-byte words per lane per chunk
template <int CB, int T>
struct TbStage {
    static constexpr int UINT4S = T > 1 ? T * CB * 64 : 0;  // per compute wave
};
__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// DBG: per-stripe timestamps into p.dbg (s_memtime shares lgkmcnt with LDS reads, so the
// timing code stays out of the production variants)
template <int CB, typename QT, bool TB, bool FULL, int NWC, int T, bool DBG>
__global__ void __launch_bounds__(64 * (NWC + 1)) fill_kernel(FillArgs p) {
    static_assert(T == 1 || !FULL, "the FULL debug output is T == 1 only");
    constexpr int W = TbFmt<CB>::W;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    unsigned* cnt = reinterpret_cast<unsigned*>(smem);
    int2* ring = reinterpret_cast<int2*>(smem + FILL_CNT_BYTES);
    QT* qring = reinterpret_cast<QT*>(ring + (NWC + 1) * RING);
    // prod[k] (k >= 1) and cons[k] interleaved (see above); prod[0] apart
    struct PC {
        unsigned* c;
        __device__ unsigned& prod(int k) { return k == 0 ? c[CI_PROD0] : c[2 * k - 1]; }
        __device__ unsigned& cons(int k) { return c[2 * k]; }
    } pc{cnt};
    unsigned* abort_sh = cnt + CI_ABORT;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave index: uniform
    if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x == 0) cnt[CI_SLAB] = atomicAdd(p.ticket, 1u);
    __syncthreads();
    const int g = __builtin_amdgcn_readfirstlane((int)cnt[CI_SLAB]);  // slab of this workgroup (ticket order)
    const int m = p.m, o = p.o;
    const int nch = (m + FROWS - 1) / FROWS;
    const int mpad = nch * FROWS;
    const int nlive = min(NWC, p.nstripes - g * NWC);
    const int QR = p.qrows;
    const unsigned qmask = (unsigned)QR - 1u;

    if (w == NWC) {
        // ---------------- IO wave: slab edges HBM <-> LDS rings, query profile ----------------
        const int2* src = g == 0 ? p.left : p.hand + (long long)(g - 1) * (m + 1);
        const unsigned* src_prog = g == 0 ? p.left_prog : nullptr;  // g > 0: the rows themselves (in_sent)
        const unsigned limit = (g == 0 && p.left_prog != nullptr) ? p.halo_spin_limit : p.spin_limit;
        const bool src_sc1 = p.left_prog != nullptr;  // another GPU's edge, landing while the fill runs
        const bool last_slab = g == p.nslabs - 1;
        int2* dst = (last_slab && p.edge_out != nullptr) ? p.edge_out : p.hand + (long long)g * (m + 1);
        int2* rin0 = ring;
        const int2* rout = ring + nlive * RING;
        const int K = p.K;
        const int h00 = p.top[g * NWC * 64 * T].x;  // H'(0, left edge of this workgroup's columns)
        // workgroup hand-offs poll the rows themselves (HAND_SENT until written, ga_device.h);
        // only the slab's own right edge out to another GPU keeps the progress word
        const bool in_sent = g > 0, out_sent = !(last_slab && p.edge_out != nullptr);
        int hlast = h00;  // H' of row in_next of the left edge
        unsigned in_next = 0, out_next = 0, q_next = 0, spins = 0, in_win = 64;
        while (in_next < (unsigned)m || out_next < (unsigned)m || q_next < (unsigned)m) {
            bool moved = false;
            if (q_next < (unsigned)m) {
                // profile rows of chunks the slowest wave (ring nlive's producer) has finished are free
                const unsigned pl = lds_ld(&pc.prod(nlive));
                const unsigned space = (pl & ~(unsigned)(FROWS - 1)) + QR - FROWS;
                const unsigned hi = min(min(space, (unsigned)m), q_next + 64);
                // whole 64-row batches (or the tail): the IO wave shares a SIMD with compute wave 0
                if (hi > q_next && (hi - q_next >= 64 || hi == (unsigned)m)) {
                    const unsigned r = q_next + 1 + lane;
                    if (r <= hi) {
                        const int x = p.a[r - 1];
                        const int* sp = p.subp + x * K;
                        QT* qd = qring + ((r - 1) & qmask);
                        for (int c = 0; c < K; c++) qd[c * QR] = (QT)sp[c];
                    }
                    // done: past the padded rows (the blocked waves read one chunk ahead)
                    if (lane == 0) lds_st(&cnt[CI_PRODQ], hi == (unsigned)m ? (unsigned)(mpad + FROWS) : hi);
                    q_next = hi;
                    moved = true;
                }
            }
            if (in_next < (unsigned)m && in_sent) {
                // the contiguous written prefix of the next (up to) 64 rows, as far as ring 0 has space
                const unsigned cap = min(min(lds_ld(&pc.cons(0)) + RING, (unsigned)m), in_next + in_win);
                if (cap > in_next) {
                    const unsigned r = in_next + 1 + lane;
                    const int2 e1 = r <= cap ? unpack64(g_ld64(src + r)) : make_int2(HAND_SENT, 0);
                    const unsigned long long ok = __ballot(e1.x != HAND_SENT);
                    const unsigned k = ~ok ? (unsigned)__builtin_ctzll(~ok) : 64u;  // rows in_next+1 .. +k
                    // poll window: the writer publishes GOUT rows at a time, so a waiting reader looks
                    // at the next 8 rows only; a reader that found its whole window written is behind
                    // and takes 64 at a time (the full window polled 3.5 GB of unwritten rows per C4 fill)
                    in_win = k >= cap - in_next ? 64u : 8u;
                    if (k > 0) {
                        // H' of row r-1: the lane before (lane 0: the last row of the previous batch)
                        const int h0 = __builtin_amdgcn_update_dpp(hlast, e1.x, 0x138, 0xf, 0xf, false);
                        if (lane < (int)k) rin0[(r - 1) & RMASK] = make_int2(h0, e1.y - o);
                        hlast = __builtin_amdgcn_readlane(e1.x, (int)k - 1);
                        const unsigned hi = in_next + k;
                        if (lane == 0) lds_st(&pc.prod(0), hi == (unsigned)m ? (unsigned)mpad : hi);
                        in_next = hi;
                        moved = true;
                    }
                }
            } else if (in_next < (unsigned)m) {
                // ring 0 slots are free below cons[0]
                const unsigned space = lds_ld(&pc.cons(0)) + RING;
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
                    if (r <= hi) {
                        const int2 e1 = src_sc1 ? unpack64(s_ld64(src + r)) : src[r];
                        const int h0 = r == 1 ? h00 : (src_sc1 ? unpack64(s_ld64(src + r - 1)) : src[r - 1]).x;
                        rin0[(r - 1) & RMASK] = make_int2(h0, e1.y - o);
                    }
                    // rows past m are padding (garbage nobody reads back)
                    if (lane == 0) lds_st(&pc.prod(0), hi == (unsigned)m ? (unsigned)mpad : hi);
                    in_next = hi;
                    moved = true;
                }
            }
            if (out_next < (unsigned)m) {
                // row r of the right edge: H' from slot r (row r+1's entry), V~ from slot r-1
                const unsigned P = lds_ld(&pc.prod(nlive));
                const unsigned hi = min(min(P, (unsigned)mpad + 1u) - 1u, min((unsigned)m, out_next + 64));
                if (P > 0 && hi > out_next && (hi - out_next >= GOUT || hi == (unsigned)m)) {
                    const unsigned r = out_next + 1 + lane;
                    if (r <= hi) {
                        const int H = rout[r & RMASK].x;
                        const int2 e = make_int2(H, rout[(r - 1) & RMASK].y + o);
                        if (out_sent) g_st64(dst + r, e);
                        else s_st64(dst + r, e);  // another GPU's halo
                        if (T == 1 && last_slab && r == (unsigned)m) p.out_last[0] = H;  // H'(m, n): the cost
                    }
                    if (!out_sent) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (lane == 0) __hip_atomic_store(p.edge_prog, hi, RLX, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    if (lane == 0) lds_st(&pc.cons(nlive), hi - 1u);
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
        // gave up before the right edge was complete: tell the reader of the edge (the next slab's fill)
        if (!out_sent && out_next < (unsigned)m && p.edge_prog != nullptr && lane == 0) s_prog_abort(p.edge_prog);
        return;
    }
    if (w >= nlive) return;
    if constexpr (T > 1) {
        uint4* tbstage = reinterpret_cast<uint4*>(
                             smem + align16((size_t)FILL_CNT_BYTES + (size_t)(NWC + 1) * RING * sizeof(int2) +
                                            (size_t)p.K * p.qrows * sizeof(QT))) +
                         (size_t)w * TbStage<CB, T>::UINT4S;
        fill_blocked<CB, QT, TB, T, DBG>(p, cnt, ring, qring, tbstage, w, g, lane);
        return;
    }

    // ---------------- compute wave w: stripe s ----------------
    // compute waves win VALU arbitration against the IO wave on their SIMD (the chain head,
    // wave 0, shares one with it)
    __builtin_amdgcn_s_setprio(2);
    const int s = g * NWC + w;
    const int j0 = s * 64;                    // columns j0+1 .. j0+64
    const int jcol = j0 + lane + 1;
    const bool colok = jcol <= p.n;
    const int srcl = min(63, p.n - 1 - j0);   // the lane whose column is this stripe's right edge
    const int bcode = colok ? p.b[jcol - 1] : 0;
    const QT* qcol = qring + bcode * QR;
    int Hprev, Yc;                            // H'(i-1, j), h2'(i-1, j)
    {
        const int2 t = p.top[colok ? jcol : p.n];
        Hprev = t.x;
        Yc = t.y;
    }
    const unsigned op1 = (unsigned)o + 1u;
    const int2* rin = ring + w * RING;
    int2* rout = ring + (w + 1) * RING;
    uint4* tbw = TB ? reinterpret_cast<uint4*>(p.tb) + (long long)s * p.TC * 64 + lane : nullptr;
    unsigned avail = 0, outfree = 0, qavail = 0;
    unsigned long long stamp0 = 0, stamp1 = 0, clk0 = 0;
    const unsigned pc_lds = lds_addr(&pc.cons(w));  // {cons[w], prod[w + 1]}
    const unsigned rout_lds = lds_addr(rout);
    const unsigned long long srcmask = 1ull << srcl;
    // wait (wave-uniform) until *ctr + add >= target.  A wait that gives up (the workgroup
    // aborted) makes every later wait a no-op: the wave runs to its end on garbage and the
    // host reports the abort word, so the loops below have no early exits (clean unrolling).
    bool aborted = false;
    auto wait_ge = [&](unsigned* ctr, unsigned add, unsigned& cached, int target) {
        unsigned spins = 0;
        cached = sgpr_u(cached);
        while ((int)cached < target && !aborted) {
            cached = lds_ldu(ctr) + add;
            if ((int)cached >= target) break;
            if (!spin_ok_lds(spins, p.spin_limit, abort_sh)) aborted = true;
        }
        // the reads of what the counter guards stay after it (the LDS itself keeps order)
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    };
    wait_ge(&pc.prod(w), 0, avail, 4);  // rows 1..4 before the first edge read
    int4 e01 = reinterpret_cast<const int4*>(rin)[0];  // slots 0..3: (H'(i-1), V~(i)) of rows 1..4
    int4 e23 = reinterpret_cast<const int4*>(rin)[1];
    // the counter is read one sub-chunk before it is needed (a plain load: the asm stores'
    // memory clobbers keep the compiler from reusing an old value, and it waits at the use)
    const unsigned* prod_in = &pc.prod(w);
    unsigned pnext = *prod_in;

    // traceback codes are software-pipelined one sub-chunk behind the DP chain, so their
    // VALU work fills the chain's DPP hazard slots: pM/pX/pY/pH hold the previous
    // sub-chunk's rows, accP the previous chunk's words (finished in sub-chunk 0)
    int pM[4] = {0, 0, 0, 0}, pX[4] = {0, 0, 0, 0}, pY[4] = {0, 0, 0, 0}, pH[4] = {0, 0, 0, 0};
    uint32_t accP[4 * CB];
#pragma unroll
    for (int k = 0; k < 4 * CB; k++) accP[k] = 0;
    auto code_of = [&](int u) -> unsigned {
        return min((unsigned)(pX[u] - pH[u]), op1) | (min((unsigned)(pY[u] - pH[u]), op1) << W) |
               (min((unsigned)(pM[u] - pH[u]), 1u) << (2 * W));
    };
    // the words of chunk cc at tbw; each chunk's CB 16-byte words per lane are 64 lanes apart
    auto store_words = [&](const uint32_t* wds) {
#pragma unroll
        for (int k = 0; k < CB; k++)
            tbw[k * 64] = make_uint4(wds[4 * k], wds[4 * k + 1], wds[4 * k + 2], wds[4 * k + 3]);
        tbw += CB * 64;
    };

    for (int c = 0; c < nch; c++) {
        const int row0 = __builtin_amdgcn_readfirstlane(c * FROWS);
        if (DBG && c == 1) {
            stamp0 = __builtin_amdgcn_s_memrealtime();
            clk0 = __builtin_amdgcn_s_memtime();
        }
        if (DBG && c == nch / 2) stamp1 = __builtin_amdgcn_s_memrealtime();
        // output ring slots row0 .. row0+FROWS (the tail write included) must be free
        wait_ge(&pc.cons(w + 1), RING, outfree, row0 + FROWS + 1);
        wait_ge(&cnt[CI_PRODQ], 0, qavail, row0 + FROWS);
        QPack<QT> q;
        q.load(qcol + ((unsigned)row0 & qmask));
        uint32_t acc[4 * CB];
#pragma unroll
        for (int k = 0; k < 4 * CB; k++) acc[k] = 0;
#pragma unroll
        for (int sc = 0; sc < FROWS / 4; sc++) {
            const int r0 = __builtin_amdgcn_readfirstlane(row0 + 4 * sc);  // rows r0+1 .. r0+4 (edges in e01/e23)
            const int eh[4] = {e01.x, e01.z, e23.x, e23.z};  // H'(i-1, edge)
            const int ev[4] = {e01.y, e01.w, e23.y, e23.w};  // V~(i, edge)
            int4 n01, n23;                    // the next sub-chunk's edges
            int sM[4], sX[4], sY[4], sH[4], oH[4], oV[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int uu = 4 * sc + u;       // row within the chunk; row i = row0 + uu + 1
                int M, X, H, Vt, Ycn;
                if (TB && !FULL) {
                    // the code of row u of the previous sub-chunk (of the previous chunk when sc == 0)
                    constexpr int QB = (int)sizeof(QT);
                    const int pu = (4 * ((sc + 3) & 3) + u) * CB;
                    uint32_t& dstw = sc == 0 ? accP[pu >> 2] : acc[pu >> 2];
                    const uint32_t qw = q.w[(uu * QB) >> 2];
                    const unsigned sh = (unsigned)(pu * 8 & 31);
                    switch (((uu * QB) & 3) / QB) {
                        case 0: row_asm<W, 0, QB == 2>(Hprev, Yc, eh[u], ev[u], qw, pM[u], pX[u], pY[u], pH[u], op1, o, sh, dstw, M, X, H, Vt, Ycn); break;
                        case 1: row_asm<W, 1, QB == 2>(Hprev, Yc, eh[u], ev[u], qw, pM[u], pX[u], pY[u], pH[u], op1, o, sh, dstw, M, X, H, Vt, Ycn); break;
                        case 2: row_asm<W, 2, QB == 2>(Hprev, Yc, eh[u], ev[u], qw, pM[u], pX[u], pY[u], pH[u], op1, o, sh, dstw, M, X, H, Vt, Ycn); break;
                        default: row_asm<W, 3, QB == 2>(Hprev, Yc, eh[u], ev[u], qw, pM[u], pX[u], pY[u], pH[u], op1, o, sh, dstw, M, X, H, Vt, Ycn); break;
                    }
                } else {
                    M = shr1(eh[u], Hprev) + q.get(uu);
                    Vt = min(wave_scan_min(min(M, Yc)), ev[u]);
                    X = shr1(ev[u], Vt) + o;
                    H = min(min(M, X), Yc);
                    Ycn = min(Yc, H + o);
                    if (TB) {
                        const int pu = (4 * ((sc + 3) & 3) + u) * CB;
                        uint32_t* dstw = sc == 0 ? accP : acc;
                        dstw[pu >> 2] |= code_of(u) << (pu * 8 & 31);
                    }
                }
                if (FULL) {
                    const int i = row0 + uu + 1;
                    if (colok && i <= m) {
                        int* f = p.full + 3 * ((long long)i * (p.n + 1) + jcol);
                        f[0] = M; f[1] = X; f[2] = Yc;
                    }
                }
                if (u == GA_EDGE_U) {
                    // after GA_EDGE_U + 1 rows: check the next sub-chunk's rows and read their edges,
                    // 3 - GA_EDGE_U rows before their use (later = the stripe trails its left
                    // neighbour by fewer rows; row 2 measured best: one row covers the LDS latency)
                    if (r0 + 4 < mpad) {
                        avail = sgpr_u(max(avail, pnext));
                        wait_ge(&pc.prod(w), 0, avail, r0 + 8);
                    }
                    const int4* e4 = reinterpret_cast<const int4*>(rin + ((r0 + 4) & RMASK));
                    n01 = e4[0];
                    n23 = e4[1];
                    pnext = *prod_in;
                }
                sM[u] = M; sX[u] = X; sY[u] = Yc; sH[u] = H;
                oH[u] = Hprev;
                oV[u] = Vt;
                Yc = Ycn;
                Hprev = H;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) { pM[u] = sM[u]; pX[u] = sX[u]; pY[u] = sY[u]; pH[u] = sH[u]; }
            if (TB && sc == 0) {
                // the previous chunk's words are complete
                if (c > 0) store_words(accP);
            }
            // the right edge of these rows goes out; LDS executes one wave's operations in
            // order: the rows land before the counters
            lds_publish(rout_lds + (unsigned)(r0 & RMASK) * 8u, pc_lds, srcmask, v4i{oH[0], oV[0], oH[1], oV[1]},
                        v4i{oH[2], oV[2], oH[3], oV[3]}, (unsigned)(r0 + 3), (unsigned)(r0 + 4));
            e01 = n01;
            e23 = n23;
        }
#pragma unroll
        for (int k = 0; k < 4 * CB; k++) accP[k] = acc[k];
        // checkpoint row (banded traceback): (H', h2') of every column after row row0+16
        if (p.ckpt != nullptr && (row0 + FROWS) % p.ckpt_rows == 0 && row0 + FROWS < m && colok)
            p.ckpt[(long long)((row0 + FROWS) / p.ckpt_rows - 1) * (p.n + 1) + jcol] = make_int2(Hprev, Yc);
    }
    if (TB) {
        // the last sub-chunk's codes, then the last chunk's words
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int pu = (12 + u) * CB;
            accP[pu >> 2] |= code_of(u) << (pu * 8 & 31);
        }
        store_words(accP);
    }
    // H' of the last (padded) row, for the reader's hand-off of row m when m == mpad
    if (lane == srcl) rout[mpad & RMASK].x = Hprev;
    if (lane == 0) __hip_atomic_store(&pc.prod(w + 1), (unsigned)(mpad + 1), RLX, WGS);
    if (DBG && lane == 0) {
        p.dbg[8 * s + 0] = stamp0;
        p.dbg[8 * s + 1] = stamp1;
        p.dbg[8 * s + 2] = __builtin_amdgcn_s_memrealtime();
        p.dbg[8 * s + 3] = __builtin_amdgcn_s_memtime() - clk0;  // shader clocks from chunk 1 to the end
    }
}

// ---------------- blocked compute wave: T columns per lane ----------------
// Stripe s covers columns 64*T*s + 1 .. 64*T*(s+1); lane l owns the T consecutive columns
// 64*T*s + l*T + 1 .. + T.  One row (the same recurrence as the T == 1 loop above):
//   M' = H'(i-1, j-1) + sub'           (column 0 of a lane: the left lane's last column, DPP)
//   U  = min(M', Y')                    per column
//   P  = in-register prefix-min of U over the lane's T columns
//   S  = ONE wave scan of the lanes' totals P[T-1] (six DPP steps for 64*T cells)
//   C  = S of the lane to the left (lane 0: the stripe's left-edge V~), V~ = min(C, P)
//   X' = V~(j-1) + o,  H' = min(U, X'),  h2' = min(Y', H' + o)
// so the scan, the edge traffic and the wave-uniform control are paid once per 64*T cells.
// The stripe's right edge is lane 63's last column; only the stripe holding column n may be
// partial, and its compute wave writes the cost H'(m, n) itself.  Traceback words keep the
// 64-column layout of ga_device.h: column (l, k) is lane (l*T + k) % 64 of 64-column stripe
// T*s + (l*T) / 64, so a lane's T words are one contiguous 16*T-byte run.
template <int CB, typename QT, bool TB, int T, bool DBG>
__device__ void fill_blocked(FillArgs& p, unsigned* cnt, int2* ring, QT* qring, uint4* tbstage, int w, int g, int lane) {
    __builtin_amdgcn_s_setprio(2);
    unsigned* abort_sh = cnt + CI_ABORT;
    auto prod = [&](int k) -> unsigned* { return k == 0 ? cnt + CI_PROD0 : cnt + 2 * k - 1; };
    auto cons = [&](int k) -> unsigned* { return cnt + 2 * k; };
    const int m = p.m, o = p.o, n = p.n;
    const int nch = (m + FROWS - 1) / FROWS;
    const int mpad = nch * FROWS;
    const int QR = p.qrows;
    const unsigned qmask = (unsigned)QR - 1u;
    const int s = g * p.nwc + w;
    const int j0 = s * 64 * T;
    const int jl = j0 + lane * T;  // this lane: columns jl+1 .. jl+T
    const QT* qcol[T];
    int Hprev[T], Yc[T];  // H'(i-1, j), h2'(i-1, j)
#pragma unroll
    for (int k = 0; k < T; k++) {
        const int jc = jl + k + 1;
        const bool ok = jc <= n;
        qcol[k] = qring + (ok ? p.b[jc - 1] : 0) * QR;
        const int2 t = p.top[ok ? jc : n];
        Hprev[k] = t.x;
        Yc[k] = t.y;
    }
    // the stripe holding column n (the last one) reports H'(m, n) from lane ke_l, column ke_k
    const bool has_n = j0 < n && n <= j0 + 64 * T;
    const int ke_l = (n - 1 - j0) / T, ke_k = (n - 1 - j0) % T;
    int Hm[T];
#pragma unroll
    for (int k = 0; k < T; k++) Hm[k] = 0;
    const unsigned op1 = (unsigned)o + 1u;
    const int2* rin = ring + w * RING;
    int2* rout = ring + (w + 1) * RING;
    // traceback words: this wave's T 64-column stripes T*s .. T*s+T-1; lane = column within a stripe
    uint4* tbg = TB ? reinterpret_cast<uint4*>(p.tb) + ((long long)(T * s) * p.TC) * 64 + lane : nullptr;
    unsigned avail = 0, outfree = 0, qavail = 0;
    const unsigned pc_lds = lds_addr(cons(w));  // {cons[w], prod[w + 1]}
    const unsigned rout_lds = lds_addr(rout);
    const unsigned long long edgemask = 1ull << 63;
    bool aborted = false;
    constexpr bool dbg = DBG;
    unsigned long long wcyc[3] = {0, 0, 0}, nsleep = 0, clk0 = 0, stamp0 = 0, stamp1 = 0;
    // wait (wave-uniform) until *ctr + add >= target; kind: 0 edges in, 1 ring space out, 2 profile
    auto wait_ge = [&](unsigned* ctr, unsigned add, unsigned& cached, int target, int kind) {
        unsigned spins = 0;
        cached = sgpr_u(cached);
        unsigned long long t0 = 0;
        if (dbg && (int)cached < target) t0 = __builtin_amdgcn_s_memtime();
        while ((int)cached < target && !aborted) {
            cached = lds_ldu(ctr) + add;
            if ((int)cached >= target) break;
            if (!spin_ok_lds(spins, p.spin_limit, abort_sh)) aborted = true;
        }
        if (dbg && t0) {
            wcyc[kind] += __builtin_amdgcn_s_memtime() - t0;
            nsleep += spins;
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    };
    wait_ge(prod(w), 0, avail, 4, 0);
    int4 e01 = reinterpret_cast<const int4*>(rin)[0];
    int4 e23 = reinterpret_cast<const int4*>(rin)[1];
    const unsigned* prod_in = prod(w);
    unsigned pnext = *prod_in;
    // the profile is read one chunk ahead (its LDS latency is off the row chain)
    wait_ge(&cnt[CI_PRODQ], 0, qavail, FROWS, 2);
    QPack<QT> q[T];
#pragma unroll
    for (int k = 0; k < T; k++) q[k].load(qcol[k]);

    for (int c = 0; c < nch; c++) {
        const int row0 = __builtin_amdgcn_readfirstlane(c * FROWS);
        if (dbg && c == 1) {
            stamp0 = __builtin_amdgcn_s_memrealtime();
            clk0 = __builtin_amdgcn_s_memtime();
        }
        if (dbg && c == nch / 2) stamp1 = __builtin_amdgcn_s_memrealtime();
        wait_ge(cons(w + 1), RING, outfree, row0 + FROWS + 1, 1);
        wait_ge(&cnt[CI_PRODQ], 0, qavail, row0 + 2 * FROWS, 2);
        QPack<QT> qn[T];
#pragma unroll
        for (int k = 0; k < T; k++) qn[k].load(qcol[k] + ((unsigned)(row0 + FROWS) & qmask));
        // row m inside this chunk (uniform; -1: none / not the stripe holding column n)
        const int um = __builtin_amdgcn_readfirstlane((has_n && m - 1 - row0 < FROWS) ? m - 1 - row0 : -1);
        uint32_t acc[T][4 * CB];
        if (TB) {
#pragma unroll
            for (int k = 0; k < T; k++)
#pragma unroll
                for (int d = 0; d < 4 * CB; d++) acc[k][d] = 0;
        }
#pragma unroll
        for (int sc = 0; sc < FROWS / 4; sc++) {
            const int r0 = __builtin_amdgcn_readfirstlane(row0 + 4 * sc);
            const int eh[4] = {e01.x, e01.z, e23.x, e23.z};  // H'(i-1, edge)
            const int ev[4] = {e01.y, e01.w, e23.y, e23.w};  // V~(i, edge)
            int4 n01, n23;
            int oH[4], oV[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int uu = 4 * sc + u;
                int sub[T];
#pragma unroll
                for (int k = 0; k < T; k++) sub[k] = q[k].get(uu);
                blocked_row<T, TB, CB>(Hprev, Yc, eh[u], ev[u], sub, o, op1, uu, acc, oH[u], oV[u]);
                if (uu == um) {
#pragma unroll
                    for (int k = 0; k < T; k++) Hm[k] = Hprev[k];
                }
                if (u == GA_EDGE_U) {
                    if (r0 + 4 < mpad) {
                        avail = sgpr_u(max(avail, pnext));
                        wait_ge(prod(w), 0, avail, r0 + 8, 0);
                    }
                    const int4* e4 = reinterpret_cast<const int4*>(rin + ((r0 + 4) & RMASK));
                    n01 = e4[0];
                    n23 = e4[1];
                    pnext = *prod_in;
                }
            }
            lds_publish(rout_lds + (unsigned)(r0 & RMASK) * 8u, pc_lds, edgemask, v4i{oH[0], oV[0], oH[1], oV[1]},
                        v4i{oH[2], oV[2], oH[3], oV[3]}, (unsigned)(r0 + 3), (unsigned)(r0 + 4));
            e01 = n01;
            e23 = n23;
        }
        if (TB) {
            // through LDS so that every global store is one whole 1 KiB run of a 64-column stripe
            // (a lane's own T words sit 16*T bytes apart in it: stored directly, each store
            // instruction would write a 1/T-dense pattern and HBM sees ~9x the bytes at T = 4)
            const int sl = (lane * T) >> 6, l0 = (lane * T) & 63;
#pragma unroll
            for (int d = 0; d < CB; d++)
#pragma unroll
                for (int k = 0; k < T; k++)
                    tbstage[(sl * CB + d) * 64 + l0 + k] =
                        make_uint4(acc[k][4 * d], acc[k][4 * d + 1], acc[k][4 * d + 2], acc[k][4 * d + 3]);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);  // one wave's LDS operations execute in order
#pragma unroll
            for (int s2 = 0; s2 < T; s2++)
#pragma unroll
                for (int d = 0; d < CB; d++) tbg[(size_t)s2 * p.TC * 64 + d * 64] = tbstage[(s2 * CB + d) * 64 + lane];
            tbg += CB * 64;
        }
#pragma unroll
        for (int k = 0; k < T; k++) q[k] = qn[k];
        // checkpoint row (banded traceback): (H', h2') of every column after row row0+16
        if (p.ckpt != nullptr && (row0 + FROWS) % p.ckpt_rows == 0 && row0 + FROWS < m) {
            int2* ck = p.ckpt + (long long)((row0 + FROWS) / p.ckpt_rows - 1) * (n + 1);
#pragma unroll
            for (int k = 0; k < T; k++)
                if (jl + k + 1 <= n) ck[jl + k + 1] = make_int2(Hprev[k], Yc[k]);
        }
    }
    if (lane == 63) rout[mpad & RMASK].x = Hprev[T - 1];
    if (lane == 0) __hip_atomic_store(prod(w + 1), (unsigned)(mpad + 1), RLX, WGS);
    if (has_n && lane == ke_l) {
        int v = Hm[0];
#pragma unroll
        for (int k = 1; k < T; k++)
            if (k == ke_k) v = Hm[k];
        p.out_last[0] = v;
    }
    if (dbg && lane == 0) {
        unsigned long long* d = p.dbg + 8 * s;
        d[0] = stamp0;
        d[1] = stamp1;
        d[2] = __builtin_amdgcn_s_memrealtime();
        d[3] = __builtin_amdgcn_s_memtime() - clk0;
        d[4] = wcyc[0];
        d[5] = wcyc[1];
        d[6] = wcyc[2];
        d[7] = nsleep;
    }
}

// ----------------------------------------------------------------------------------
// The anti-diagonal (skewed) score-only fill (dp_array_forward :366-392 without
// traceback words).  One wave owns a 64-column stripe; lane l owns column 64s+l+1 and
// at step t works on row i = t - l + 1, so a step is one anti-diagonal of the stripe
// and the left neighbour's values are one DPP lane shift of the previous step:
//     M' = H'(i-1, j-1) + sub'        (H' the left lane shifted in a step earlier)
//     X' = h1'(i, j-1)                (the left lane's h1' of the previous step)
//     H' = min(M', X', Y'),  h1' = min(X', H' + o),  h2' = min(Y', H' + o)
// Seven VALU per 64 cells and no per-row scan: the dependent chain of a step is
// DPP -> min3 -> add -> min.  Lane 0 takes the stripe's left edge (H', h1') of row t+1
// from the LDS ring (a broadcast read per 4 steps); lane 63 publishes row t-62 of the
// right edge every 4 steps.  sub' of the lane's row comes from the LDS query profile by
// one byte read per step (the ring has a 16-row mirror tail so a lane's 16 reads of a
// chunk never wrap).  Columns past n (the last stripe only) forward their left input,
// so lane 63 always carries column n of the partial stripe: the right edge and the
// cost come out of the same ring as for a full stripe.
constexpr int QMIRROR = 16;
constexpr int DSUB = 8;  // steps per sub-chunk of the anti-diagonal fill (edge read / wait / publish unit)

// lane 63's publication of eight rows (carry + the sub-chunk's first seven): (H', h1') pairs with one
// ds_write2_b32 each (no packing into consecutive registers), then {cons, prod}; exec narrowed as
// in lds_publish
__device__ __forceinline__ void lds_publish8(unsigned ring_addr, unsigned pc_addr, unsigned long long lanemask, int cH,
                                             int cX, const int (&h)[DSUB], const int (&x)[DSUB], unsigned cons,
                                             unsigned prod) {
    unsigned long long saved;
    const v2u cp = {cons, prod};
    asm volatile(
        "s_mov_b64 %0, exec\n\ts_mov_b64 exec, %3\n\t"
        "ds_write2_b32 %1, %4, %5 offset0:0 offset1:1\n\t"
        "ds_write2_b32 %1, %6, %7 offset0:2 offset1:3\n\t"
        "ds_write2_b32 %1, %8, %9 offset0:4 offset1:5\n\t"
        "ds_write2_b32 %1, %10, %11 offset0:6 offset1:7\n\t"
        "ds_write2_b32 %1, %12, %13 offset0:8 offset1:9\n\t"
        "ds_write2_b32 %1, %14, %15 offset0:10 offset1:11\n\t"
        "ds_write2_b32 %1, %16, %17 offset0:12 offset1:13\n\t"
        "ds_write2_b32 %1, %18, %19 offset0:14 offset1:15\n\t"
        "ds_write_b64 %2, %20\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "v"(ring_addr), "v"(pc_addr), "s"(lanemask), "v"(cH), "v"(cX), "v"(h[0]), "v"(x[0]), "v"(h[1]), "v"(x[1]),
          "v"(h[2]), "v"(x[2]), "v"(h[3]), "v"(x[3]), "v"(h[4]), "v"(x[4]), "v"(h[5]), "v"(x[5]), "v"(h[6]),
          "v"(x[6]), "v"(cp)
        : "memory");
}

template <typename QT, int NWC, int TD, bool FULL, bool DBG>
__global__ void __launch_bounds__(64 * (NWC + 1)) fill_diag_kernel(FillArgs p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    unsigned* cnt = reinterpret_cast<unsigned*>(smem);
    int2* ring = reinterpret_cast<int2*>(smem + FILL_CNT_BYTES);
    QT* qring = reinterpret_cast<QT*>(ring + (NWC + 1) * RING);
    auto prod = [&](int k) -> unsigned* { return k == 0 ? cnt + CI_PROD0 : cnt + 2 * k - 1; };
    auto cons = [&](int k) -> unsigned* { return cnt + 2 * k; };
    unsigned* abort_sh = cnt + CI_ABORT;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x == 0) cnt[CI_SLAB] = atomicAdd(p.ticket, 1u);
    __syncthreads();
    const int g = __builtin_amdgcn_readfirstlane((int)cnt[CI_SLAB]);
    const int m = p.m, o = p.o;
    const int nsteps = m + 64 * TD - 1;              // lane 63's last column reaches row m at step m + 64TD - 2
    const int nch = (nsteps + FROWS - 1) / FROWS;
    const unsigned rows_end = (unsigned)(nch * FROWS + 16);  // every row a consumer may ask for
    const int nlive = min(NWC, p.nstripes - g * NWC);
    const int QR = p.qrows;                          // ring rows (power of two) + QMIRROR mirror rows
    const int QS = QR + QMIRROR;                     // per-code stride
    const unsigned qmask = (unsigned)QR - 1u;

    if (w == NWC) {
        // ---------------- IO wave: slab edges HBM <-> LDS rings, query profile ----------------
        const int2* src = g == 0 ? p.left : p.hand + (long long)(g - 1) * (m + 1);
        const unsigned* src_prog = g == 0 ? p.left_prog : nullptr;  // g > 0: the rows themselves (in_sent)
        const unsigned limit = (g == 0 && p.left_prog != nullptr) ? p.halo_spin_limit : p.spin_limit;
        const bool src_sc1 = p.left_prog != nullptr;  // another GPU's edge, landing while the fill runs
        const bool last_slab = g == p.nslabs - 1;
        int2* dst = (last_slab && p.edge_out != nullptr) ? p.edge_out : p.hand + (long long)g * (m + 1);
        int2* rin0 = ring;
        const int2* rout = ring + nlive * RING;
        const int K = p.K;
        const bool in_sent = g > 0, out_sent = !(last_slab && p.edge_out != nullptr);  // as in fill_kernel
        unsigned in_next = 0, out_next = 0, q_next = 0, spins = 0, in_win = 64;
        while (in_next < (unsigned)m || out_next < (unsigned)m || q_next < (unsigned)m) {
            bool moved = false;
            if (q_next < (unsigned)m) {
                // rows the last wave's lane 63 has published (minus its chunk in flight) are free
                const unsigned pl = lds_ld(prod(nlive));
                const unsigned space = (pl > 24u ? pl - 24u : 0u) + (unsigned)QR;
                const unsigned hi = min(min(space, (unsigned)m), q_next + 64);
                if (hi > q_next && (hi - q_next >= 64 || hi == (unsigned)m)) {
                    const unsigned r = q_next + 1 + lane;
                    if (r <= hi) {
                        const int x = p.a[r - 1];
                        const int* sp = p.subp + x * K;
                        const unsigned slot = (r - 1) & qmask;
                        QT* qd = qring + slot;
                        for (int c = 0; c < K; c++) qd[c * QS] = (QT)sp[c];
                        if (slot < (unsigned)QMIRROR)
                            for (int c = 0; c < K; c++) qd[c * QS + QR] = (QT)sp[c];
                    }
                    if (lane == 0) lds_st(&cnt[CI_PRODQ], hi == (unsigned)m ? rows_end : hi);
                    q_next = hi;
                    moved = true;
                }
            }
            if (in_next < (unsigned)m && in_sent) {
                const unsigned cap = min(min(lds_ld(cons(0)) + RING, (unsigned)m), in_next + in_win);
                if (cap > in_next) {
                    const unsigned r = in_next + 1 + lane;
                    const int2 e1 = r <= cap ? unpack64(g_ld64(src + r)) : make_int2(HAND_SENT, 0);
                    const unsigned long long ok = __ballot(e1.x != HAND_SENT);
                    const unsigned k = ~ok ? (unsigned)__builtin_ctzll(~ok) : 64u;
                    in_win = k >= cap - in_next ? 64u : 8u;  // poll window (as in fill_kernel)
                    if (k > 0) {
                        if (lane < (int)k) rin0[(r - 1) & RMASK] = e1;
                        const unsigned hi = in_next + k;
                        if (lane == 0) lds_st(prod(0), hi == (unsigned)m ? rows_end : hi);
                        in_next = hi;
                        moved = true;
                    }
                }
            } else if (in_next < (unsigned)m) {
                const unsigned space = lds_ld(cons(0)) + RING;
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
                    // rows past m are padding (garbage only rows past m read)
                    if (lane == 0) lds_st(prod(0), hi == (unsigned)m ? rows_end : hi);
                    in_next = hi;
                    moved = true;
                }
            }
            if (out_next < (unsigned)m) {
                const unsigned P = lds_ld(prod(nlive));
                const unsigned hi = min(min(P, (unsigned)m), out_next + 64);
                if (hi > out_next && (hi - out_next >= GOUT || hi == (unsigned)m)) {
                    const unsigned r = out_next + 1 + lane;
                    if (r <= hi) {
                        const int2 e = rout[(r - 1) & RMASK];
                        if (out_sent) g_st64(dst + r, e);
                        else s_st64(dst + r, e);  // another GPU's halo
                        // H'(m, n): the cost (a partial last stripe's compute wave writes it)
                        if (last_slab && r == (unsigned)m && p.n % (64 * TD) == 0) p.out_last[0] = e.x;
                    }
                    if (!out_sent) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (lane == 0) __hip_atomic_store(p.edge_prog, hi, RLX, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    if (lane == 0) lds_st(cons(nlive), hi);
                    out_next = hi;
                    moved = true;
                }
            }
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
        if (!out_sent && out_next < (unsigned)m && p.edge_prog != nullptr && lane == 0) s_prog_abort(p.edge_prog);
        return;
    }
    if (w >= nlive) return;

    // ---------------- compute wave w: stripe s (64*TD columns) ----------------
    __builtin_amdgcn_s_setprio(2);
    const int s = g * NWC + w;
    const int j0 = s * 64 * TD;
    const int jl = j0 + lane * TD;                // this lane: columns jl+1 .. jl+TD
    // the stripe holding column n, when it is not whole: its columns past n compute garbage and the
    // lane holding column n reports H'(m, n) itself (column c of the stripe has row m at step m+c-1)
    const bool partial = j0 + 64 * TD > p.n;
    const int cn = p.n - 1 - j0;
    const int tm = partial ? m - 1 + cn : -1;
    int Hm = 0;
    const QT* qcol[TD];
    bool colok[TD];
    // per column: H' of the last two steps (by step parity), the h1' it passes right, h2'
    int Hp[2][TD], Xo[TD], Yc[TD];
#pragma unroll
    for (int k = 0; k < TD; k++) {
        const int jc = jl + k + 1;
        colok[k] = jc <= p.n;
        qcol[k] = qring + (colok[k] ? p.b[jc - 1] : 0) * QS;
        const int2 t = p.top[colok[k] ? jc : p.n];
        Hp[0][k] = Hp[1][k] = t.x;                // H'(0, j) until the column reaches row 1
        Yc[k] = t.y;                              // h2'(0, j)
        Xo[k] = 0;
    }
    int Hd0 = p.top[min(jl, p.n)].x;              // column 0's diagonal: H'(0, jl) for row 1
    int2* rout = ring + (w + 1) * RING;
    const unsigned rout_lds = lds_addr(rout);
    const unsigned pc_lds = lds_addr(cons(w));  // {cons[w], prod[w + 1]}
    const unsigned long long edgemask = 1ull << 63;
    unsigned avail = 0, outfree = 0, qavail = 0;
    bool aborted = false;
    constexpr bool dbg = DBG;  // timestamps (s_memtime shares lgkmcnt with LDS reads: off the hot path)
    unsigned long long wcyc[3] = {0, 0, 0}, nsleep = 0, clk0 = 0, stamp0 = 0, stamp1 = 0;
    auto wait_ge = [&](unsigned* ctr, unsigned add, unsigned& cached, int target, int kind) {
        unsigned spins = 0;
        cached = sgpr_u(cached);
        unsigned long long t0 = 0;
        if (dbg && (int)cached < target) t0 = __builtin_amdgcn_s_memtime();
        while ((int)cached < target && !aborted) {
            cached = lds_ldu(ctr) + add;
            if ((int)cached >= target) break;
            if (!spin_ok_lds(spins, p.spin_limit, abort_sh)) aborted = true;
        }
        if (dbg && t0) {
            wcyc[kind] += __builtin_amdgcn_s_memtime() - t0;
            nsleep += spins;
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    };
    const int2* rin = ring + w * RING;
    const unsigned* prod_in = prod(w);
    // slot (r - 1) & RMASK of a ring holds (H', h1') of row r.  Edges are read one sub-chunk
    // (4 steps) ahead into ping-pong registers, the producer's counter one sub-chunk ahead of its
    // use, the profile one chunk ahead.
    wait_ge(prod(w), 0, avail, DSUB, 0);
    int4 A[DSUB / 2], B[DSUB / 2];  // (H', h1') of two rows each: rows 1..8 (sub-chunk 0) in A
#pragma unroll
    for (int k = 0; k < DSUB / 2; k++) A[k] = reinterpret_cast<const int4*>(rin)[k];
    unsigned pnext = *prod_in;
    int cH = 0, cX = 0;  // lane 63's last column's (H', h1') of the last step of the previous sub-chunk
    // column k of this lane works on row t - (lane*TD + k) + 1 at step t: its 16 profile values of
    // chunk 0 are rows 1-c .. 16-c (never wrap: mirror tail)
    wait_ge(&cnt[CI_PRODQ], 0, qavail, FROWS, 2);
    QPack<QT> sub[TD];
#pragma unroll
    for (int k = 0; k < TD; k++) sub[k].load_unaligned(qcol[k] + (((unsigned)(-(lane * TD + k))) & qmask));

    // one step: the columns right to left, so that column k reads column k-1's values of the
    // previous step (h1') and of the one before (H', the diagonal) before they are replaced
    auto step = [&](int eh, int ex, int u, int t, auto MASKED) {
        constexpr bool MK = decltype(MASKED)::value;
        const int pp = u & 1;  // t and u have the same parity (t0 is a multiple of 16)
        const int HL = __builtin_amdgcn_update_dpp(eh, Hp[pp ^ 1][TD - 1], 0x138, 0xf, 0xf, false);  // lane 0: edge
        const int XL0 = __builtin_amdgcn_update_dpp(ex, Xo[TD - 1], 0x138, 0xf, 0xf, false);
#pragma unroll
        for (int k = TD - 1; k >= 0; k--) {
            const int M = (k == 0 ? Hd0 : Hp[pp][k - 1]) + sub[k].get(u);
            const int XL = k == 0 ? XL0 : Xo[k - 1];
            if (k == 0) Hd0 = HL;
            if (!MK) {
                const int H = min(min(M, XL), Yc[k]);
                const int Ho = H + o;
                Xo[k] = min(XL, Ho);
                Yc[k] = min(Yc[k], Ho);
                Hp[pp][k] = H;
            } else {
                const int i = t - (lane * TD + k) + 1;
                if (!colok[k]) {  // columns past n forward their left input (the FULL debug output)
                    Hp[pp][k] = k == 0 ? HL : Hp[pp ^ 1][k - 1];
                    Xo[k] = XL;
                } else if (i >= 1) {
                    const int H = min(min(M, XL), Yc[k]);
                    const int Ho = H + o;
                    if (FULL && i <= m) {
                        int* f = p.full + 3 * ((long long)i * (p.n + 1) + jl + k + 1);
                        f[0] = M; f[1] = XL; f[2] = Yc[k];
                    }
                    Xo[k] = min(XL, Ho);
                    Yc[k] = min(Yc[k], Ho);
                    Hp[pp][k] = H;
                }
            }
        }
    };

    for (int c = 0; c < nch; c++) {
        const int t0 = __builtin_amdgcn_readfirstlane(c * FROWS);
        if (dbg && c == 1) {
            stamp0 = __builtin_amdgcn_s_memrealtime();
            clk0 = __builtin_amdgcn_s_memtime();
        }
        if (dbg && c == nch / 2) stamp1 = __builtin_amdgcn_s_memrealtime();
        // ring slots of the rows this chunk publishes (t0-64TD+1 .. t0-64TD+16) must be free
        wait_ge(cons(w + 1), RING, outfree, t0 - 64 * TD + 17, 1);
        // the next chunk's profile values (rows up to t0+32 for lane 0)
        wait_ge(&cnt[CI_PRODQ], 0, qavail, t0 + 2 * FROWS, 2);
        QPack<QT> subn[TD];
#pragma unroll
        for (int k = 0; k < TD; k++)
            subn[k].load_unaligned(qcol[k] + (((unsigned)(t0 + FROWS - (lane * TD + k))) & qmask));
        auto sub_chunks = [&](auto MASKED) {
#pragma unroll
            for (int sc = 0; sc < FROWS / DSUB; sc++) {
                const int r0 = __builtin_amdgcn_readfirstlane(t0 + DSUB * sc);  // steps r0 .. r0+7: lane 0 rows r0+1 .. r0+8
                // this sub-chunk's edges (read a sub-chunk ago) and the next one's (FROWS / DSUB is even)
                int4(&C)[DSUB / 2] = (sc & 1) ? B : A;
                int4(&N)[DSUB / 2] = (sc & 1) ? A : B;
                int eh[DSUB], ex[DSUB];
#pragma unroll
                for (int k = 0; k < DSUB / 2; k++) {
                    eh[2 * k] = C[k].x; ex[2 * k] = C[k].y; eh[2 * k + 1] = C[k].z; ex[2 * k + 1] = C[k].w;
                }
                // left edges one sub-chunk ahead: rows r0+9 .. r0+16 (slots r0+8 .. r0+15)
                wait_ge(prod(w), 0, avail, r0 + 2 * DSUB, 0);
                {
                    const int4* e4 = reinterpret_cast<const int4*>(rin + ((r0 + DSUB) & RMASK));
#pragma unroll
                    for (int k = 0; k < DSUB / 2; k++) N[k] = e4[k];
                    pnext = *prod_in;
                }
                int oH[DSUB], oX[DSUB];
                auto steps = [&](auto CAP) {
                    if constexpr (TD == 1 && !decltype(MASKED)::value && !decltype(CAP)::value) {
                        // one column per lane, no masks: two hand-scheduled 4-step blocks (ga_row.h
                        // diag4_asm); the state moves in and out of the parity-buffered form
                        constexpr int QB = (int)sizeof(QT);
                        int H = Hp[1][0], X = Xo[0], Y = Yc[0];
#pragma unroll
                        for (int hb = 0; hb < DSUB / 4; hb++) {
                            const int u0 = DSUB * sc + 4 * hb;
                            int o4H[4], o4X[4];
                            diag4_asm<QB == 2>(eh[4 * hb], eh[4 * hb + 1], eh[4 * hb + 2], eh[4 * hb + 3], ex[4 * hb],
                                               ex[4 * hb + 1], ex[4 * hb + 2], ex[4 * hb + 3], Hd0, H, X, Y,
                                               sub[0].w[(u0 * QB) >> 2], sub[0].w[((u0 + 2) * QB) >> 2], o, o4H, o4X);
                            Hd0 = eh[4 * hb + 3];
#pragma unroll
                            for (int u = 0; u < 4; u++) {
                                oH[4 * hb + u] = o4H[u];
                                oX[4 * hb + u] = o4X[u];
                            }
                        }
                        Hp[0][0] = oH[DSUB - 2];
                        Hp[1][0] = oH[DSUB - 1];
                        Xo[0] = X;
                        Yc[0] = Y;
                        return;
                    }
#pragma unroll
                    for (int u = 0; u < DSUB; u++) {
                        step(eh[u], ex[u], DSUB * sc + u, r0 + u, MASKED);
                        oH[u] = Hp[u & 1][TD - 1];
                        oX[u] = Xo[TD - 1];
                        if (decltype(CAP)::value && tm == r0 + u) {  // once per stripe
#pragma unroll
                            for (int k = 0; k < TD; k++)
                                if (cn % TD == k) Hm = Hp[u & 1][k];
                        }
                    }
                };
                if ((unsigned)(tm - r0) < (unsigned)DSUB) steps(std::true_type{});
                else steps(std::false_type{});
                // the counter read before the block has landed: no wait on the LDS here, nor at the
                // next sub-chunk's check (used after the publish, whose LDS operations the compiler
                // does not count, it would wait for every LDS operation in flight)
                asm volatile("" : "+v"(pnext));  // keeps the counter's use (and its wait) after the block
                avail = sgpr_u(max(avail, pnext));
                // lane 63's last column has rows r0-64TD+2 .. r0-64TD+9; it publishes the 8-slot-aligned
                // group r0-64TD+1 .. r0-64TD+8 (the first from the previous sub-chunk) so a group never
                // straddles the ring's end; rows < 1 land in slots nobody reads before their real rows
                // overwrite them
                const int pr = r0 - 64 * TD + 1;
                lds_publish8(rout_lds + (unsigned)((pr - 1) & RMASK) * 8u, pc_lds, edgemask, cH, cX, oH, oX,
                             (unsigned)(r0 + DSUB), (unsigned)max(pr + DSUB - 1, 0));
                cH = oH[DSUB - 1];
                cX = oX[DSUB - 1];
            }
        };
        if (FULL || t0 < 64 * TD) sub_chunks(std::true_type{});
        else sub_chunks(std::false_type{});
#pragma unroll
        for (int k = 0; k < TD; k++) sub[k] = subn[k];
    }
    // the last row lane 63's last column computed (row nch*16 - 64TD + 1), then everything (rows
    // past m are padding)
    if (lane == 63) rout[(nch * FROWS - 64 * TD) & RMASK] = make_int2(cH, cX);
    if (lane == 0) __hip_atomic_store(prod(w + 1), rows_end, RLX, WGS);
    if (partial && lane == cn / TD) p.out_last[0] = Hm;
    if (dbg && lane == 0) {
        unsigned long long* d = p.dbg + 8 * s;
        d[0] = stamp0;
        d[1] = stamp1;
        d[2] = __builtin_amdgcn_s_memrealtime();
        d[3] = __builtin_amdgcn_s_memtime() - clk0;
        d[4] = wcyc[0];
        d[5] = wcyc[1];
        d[6] = wcyc[2];
        d[7] = nsleep;
    }
}

// ----------------------------------------------------------------------------------
// Traceback walk: ga_walk.h.  The traceback words of a caller-supplied cell array (dp_array_backward shim):

// dp_array_backward over a caller-supplied dp_array (the reference walks the CALLER's cells,
// globaligner.py:425-514, whatever filled them): the traceback word of every interior cell from its
// given (M, X, Y), in the fill's layout (tb_code above).  The word only needs the differences to
// the cell's minimum, so any int32 triple is encoded exactly (saturated at o + 1 as the fill does).
__global__ void __launch_bounds__(256) tb_from_cells_kernel(const int* __restrict__ cells, int m, int n, int o, int CB,
                                                            int TC, uint8_t* __restrict__ tb) {
    const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
    if (k >= (long long)m * n) return;
    const int i = (int)(k / n) + 1, j = (int)(k % n) + 1;
    const int* v = cells + 3 * ((long long)i * (n + 1) + j);
    const long long M = v[0], X = v[1], Y = v[2];
    const long long H = min(min(M, X), Y), op1 = (long long)o + 1;
    const int W = (8 * CB - 1) / 2;
    const unsigned code = (unsigned)min(X - H, op1) | ((unsigned)min(Y - H, op1) << W) | ((M != H ? 1u : 0u) << (2 * W));
    const int s = (j - 1) >> 6, l = (j - 1) & 63, t = i - 1, spc = 16 / CB;
    uint8_t* p = tb + (((long long)s * TC + t / spc) * 64 + l) * 16 + (t % spc) * CB;
    for (int q = 0; q < CB; q++) p[q] = (uint8_t)(code >> (8 * q));
}

// ----------------------------------------------------------------------------------
// host-side launchers (called from ga_host.cpp)
int boundary_scratch_ints(int m, int n) { return (m + BSEG - 1) / BSEG + (n + BSEG - 1) / BSEG + 2; }

void launch_boundary(hipStream_t s, const uint8_t* a, int m, const uint8_t* b, int n, const int* gh, const int* gv,
                     int o, int big, int* GVp, int* GHp, int2* top, int2* left, int* bnd_row, int* bnd_col, int* meta,
                     bool custom, int* scratch) {
    if (custom) {
        custom_boundary_kernel<<<1, 1024, 0, s>>>(a, m, b, n, gh, gv, o, GVp, GHp, top, left, bnd_row, bnd_col, meta);
        return;
    }
    // small problems: one workgroup does it all (its threads' serial segments read strided codes: C5's 40k codes took
    // 55 us that way against ~15 for the spread kernels below, round 6)
    if ((long long)m + n < 4 * 1024) {
        boundary_kernel<<<1, 1024, 0, s>>>(a, m, b, n, gh, gv, o, big, GVp, GHp, top, left, bnd_row, bnd_col, meta);
        return;
    }
    const int nba = (m + BSEG - 1) / BSEG, nbb = (n + BSEG - 1) / BSEG;
    bnd_sums_kernel<<<nba + nbb, 256, 0, s>>>(a, m, b, n, gh, gv, nba, scratch);
    bnd_scan_kernel<<<1, 1024, 0, s>>>(scratch, nba, nbb);
    bnd_apply_kernel<<<nba + nbb, 256, 0, s>>>(a, m, b, n, gh, gv, nba, scratch, GVp, GHp);
    bnd_edges_kernel<<<(std::max(m, n) + 256) / 256, 256, 0, s>>>(m, n, o, big, GVp, GHp, top, left, bnd_row, bnd_col,
                                                                  meta);
}

size_t fill_lds_bytes(int nwc, int qbytes, int K, int qrows, int tb_stage_bytes_per_wave) {
    return align16((size_t)FILL_CNT_BYTES + (size_t)(nwc + 1) * RING * sizeof(int2) + (size_t)K * qrows * qbytes) +
           (size_t)nwc * tb_stage_bytes_per_wave;
}

template <int CB, typename QT, bool TB, bool FULL, int NWC, int T, bool DBG = false>
static void launch_one(hipStream_t s, const FillArgs& p) {
    // timestamped variants for the diagnostics tools (1-byte words, int8 profiles only)
    if constexpr (!DBG && CB == 1 && std::is_same<QT, int8_t>::value && !FULL)
        if (p.dbg != nullptr) return launch_one<CB, QT, TB, FULL, NWC, T, true>(s, p);
    // the LDS floor sets how many workgroups share a CU (GA_FILL_LDS_FLOOR overrides it, for tuning)
    const size_t floor_b = p.lds_floor >= 0 ? (size_t)p.lds_floor : (size_t)FILL_LDS_MIN;
    const size_t lds = std::max<size_t>(
        fill_lds_bytes(NWC, (int)sizeof(QT), p.K, p.qrows, TB ? TbStage<CB, T>::UINT4S * 16 : 0), floor_b);
    auto* fn = fill_kernel<CB, QT, TB, FULL, NWC, T, DBG>;
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fn<<<dim3(p.nslabs), dim3(64 * (NWC + 1)), lds, s>>>(p);
}

template <typename QT, int NWC, int T>
static void launch_fill_t(hipStream_t s, const FillArgs& p, int CB, bool tb, bool full) {
    if constexpr (T == 8 && sizeof(QT) == 2) return;  // register budget: the host never asks for these
    else if (!tb) return launch_one<1, QT, false, false, NWC, T>(s, p);
    if constexpr (T > 2) return;  // traceback words: T <= 2 (register budget)
    else {
    if constexpr (T == 1) {
        if (full) {
            if (CB == 1) launch_one<1, QT, true, true, NWC, 1>(s, p);
            else if (CB == 2) launch_one<2, QT, true, true, NWC, 1>(s, p);
            else launch_one<4, QT, true, true, NWC, 1>(s, p);
            return;
        }
    }
    if (CB == 1) launch_one<1, QT, true, false, NWC, T>(s, p);
    else if (CB == 2) launch_one<2, QT, true, false, NWC, T>(s, p);
    else launch_one<4, QT, true, false, NWC, T>(s, p);
    }
}

template <int T>
static void launch_fill_T(hipStream_t s, const FillArgs& p, int CB, int qbytes, bool tb, bool full) {
    if (p.nwc == 4) {
        if (qbytes == 1) launch_fill_t<int8_t, 4, T>(s, p, CB, tb, full);
        else launch_fill_t<int16_t, 4, T>(s, p, CB, tb, full);
    } else {
        if (qbytes == 1) launch_fill_t<int8_t, 8, T>(s, p, CB, tb, full);
        else launch_fill_t<int16_t, 8, T>(s, p, CB, tb, full);
    }
}

void launch_fill(hipStream_t s, const FillArgs& p, int CB, int qbytes, bool tb, bool full) {
    if (p.cols_per_lane == 8) launch_fill_T<8>(s, p, CB, qbytes, tb, full);
    else if (p.cols_per_lane == 4) launch_fill_T<4>(s, p, CB, qbytes, tb, full);
    else if (p.cols_per_lane == 2) launch_fill_T<2>(s, p, CB, qbytes, tb, full);
    else launch_fill_T<1>(s, p, CB, qbytes, tb, full);
}

size_t fill_diag_lds_bytes(int nwc, int qbytes, int K, int qrows) {
    return (size_t)FILL_CNT_BYTES + (size_t)(nwc + 1) * RING * sizeof(int2) + (size_t)K * (qrows + QMIRROR) * qbytes;
}

template <typename QT, int NWC, int TD, bool FULL, bool DBG = false>
static void launch_diag_one(hipStream_t s, const FillArgs& p) {
    if (!DBG && p.dbg != nullptr) return launch_diag_one<QT, NWC, TD, FULL, true>(s, p);
    const size_t floor_b = p.lds_floor >= 0 ? (size_t)p.lds_floor : (size_t)FILL_LDS_MIN;
    const size_t lds = std::max<size_t>(fill_diag_lds_bytes(NWC, (int)sizeof(QT), p.K, p.qrows), floor_b);
    auto* fn = fill_diag_kernel<QT, NWC, TD, FULL, DBG>;
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fn<<<dim3(p.nslabs), dim3(64 * (NWC + 1)), lds, s>>>(p);
}

template <int TD>
static void launch_diag_td(hipStream_t s, const FillArgs& p, int qbytes) {
    if (qbytes == 2) {
        if constexpr (TD <= 2) {  // the host caps int16 profiles at TD = 2 (TD = 4 spills)
            if (p.nwc == 4) launch_diag_one<int16_t, 4, TD, false>(s, p);
            else launch_diag_one<int16_t, 8, TD, false>(s, p);
        }
        return;
    }
    if (p.nwc == 4) launch_diag_one<int8_t, 4, TD, false>(s, p);
    else launch_diag_one<int8_t, 8, TD, false>(s, p);
}

void launch_fill_diag(hipStream_t s, const FillArgs& p, int qbytes, bool full) {
    // debug FULL output: 4 compute waves, int8 profiles (the host allows no other)
    if (full) {
        if (p.cols_per_lane == 1) return launch_diag_one<int8_t, 4, 1, true>(s, p);
        return launch_diag_one<int8_t, 4, 2, true>(s, p);
    }
    if (p.cols_per_lane == 4) launch_diag_td<4>(s, p, qbytes);
    else if (p.cols_per_lane == 2) launch_diag_td<2>(s, p, qbytes);
    else launch_diag_td<1>(s, p, qbytes);
}

void launch_tb_from_cells(hipStream_t s, const int* cells, int m, int n, int o, int CB, int TC, uint8_t* tb) {
    const long long cells_in = (long long)m * n;
    hipLaunchKernelGGL(tb_from_cells_kernel, dim3((unsigned)((cells_in + 255) / 256)), dim3(256), 0, s, cells, m, n, o,
                       CB, TC, tb);
}

void launch_walk(hipStream_t s, const WalkArgs& w) {
    if (w.CB == 1) walk_kernel<1><<<1, 64 * WALK_WAVES, 0, s>>>(w);
    else if (w.CB == 2) walk_kernel<2><<<1, 64 * WALK_WAVES, 0, s>>>(w);
    else walk_kernel<4><<<1, 64 * WALK_WAVES, 0, s>>>(w);
}

void launch_walk_chain(hipStream_t s, const WalkChainArgs& a) {
    const int CB = a.w[0].CB;
    if (CB == 1) walk_chain_kernel<1><<<1, 64 * WALK_WAVES, 0, s>>>(a);
    else if (CB == 2) walk_chain_kernel<2><<<1, 64 * WALK_WAVES, 0, s>>>(a);
    else walk_chain_kernel<4><<<1, 64 * WALK_WAVES, 0, s>>>(a);
}

}  // namespace ga
