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
                const unsigned avail = src_prog ? min(s_ld(src_prog), (unsigned)m) : (unsigned)m;
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
                const unsigned avail = src_prog ? min(s_ld(src_prog), (unsigned)m) : (unsigned)m;
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

constexpr int TT = 64;       // tile edge
constexpr int TB4 = 4;       // tile block edge (tiles cached per axis)
constexpr int TP = TB4 * TT; // torus pitch (256)
constexpr int NSLOT = TB4 * TB4;

__device__ __forceinline__ int slot_of(int ti, int tj) { return (ti & (TB4 - 1)) * TB4 + (tj & (TB4 - 1)); }
__device__ __forceinline__ int torus_of(int i, int j) { return ((i - 1) & (TP - 1)) * TP + ((j - 1) & (TP - 1)); }

// One loader wave decodes tile (ti, tj) into the torus: lane = column; the
// tile's 64 rows of a column are 64/SPC whole 16-byte words of its stripe's
// traceback stream (the general path; one-byte words use load_tile_b1).
template <int CB>
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
    const uint4* base = reinterpret_cast<const uint4*>(w.tb) + ((long long)tj * w.TC + ti * KW) * 64 + lane;
    const int nq = min(KW, w.TC - ti * KW);
    uint4 ch[KW];
#pragma unroll
    for (int k = 0; k < KW; k++) ch[k] = (colok && k < nq) ? base[(long long)k * 64] : make_uint4(0, 0, 0, 0);
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
__device__ void load_tile_b1(const WalkArgs& w, int ti, int tj, uint16_t* torus, uint8_t* sa, const uint16_t* lut,
                             int lane) {
    uint16_t* dst = torus + (ti & (TB4 - 1)) * TT * TP + (tj & (TB4 - 1)) * TT + lane;
    const int i0 = ti * TT + 1;
    const int j = tj * TT + lane + 1;
    sa[lane] = (i0 + lane <= w.m) ? w.a[i0 + lane - 1] : 0xff;
    const bool colok = j <= w.n;
    const unsigned bj = colok ? w.b[j - 1] : 0xfeu;
    const uint4* base = reinterpret_cast<const uint4*>(w.tb) + ((long long)tj * w.TC + ti * 4) * 64 + lane;
    const int nq = w.TC - ti * 4;
    unsigned wv[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint4 c = (colok && k < nq) ? base[(long long)k * 64] : make_uint4(0, 0, 0, 0);
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

__device__ __forceinline__ bool in_block(int cur, int ti, int tj) {
    const int dti = (cur >> 16) - ti, dtj = (cur & 0xffff) - tj;
    return cur >= 0 && dti >= 0 && dti < TB4 && dtj >= 0 && dtj < TB4;
}

// One walk by the whole workgroup (every wave returns from here once its role is done): the body of
// walk_kernel, and of walk_chain_kernel once per alignment.  It initialises all of its LDS state.
template <int CB>
__device__ __forceinline__ void walk_body(const WalkArgs& w, const uint32_t* rng) {
    // the thread index through an opaque copy: in walk_chain_kernel nothing derived from it is hoisted
    // out of the loop over walks (it would stay live in VGPRs across every role's code)
    unsigned tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    __shared__ uint16_t torus[TP * TP];
    __shared__ __attribute__((aligned(16))) uint32_t rngbuf[RB];
    __shared__ uint32_t opsbuf[RB / 16];
    __shared__ uint16_t lut[256];
    __shared__ uint8_t lutF[128];
    __shared__ __attribute__((aligned(16))) uint8_t sa[NLOAD_MAX][TT];
    __shared__ int tag[NSLOT];
    __shared__ int rtag[4];
    __shared__ int cur_tile, walk_done, wD, ops_flushed;
    __shared__ unsigned long long load_ticks;
    __shared__ int load_count;
    const int lane = tid & 63;
    const int wave = sgpr(tid >> 6);
    const int m = w.m, n = w.n, o = w.o;
    if (tid == 0) { load_ticks = 0; load_count = 0; }
    if (tid < NSLOT) tag[tid] = -1;
    if (tid < 4) rtag[tid] = -1;
    // a slab walk starts at dispatch D0: the rings start at its block
    if (tid == 0) { cur_tile = -1; walk_done = 0; wD = w.D0; ops_flushed = w.D0 >> 9; }
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
        for (;;) {
            const int d = sgpr(__hip_atomic_load(&wD, __ATOMIC_ACQUIRE, WGS));
            const int done = sgpr(__hip_atomic_load(&walk_done, __ATOMIC_ACQUIRE, WGS));
            bool moved = false;
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
                    if (lane == 0) __hip_atomic_store(&tag[sl], -1, __ATOMIC_SEQ_CST, WGS);
                    if (!in_block(sgpr(__hip_atomic_load(&cur_tile, __ATOMIC_SEQ_CST, WGS)), tti, ttj)) continue;
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    if (CB == 1) load_tile_b1(w, tti, ttj, torus, sa[li], lut, lane);
                    else load_tile<CB>(w, tti, ttj, torus, sa[li], lut, lutF, lane);
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
        auto tabs = [&](int d) { return *reinterpret_cast<const uint4*>(rngbuf + (d & (RB - 1))); };

        if ((D & 511) == 0) {
            block_start(D);
            rng_ready(D);
        }
        verify(i, j);
        int wnext = window(i, j);    // anchored at the walk's current cell
        int wcw = widen(wnext);      // the next group's window, widened (off the next group's chain)
        uint4 tnext = tabs(D);
        unsigned rel = 0;            // offset of the current cell from wnext's anchor (di*8 + dj)
        unsigned L8 = 8u * L;        // bit offset of the entering level's field in a window cell
        unsigned ops = 0;

        // One group of 4 steps: swap in the prefetched window and entries, prefetch the next ones.
        // CHECK: stop at the matrix edge; returns the steps taken when the walk ended, else 0.
        auto group = [&](auto check_tag, int gd) -> int {  // gd: dispatch of the group's first step
            constexpr bool CHECK = decltype(check_tag)::value;
            const int wcur = wcw;
            const uint4 tc = tnext;
            wnext = window(i, j);
            tnext = tabs(gd + 4);
            __builtin_amdgcn_sched_barrier(0);  // issue the prefetch here, not where the next group needs it
            const unsigned t[4] = {(unsigned)sgpr((int)tc.x), (unsigned)sgpr((int)tc.y), (unsigned)sgpr((int)tc.z),
                                   (unsigned)sgpr((int)tc.w)};
            // ix: the readlane index.  Only its low 6 bits count, so the moves go in unmasked; its low
            // byte is rel + the group's moves (diag 9, left 1, up 8: at most 4 rows and 4 columns).
            // A: the group's levels times 8, base 4.  (The walker is issue-bound: ~7 scalar ops a step.)
            unsigned ix = rel, A = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const unsigned v = (unsigned)__builtin_amdgcn_readlane(wcur, (int)ix);
                // widen the next group's window (read at this group's start) while the last step's
                // scalar chain runs
                if (k == 3) wcw = widen(wnext);
                // the chosen level comes out as the next field's bit offset (lvl * 8): two dependent
                // scalar ops fewer per step than extracting lvl and scaling it
                L8 = (t[k] >> ((v >> L8) & 31u)) & 0x18u;
                A = A * 4u + L8;
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
            const unsigned mv = (ix - rel) & 0xffu;
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
                reason = i == 0 ? iend : jend;
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

template <int CB>
__global__ void __launch_bounds__(64 * WALK_WAVES) walk_kernel(WalkArgs w) {
    walk_body<CB>(w, w.rng);
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
        walk_body<CB>(w, a.tab + G);
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
    if ((long long)m + n < 64 * 1024) {  // small problems: one workgroup does it all
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
    static const long floor_env = [] {
        const char* e = getenv("GA_FILL_LDS_FLOOR");
        return e ? atol(e) : -1L;
    }();
    const size_t floor_b = floor_env >= 0 ? (size_t)floor_env : (size_t)FILL_LDS_MIN;
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
    static const long floor_env = [] {
        const char* e = getenv("GA_FILL_LDS_FLOOR");
        return e ? atol(e) : -1L;
    }();
    const size_t floor_b = floor_env >= 0 ? (size_t)floor_env : (size_t)FILL_LDS_MIN;
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
