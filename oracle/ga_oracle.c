/*
 * ga_oracle.c -- CPU restatement of globalign's DP hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle for the MI355X product path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (globalign_amd/) never links or calls it.
 *
 * It restates, in plain C with int64 arithmetic (the reference uses unbounded
 * Python ints), the functions of /root/reference/src/globalign/globaligner.py:
 *   make_dp_array            :756-821   -> gao_boundary()
 *   get_next_best_costs      :317-363   -> gao_cell()
 *   dp_array_forward         :366-392   -> gao_fill_full(), gao_fill_sets(), gao_fill_score()
 *   dp_array_backward        :395-593   -> gao_traceback()
 *   cost_ranks_dispatcher    :595-685   -> dispatch()
 *   take_match/.../gap_2     :688-753   -> emit()
 * and CPython's random.choice -> Random._randbelow_with_getrandbits ->
 * getrandbits -> genrand_uint32 (Modules/_randommodule.c, MT19937), which the
 * dispatcher calls 18 times per traceback step.
 *
 * Parity pinning: tests/test_oracle.py checks every function here against the
 * golden fixtures the tests/golden JSON files produced by running the reference itself
 * (tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef int64_t i64;

/* ------------------------------------------------------------------ MT19937 */
#define MT_N 624
#define MT_M 397

typedef struct { uint32_t mt[MT_N]; int mti; } mt_t;

static void mt_twist(mt_t* s) {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t* mt = s->mt;
    int kk;
    uint32_t y;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < MT_N - 1; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt[MT_N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    s->mti = 0;
}

static uint32_t mt_next(mt_t* s) {
    if (s->mti >= MT_N) mt_twist(s);
    uint32_t y = s->mt[s->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* random.choice(seq) == seq[_randbelow(len(seq))]; for len 2 and 3, k = 2 bits. */
static int randbelow(mt_t* s, int n) {
    int r;
    do { r = (int)(mt_next(s) >> 30); } while (r >= n);
    return r;
}

/* -------------------------------------------------------------- boundaries */
/* make_dp_array (globaligner.py:756-821).  row0/col0 are (n+1)/(m+1) triples. */
void gao_boundary(const uint8_t* a, i64 m, const uint8_t* b, i64 n, const i64* gh, const i64* gv,
                  i64 o, i64 big, i64* row0, i64* col0) {
    row0[0] = row0[1] = row0[2] = 0;              /* :778 */
    col0[0] = col0[1] = col0[2] = 0;
    for (i64 j = 1; j <= n; j++) {                 /* :780-784, :802-809 */
        row0[3 * j + 0] = big;
        row0[3 * j + 1] = (j == 1 ? o : row0[3 * (j - 1) + 1]) + gh[b[j - 1]];
        row0[3 * j + 2] = big;
    }
    for (i64 i = 1; i <= m; i++) {                 /* :789-793, :812-819 */
        col0[3 * i + 0] = big;
        col0[3 * i + 1] = big;
        col0[3 * i + 2] = (i == 1 ? o : col0[3 * (i - 1) + 2]) + gv[a[i - 1]];
    }
}

static inline i64 min3(i64 x, i64 y, i64 z) { i64 t = x < y ? x : y; return t < z ? t : z; }

/* get_next_best_costs (globaligner.py:317-363), literally: the three minima. */
static inline void gao_cell(const i64* diag, const i64* left, const i64* up, i64 sub, i64 gh_b, i64 gv_a,
                            i64 o, i64* out) {
    out[0] = min3(diag[0], diag[1], diag[2]) + sub;                    /* :331-336, :360 */
    out[1] = min3(left[0] + o, left[1], left[2] + o) + gh_b;           /* :342-347, :361 */
    out[2] = min3(up[0] + o, up[1] + o, up[2]) + gv_a;                 /* :352-357, :362 */
}

/* dp_array_forward (globaligner.py:366-392) over a full (m+1)x(n+1)x3 array whose
 * row 0 and column 0 are already set (any values: the reference test
 * tests/globaligner_test.py:8-33 hand-writes them). */
void gao_fill_full(const uint8_t* a, i64 m, const uint8_t* b, i64 n, const i64* sub, int K,
                   const i64* gh, const i64* gv, i64 o, i64* dp) {
    const i64 W = n + 1;
    for (i64 i = 1; i <= m; i++)
        for (i64 j = 1; j <= n; j++)
            gao_cell(&dp[3 * ((i - 1) * W + j - 1)], &dp[3 * (i * W + j - 1)], &dp[3 * ((i - 1) * W + j)],
                     sub[a[i - 1] * K + b[j - 1]], gh[b[j - 1]], gv[a[i - 1]], o, &dp[3 * (i * W + j)]);
}

/* argmin set (bit k set <=> value k is a minimum) of a triple */
static inline int argmin_set(i64 x, i64 y, i64 z) {
    i64 h = min3(x, y, z);
    return (x == h) | ((y == h) << 1) | ((z == h) << 2);
}

/* The three rank sets the traceback can ask about at a cell (dp_array_backward
 * :490-514): level 0 ranks (M,X,Y); level 1 ranks (M+o,X,Y+o); level 2 ranks
 * (M+o,X+o,Y).  Packed 3 bits each. */
static inline int cell_sets(const i64* v, i64 o) {
    return argmin_set(v[0], v[1], v[2]) | (argmin_set(v[0] + o, v[1], v[2] + o) << 3) |
           (argmin_set(v[0] + o, v[1] + o, v[2]) << 6);
}

/* Same fill, rolling rows, storing only the 9-bit rank sets per interior cell
 * (uint16, row-major m x n).  Returns the final triple. */
void gao_fill_sets(const uint8_t* a, i64 m, const uint8_t* b, i64 n, const i64* sub, int K,
                   const i64* gh, const i64* gv, i64 o, const i64* row0, const i64* col0,
                   uint16_t* sets, i64* last) {
    i64* prev = (i64*)malloc(sizeof(i64) * 3 * (n + 1));
    i64* cur = (i64*)malloc(sizeof(i64) * 3 * (n + 1));
    memcpy(prev, row0, sizeof(i64) * 3 * (n + 1));
    for (i64 i = 1; i <= m; i++) {
        memcpy(cur, &col0[3 * i], sizeof(i64) * 3);
        const int ai = a[i - 1];
        for (i64 j = 1; j <= n; j++) {
            gao_cell(&prev[3 * (j - 1)], &cur[3 * (j - 1)], &prev[3 * j], sub[ai * K + b[j - 1]], gh[b[j - 1]],
                     gv[ai], o, &cur[3 * j]);
            if (sets) sets[(i - 1) * n + (j - 1)] = (uint16_t)cell_sets(&cur[3 * j], o);
        }
        i64* t = prev; prev = cur; cur = t;
    }
    memcpy(last, &prev[3 * n], sizeof(i64) * 3);
    free(prev);
    free(cur);
}

/* ------------------------------------------------------------- traceback */
enum { MV_MATCH = 0, MV_MISMATCH = 1, MV_GAP1 = 2, MV_GAP2 = 3 };

/* cost_ranks_dispatcher (globaligner.py:595-685).  The 54-entry dict literal
 * evaluates 18 random.choice calls (entries :599-671 in order) every call.
 * ranks: the 3 ranks; returns the move. */
static int dispatch(mt_t* rng, const int* ranks, int is_match) {
    static const int sizes[18] = {3, 2, 2, 2, 3, 2, 2, 2, 3, 3, 2, 2, 2, 3, 2, 2, 2, 3};
    int r[18];
    for (int k = 0; k < 18; k++) r[k] = randbelow(rng, sizes[k]);
    const int base = is_match ? 0 : 9;
    const int mm = is_match ? MV_MATCH : MV_MISMATCH;
    const int tri[3] = {mm, MV_GAP1, MV_GAP2};
    const int key = ranks[0] * 9 + ranks[1] * 3 + ranks[2];
    switch (key) {
        case 0: return tri[r[base + 0]];                                   /* (0,0,0) */
        case 1: return MV_GAP2;                                            /* (0,0,1) */
        case 3: return MV_GAP1;                                            /* (0,1,0) */
        case 9: return mm;                                                 /* (1,0,0) */
        case 2: return r[base + 1] ? MV_GAP1 : mm;                         /* (0,0,2) */
        case 6: return r[base + 2] ? MV_GAP2 : mm;                         /* (0,2,0) */
        case 18: return r[base + 3] ? MV_GAP2 : MV_GAP1;                   /* (2,0,0) */
        case 4: return mm;                                                 /* (0,1,1) */
        case 10: return MV_GAP1;                                           /* (1,0,1) */
        case 12: return MV_GAP2;                                           /* (1,1,0) */
        case 8: return mm;                                                 /* (0,2,2) */
        case 20: return MV_GAP1;                                           /* (2,0,2) */
        case 24: return MV_GAP2;                                           /* (2,2,0) */
        case 5: return mm;                                                 /* (0,1,2) */
        case 11: return MV_GAP1;                                           /* (1,0,2) */
        case 15: return MV_GAP2;                                           /* (1,2,0) */
        case 7: return mm;                                                 /* (0,2,1) */
        case 19: return MV_GAP1;                                           /* (2,0,1) */
        case 21: return MV_GAP2;                                           /* (2,1,0) */
        case 13: return tri[r[base + 4]];                                  /* (1,1,1) */
        case 14: return r[base + 5] ? MV_GAP1 : mm;                        /* (1,1,2) */
        case 16: return r[base + 6] ? MV_GAP2 : mm;                        /* (1,2,1) */
        case 22: return r[base + 7] ? MV_GAP2 : MV_GAP1;                   /* (2,1,1) */
        case 17: return mm;                                                /* (1,2,2) */
        case 23: return MV_GAP1;                                           /* (2,1,2) */
        case 25: return MV_GAP2;                                           /* (2,2,1) */
        default: return tri[r[base + 8]];                                  /* (2,2,2) */
    }
}

/* [sorted(c).index(x) for x in c] (globaligner.py:435, :514) */
static void ranks_of(const i64* c, int* rk) {
    for (int k = 0; k < 3; k++) {
        int below = 0;
        for (int q = 0; q < 3; q++) below += c[q] < c[k];
        rk[k] = below;
    }
}

/* Cell access for the walk.  mode 0: full value array; mode 1: rank sets for
 * interior cells plus boundary triples. */
struct tiles_s;
typedef struct {
    int mode;
    i64 m, n, o;
    const i64* dp;        /* mode 0: (m+1)(n+1)x3 */
    const uint16_t* sets; /* mode 1: m x n */
    const i64* row0;      /* mode 1, 2 */
    const i64* col0;      /* mode 1, 2 */
    struct tiles_s* tiles; /* mode 2: rank sets of one tile at a time, recomputed from checkpoints (gao_align_ckpt) */
} cells_t;

static int tile_set(struct tiles_s* t, i64 ri, i64 rj);

/* Ranks of (values + level offsets).  For interior cells in mode 1 the rank
 * tuple is rebuilt from the argmin set: ties among the minima -> rank 0, the
 * others get distinct non-zero ranks whose order the dispatcher never uses
 * (every key with a unique minimum maps to the same move). */
static void cell_ranks(const cells_t* cs, i64 ri, i64 rj, int level, const i64 add[3], int* rk) {
    if (cs->mode == 0 || ri == 0 || rj == 0) {
        const i64* v;
        if (cs->mode == 0) v = &cs->dp[3 * (ri * (cs->n + 1) + rj)];
        else v = (ri == 0) ? &cs->row0[3 * rj] : &cs->col0[3 * ri];
        i64 c[3] = {v[0] + add[0], v[1] + add[1], v[2] + add[2]};
        ranks_of(c, rk);
        return;
    }
    int set = (cs->mode == 2 ? tile_set(cs->tiles, ri, rj) : cs->sets[(ri - 1) * cs->n + (rj - 1)]) >> (3 * level) & 7;
    /* minima get rank 0, the others distinct ranks starting at the number of
     * minima (what sorted().index yields when the non-minima differ; when they
     * tie the reference key differs but maps to the same move). */
    int nxt = __builtin_popcount(set);
    for (int k = 0; k < 3; k++) rk[k] = (set >> k & 1) ? 0 : nxt++;
}

/* Python index of a length-L sequence; returns -1 on IndexError. */
static inline i64 pyidx(i64 k, i64 L) {
    if (k < 0) k += L;
    return (k < 0 || k >= L) ? -1 : k;
}

/* dp_array_backward (globaligner.py:395-593).
 * chars a_chr/b_chr are the original (upper-cased) sequences; codes a/b index the tables.
 * Output strings are written reversed-then-fixed, cap >= m+n+1.
 * Returns 0 on success, 1 on IndexError (the reference raises IndexError), and
 * the number of dispatcher calls through *ndispatch; mt state is updated in place
 * (625 words, python getstate()[1] layout). */
int gao_traceback(const cells_t* cs, const uint8_t* a, const uint8_t* b, const char* a_chr, const char* b_chr,
                  const i64* sub, int K, const i64* gh, int gap_code, uint32_t* mt_state,
                  char* out_a, char* out_mid, char* out_b, i64* out_len, i64* ndispatch) {
    (void)gap_code;
    const i64 m = cs->m, n = cs->n, o = cs->o;
    mt_t rng;
    memcpy(rng.mt, mt_state, sizeof(uint32_t) * MT_N);
    rng.mti = (int)mt_state[MT_N];
    i64 len = 0, nd = 0;
    int status = 0;
    i64 i = m, j = n;
    int level = 0;
    int first = 1;
    i64 h = 0;
    const i64 max_moves = m + n;  /* dim_1 + dim_2 - 2 (:473) */
    for (;;) {
        i64 si = i - 1, sj = j - 1;
        i64 ri = pyidx(i, m + 1), rj = pyidx(j, n + 1);       /* dp_array[i][j] */
        if (ri < 0 || rj < 0) { status = 1; break; }
        i64 add[3] = {0, 0, 0};
        if (!first) {
            if (level == 0) {                                 /* :490-493 */
                i64 pa = pyidx(si, m);
                if (pa < 0) { status = 1; break; }
                i64 pb = pyidx(sj, n);
                if (pb < 0) { status = 1; break; }
                add[0] = add[1] = add[2] = sub[a[pa] * K + b[pb]];
            } else {
                i64 pb = pyidx(sj, n);                        /* :494-505 */
                if (pb < 0) { status = 1; break; }
                i64 g = gh[b[pb]];
                if (level == 1) { add[0] = o + g; add[1] = g; add[2] = o + g; }
                else { add[0] = o + g; add[1] = o + g; add[2] = g; }
            }
        }
        int rk[3];
        cell_ranks(cs, ri, rj, first ? 0 : level, add, rk);
        i64 pa = pyidx(si, m), pb = pyidx(sj, n);             /* is_match (:436, :515) */
        if (pa < 0 || pb < 0) { status = 1; break; }
        int is_match = a_chr[pa] == b_chr[pb];
        int mv = dispatch(&rng, rk, is_match);
        nd++;
        switch (mv) {                                         /* take_* (:688-753) */
            case MV_MATCH: out_a[len] = a_chr[pa]; out_mid[len] = '|'; out_b[len] = b_chr[pb]; i--; j--; level = 0; break;
            case MV_MISMATCH: out_a[len] = a_chr[pa]; out_mid[len] = '*'; out_b[len] = b_chr[pb]; i--; j--; level = 0; break;
            case MV_GAP1: out_a[len] = '-'; out_mid[len] = ' '; out_b[len] = b_chr[pb]; j--; level = 1; break;
            default: out_a[len] = a_chr[pa]; out_mid[len] = ' '; out_b[len] = '-'; i--; level = 2; break;
        }
        len++;
        if (first) {
            first = 0;
            if (i == 0 && j == 0) break;                      /* :460-470 */
            continue;
        }
        if (i == 0) {                                         /* :542-561 */
            for (i64 jj = j; jj > 0; jj--) {
                out_a[len] = '-'; out_mid[len] = ' '; out_b[len] = b_chr[jj - 1]; len++;
            }
            break;
        } else if (j == 0) {                                  /* :562-581 */
            for (i64 ii = i; ii > 0; ii--) {
                out_a[len] = a_chr[ii - 1]; out_mid[len] = ' '; out_b[len] = '-'; len++;
            }
            break;
        }
        if (++h >= max_moves) break;                          /* loop bound (:475) */
    }
    /* reverse (:584-586) */
    for (i64 p = 0, q = len - 1; p < q; p++, q--) {
        char t;
        t = out_a[p]; out_a[p] = out_a[q]; out_a[q] = t;
        t = out_mid[p]; out_mid[p] = out_mid[q]; out_mid[q] = t;
        t = out_b[p]; out_b[p] = out_b[q]; out_b[q] = t;
    }
    memcpy(mt_state, rng.mt, sizeof(uint32_t) * MT_N);
    mt_state[MT_N] = (uint32_t)rng.mti;
    *out_len = len;
    *ndispatch = nd;
    return status;
}

/* ---------------------------------------------------------- flat wrappers */
/* Convenience entry points with flat arguments (ctypes-friendly). */
int gao_traceback_full(const i64* dp, i64 m, i64 n, i64 o, const uint8_t* a, const uint8_t* b,
                       const char* a_chr, const char* b_chr, const i64* sub, int K, const i64* gh,
                       uint32_t* mt_state, char* out_a, char* out_mid, char* out_b, i64* out_len, i64* nd) {
    cells_t cs = {0, m, n, o, dp, NULL, NULL, NULL, NULL};
    return gao_traceback(&cs, a, b, a_chr, b_chr, sub, K, gh, 0, mt_state, out_a, out_mid, out_b, out_len, nd);
}

int gao_traceback_sets(const uint16_t* sets, const i64* row0, const i64* col0, i64 m, i64 n, i64 o,
                       const uint8_t* a, const uint8_t* b, const char* a_chr, const char* b_chr, const i64* sub,
                       int K, const i64* gh, uint32_t* mt_state, char* out_a, char* out_mid, char* out_b,
                       i64* out_len, i64* nd) {
    cells_t cs = {1, m, n, o, NULL, sets, row0, col0, NULL};
    return gao_traceback(&cs, a, b, a_chr, b_chr, sub, K, gh, 0, mt_state, out_a, out_mid, out_b, out_len, nd);
}

/* Score-only fill (rolling rows), for sizes where no traceback is wanted. */
void gao_fill_score(const uint8_t* a, i64 m, const uint8_t* b, i64 n, const i64* sub, int K, const i64* gh,
                    const i64* gv, i64 o, const i64* row0, const i64* col0, i64* last) {
    gao_fill_sets(a, m, b, n, sub, K, gh, gv, o, row0, col0, NULL, last);
}

/* Right-edge slab fill for the multi-rank decomposition tests: fills columns
 * [1, n] given a left column (m+1 triples, i.e. col0) and a top row, and
 * returns the right-most column (m+1 triples). */
void gao_fill_slab(const uint8_t* a, i64 m, const uint8_t* b, i64 n, const i64* sub, int K, const i64* gh,
                   const i64* gv, i64 o, const i64* row0, const i64* col0, i64* right_col) {
    i64* prev = (i64*)malloc(sizeof(i64) * 3 * (n + 1));
    i64* cur = (i64*)malloc(sizeof(i64) * 3 * (n + 1));
    memcpy(prev, row0, sizeof(i64) * 3 * (n + 1));
    memcpy(&right_col[0], &row0[3 * n], sizeof(i64) * 3);
    for (i64 i = 1; i <= m; i++) {
        memcpy(cur, &col0[3 * i], sizeof(i64) * 3);
        for (i64 j = 1; j <= n; j++)
            gao_cell(&prev[3 * (j - 1)], &cur[3 * (j - 1)], &prev[3 * j], sub[a[i - 1] * K + b[j - 1]],
                     gh[b[j - 1]], gv[a[i - 1]], o, &cur[3 * j]);
        memcpy(&right_col[3 * i], &cur[3 * n], sizeof(i64) * 3);
        i64* t = prev; prev = cur; cur = t;
    }
    free(prev);
    free(cur);
}

/* MT helpers for tests: advance by `choices` calls of random.choice on the
 * dispatcher's size pattern is not needed; expose raw draws instead. */
void gao_mt_draws(uint32_t* mt_state, int nsizes, const int* sizes, int* out) {
    mt_t rng;
    memcpy(rng.mt, mt_state, sizeof(uint32_t) * MT_N);
    rng.mti = (int)mt_state[MT_N];
    for (int k = 0; k < nsizes; k++) out[k] = randbelow(&rng, sizes[k]);
    memcpy(mt_state, rng.mt, sizeof(uint32_t) * MT_N);
    mt_state[MT_N] = (uint32_t)rng.mti;
}

/* Score-only fill on T host threads (test infrastructure: pins the C4 cost).
 * Column slabs, one per thread; row bands of B rows.  Thread k fills band r of its
 * slab once thread k-1 has published band r of its right column (a wavefront
 * over slabs).  Every cell is gao_cell, the literal get_next_best_costs. */
#include <pthread.h>
#include <stdatomic.h>

typedef struct {
    const uint8_t* a; i64 m; const uint8_t* b; i64 n; const i64* sub; int K; const i64* gh; const i64* gv; i64 o;
    const i64* row0; const i64* col0;
    int T; i64 B; i64* edges;         /* [T+1][m+1][3]: edge k = left column of slab k */
    _Atomic i64* done;                /* [T]: rows of slab k's right edge published */
    i64* last;
} par_t;

typedef struct { par_t* p; int k; } par_arg;

static void* par_worker(void* vp) {
    par_arg* pa = (par_arg*)vp;
    par_t* p = pa->p;
    const int k = pa->k;
    const i64 c0 = p->n * k / p->T, c1 = p->n * (k + 1) / p->T, w = c1 - c0;
    i64* prev = (i64*)malloc(sizeof(i64) * 3 * (w + 1));
    i64* cur = (i64*)malloc(sizeof(i64) * 3 * (w + 1));
    memcpy(prev, &p->row0[3 * c0], sizeof(i64) * 3 * (w + 1));
    const i64* left = p->edges + (size_t)k * 3 * (p->m + 1);
    i64* right = p->edges + (size_t)(k + 1) * 3 * (p->m + 1);
    memcpy(&right[0], &p->row0[3 * c1], sizeof(i64) * 3);
    for (i64 r0 = 1; r0 <= p->m; r0 += p->B) {
        const i64 r1 = r0 + p->B - 1 < p->m ? r0 + p->B - 1 : p->m;
        if (k > 0)
            while (atomic_load_explicit(&p->done[k - 1], memory_order_acquire) < r1) sched_yield();
        for (i64 i = r0; i <= r1; i++) {
            memcpy(cur, &left[3 * i], sizeof(i64) * 3);
            const uint8_t ai = p->a[i - 1];
            for (i64 j = 1; j <= w; j++)
                gao_cell(&prev[3 * (j - 1)], &cur[3 * (j - 1)], &prev[3 * j], p->sub[ai * p->K + p->b[c0 + j - 1]],
                         p->gh[p->b[c0 + j - 1]], p->gv[ai], p->o, &cur[3 * j]);
            memcpy(&right[3 * i], &cur[3 * w], sizeof(i64) * 3);
            i64* t = prev; prev = cur; cur = t;
        }
        atomic_store_explicit(&p->done[k], r1, memory_order_release);
    }
    if (k == p->T - 1) memcpy(p->last, &prev[3 * w], sizeof(i64) * 3);
    free(prev);
    free(cur);
    return NULL;
}

void gao_fill_score_parallel(const uint8_t* a, i64 m, const uint8_t* b, i64 n, const i64* sub, int K, const i64* gh,
                             const i64* gv, i64 o, const i64* row0, const i64* col0, int T, i64* last) {
    if (T < 1) T = 1;
    if (T > n) T = (int)n;
    par_t p = {a, m, b, n, sub, K, gh, gv, o, row0, col0, T, 256, NULL, NULL, last};
    p.edges = (i64*)malloc(sizeof(i64) * 3 * (size_t)(m + 1) * (T + 1));
    memcpy(p.edges, col0, sizeof(i64) * 3 * (m + 1));
    p.done = (_Atomic i64*)calloc(T, sizeof(i64));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * T);
    par_arg* args = (par_arg*)malloc(sizeof(par_arg) * T);
    for (int k = 0; k < T; k++) {
        args[k].p = &p;
        args[k].k = k;
        pthread_create(&th[k], NULL, par_worker, &args[k]);
    }
    for (int k = 0; k < T; k++) pthread_join(th[k], NULL);
    free(th);
    free(args);
    free((void*)p.done);
    free(p.edges);
}

/* ------------------------------------------- checkpoint-and-recompute traceback */
/* The same alignment as gao_fill_sets + gao_traceback_sets without m x n rank sets (test infrastructure: pins the
 * C4 full-traceback alignment, 10^12 cells; the reference's own traceback reads the whole
 * dp_array, globaligner.py:395-593).  A forward pass on T threads (the column-slab wavefront above) saves every
 * BH-th row and every CW-th column of triples; the walk then recomputes, one BH x CW tile at a time, the rank sets
 * of the tile it is in, from the tile's top row and left column (gao_cell, the literal get_next_best_costs), and
 * reads them exactly as mode 1 does.  The walk only moves up and left, so each tile is recomputed once. */
typedef struct tiles_s {
    const uint8_t* a; const uint8_t* b; const i64* sub; int K; const i64* gh; const i64* gv; i64 o;
    i64 m, n, BH, CW;
    const i64* row0; const i64* col0;
    const i64* rowck;   /* [m / BH][n + 1][3]: row k*BH, k >= 1 */
    const i64* colck;   /* [n / CW][m + 1][3]: column k*CW, k >= 1 */
    i64 bi, bj;         /* the tile held (-1: none) */
    uint16_t* sets;     /* [BH][CW] */
    i64* prev; i64* cur;
    i64 recomputed;
} tiles_t;

static int tile_set(tiles_t* t, i64 ri, i64 rj) {
    const i64 bi = (ri - 1) / t->BH, bj = (rj - 1) / t->CW;
    if (bi != t->bi || bj != t->bj) {
        const i64 r0 = bi * t->BH, c0 = bj * t->CW;
        const i64 r1 = r0 + t->BH < t->m ? r0 + t->BH : t->m, c1 = c0 + t->CW < t->n ? c0 + t->CW : t->n;
        const i64 w = c1 - c0;
        const i64* top = bi == 0 ? t->row0 : t->rowck + (size_t)(bi - 1) * 3 * (t->n + 1);
        const i64* left = bj == 0 ? t->col0 : t->colck + (size_t)(bj - 1) * 3 * (t->m + 1);
        memcpy(t->prev, &top[3 * c0], sizeof(i64) * 3 * (w + 1));
        for (i64 i = r0 + 1; i <= r1; i++) {
            memcpy(t->cur, &left[3 * i], sizeof(i64) * 3);
            const int ai = t->a[i - 1];
            for (i64 j = 1; j <= w; j++) {
                const int bj1 = t->b[c0 + j - 1];
                gao_cell(&t->prev[3 * (j - 1)], &t->cur[3 * (j - 1)], &t->prev[3 * j], t->sub[ai * t->K + bj1],
                         t->gh[bj1], t->gv[ai], t->o, &t->cur[3 * j]);
                t->sets[(i - r0 - 1) * t->CW + (j - 1)] = (uint16_t)cell_sets(&t->cur[3 * j], t->o);
            }
            i64* x = t->prev; t->prev = t->cur; t->cur = x;
        }
        t->bi = bi;
        t->bj = bj;
        t->recomputed++;
    }
    return t->sets[(ri - 1 - bi * t->BH) * t->CW + (rj - 1 - bj * t->CW)];
}

typedef struct {
    const uint8_t* a; i64 m; const uint8_t* b; i64 n; const i64* sub; int K; const i64* gh; const i64* gv; i64 o;
    const i64* row0; int T; i64 B, BH, CW;
    i64* edges; _Atomic i64* done; i64* rowck; i64* colck; i64* last;
} ckf_t;

typedef struct { ckf_t* p; int k; } ckf_arg;

static void* ckf_worker(void* vp) {
    ckf_arg* pa = (ckf_arg*)vp;
    ckf_t* p = pa->p;
    const int k = pa->k;
    const i64 c0 = p->n * k / p->T, c1 = p->n * (k + 1) / p->T, w = c1 - c0;
    i64* prev = (i64*)malloc(sizeof(i64) * 3 * (w + 1));
    i64* cur = (i64*)malloc(sizeof(i64) * 3 * (w + 1));
    memcpy(prev, &p->row0[3 * c0], sizeof(i64) * 3 * (w + 1));
    const i64* left = p->edges + (size_t)k * 3 * (p->m + 1);
    i64* right = p->edges + (size_t)(k + 1) * 3 * (p->m + 1);
    memcpy(&right[0], &p->row0[3 * c1], sizeof(i64) * 3);
    /* the checkpoint columns inside this slab (c0, c1] and their row 0 */
    const i64 q0 = c0 / p->CW + 1, q1 = c1 / p->CW;
    for (i64 q = q0; q <= q1; q++) memcpy(&p->colck[(size_t)(q - 1) * 3 * (p->m + 1)], &p->row0[3 * q * p->CW], sizeof(i64) * 3);
    for (i64 r0 = 1; r0 <= p->m; r0 += p->B) {
        const i64 r1 = r0 + p->B - 1 < p->m ? r0 + p->B - 1 : p->m;
        if (k > 0)
            while (atomic_load_explicit(&p->done[k - 1], memory_order_acquire) < r1) sched_yield();
        for (i64 i = r0; i <= r1; i++) {
            memcpy(cur, &left[3 * i], sizeof(i64) * 3);
            const uint8_t ai = p->a[i - 1];
            for (i64 j = 1; j <= w; j++)
                gao_cell(&prev[3 * (j - 1)], &cur[3 * (j - 1)], &prev[3 * j], p->sub[ai * p->K + p->b[c0 + j - 1]],
                         p->gh[p->b[c0 + j - 1]], p->gv[ai], p->o, &cur[3 * j]);
            memcpy(&right[3 * i], &cur[3 * w], sizeof(i64) * 3);
            for (i64 q = q0; q <= q1; q++)
                memcpy(&p->colck[(size_t)(q - 1) * 3 * (p->m + 1) + 3 * i], &cur[3 * (q * p->CW - c0)], sizeof(i64) * 3);
            if (i % p->BH == 0 && i / p->BH <= p->m / p->BH)
                memcpy(&p->rowck[(size_t)(i / p->BH - 1) * 3 * (p->n + 1) + 3 * c0], cur, sizeof(i64) * 3 * (w + 1));
            i64* t = prev; prev = cur; cur = t;
        }
        atomic_store_explicit(&p->done[k], r1, memory_order_release);
    }
    if (k == p->T - 1) memcpy(p->last, &prev[3 * w], sizeof(i64) * 3);
    free(prev);
    free(cur);
    return NULL;
}

/* Returns as gao_traceback (0 ok, 1 IndexError, -1 out of memory); *ntiles: tiles the walk recomputed. */
int gao_align_ckpt(const uint8_t* a, i64 m, const uint8_t* b, i64 n, const char* a_chr, const char* b_chr,
                   const i64* sub, int K, const i64* gh, const i64* gv, i64 o, const i64* row0, const i64* col0,
                   int T, i64 BH, i64 CW, uint32_t* mt_state, char* out_a, char* out_mid, char* out_b, i64* out_len,
                   i64* nd, i64* last, i64* ntiles) {
    if (T < 1) T = 1;
    if (T > n) T = (int)n;
    if (BH < 1) BH = 1;
    if (CW < 1) CW = 1;
    ckf_t p = {a, m, b, n, sub, K, gh, gv, o, row0, T, 256, BH, CW, NULL, NULL, NULL, NULL, last};
    const i64 nbr = m / BH, nbc = n / CW;
    p.edges = (i64*)malloc(sizeof(i64) * 3 * (size_t)(m + 1) * (T + 1));
    p.rowck = (i64*)malloc(sizeof(i64) * 3 * (size_t)(n + 1) * (nbr > 0 ? nbr : 1));
    p.colck = (i64*)malloc(sizeof(i64) * 3 * (size_t)(m + 1) * (nbc > 0 ? nbc : 1));
    p.done = (_Atomic i64*)calloc(T, sizeof(i64));
    tiles_t tl = {a, b, sub, K, gh, gv, o, m, n, BH, CW, row0, col0, NULL, NULL, -1, -1, NULL, NULL, NULL, 0};
    tl.sets = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)BH * CW);
    tl.prev = (i64*)malloc(sizeof(i64) * 3 * (CW + 1));
    tl.cur = (i64*)malloc(sizeof(i64) * 3 * (CW + 1));
    int status = -1;
    if (p.edges && p.rowck && p.colck && p.done && tl.sets && tl.prev && tl.cur) {
        memcpy(p.edges, col0, sizeof(i64) * 3 * (m + 1));
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * T);
        ckf_arg* args = (ckf_arg*)malloc(sizeof(ckf_arg) * T);
        for (int k = 0; k < T; k++) {
            args[k].p = &p;
            args[k].k = k;
            pthread_create(&th[k], NULL, ckf_worker, &args[k]);
        }
        for (int k = 0; k < T; k++) pthread_join(th[k], NULL);
        free(th);
        free(args);
        free(p.edges);
        p.edges = NULL;
        tl.rowck = p.rowck;
        tl.colck = p.colck;
        cells_t cs = {2, m, n, o, NULL, NULL, row0, col0, &tl};
        status = gao_traceback(&cs, a, b, a_chr, b_chr, sub, K, gh, 0, mt_state, out_a, out_mid, out_b, out_len, nd);
    }
    *ntiles = tl.recomputed;
    free(p.edges);
    free(p.rowck);
    free(p.colck);
    free((void*)p.done);
    free(tl.sets);
    free(tl.prev);
    free(tl.cur);
    return status;
}
