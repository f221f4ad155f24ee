// ga_device.h -- types shared by the HIP kernels (ga_kernels.hip) and the host
// library (ga_host.cpp).  See DESIGN.md for the layouts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ga {

// Row-scan fill: a workgroup = NWC compute waves (4 or 8) + 1 IO wave.
constexpr int RING = 256;        // rows per LDS edge ring between consecutive waves
constexpr int RMASK = RING - 1;
constexpr int FROWS = 16;        // rows per fill chunk (one 16-byte traceback store per lane per CB)
#ifndef GA_GOUT
#define GA_GOUT 4
#endif
constexpr int GOUT = GA_GOUT;    // rows per cross-workgroup publish (4: C3 cross-workgroup lag 4.8 -> 3.5 us)
// an unwritten row of the workgroup hand-off buffer (memset byte 0x80): no H' reaches it (the
// int32 range guard keeps every value below INT32_MAX / 4 in magnitude)
constexpr int HAND_SENT = (int)0x80808080u;
constexpr int FILL_LDS_MIN = 82 * 1024;  // > 80 KB: one fill workgroup per CU

// the recompute fill's right-edge checkpoints: a stripe's rows 0..m, then this many scratch slots of its own (a store's
// offset from the stripe's base then fits the 32-bit VGPR offset of a global store with an SGPR base)
constexpr int COLCK_PAD = 64;

struct FillArgs {
    const uint8_t* a;         // m codes (seq_1)
    const int* subp;          // K x K: sub'(x, y) = sub(x, y) - gV(x) - gH(y)
    int K;
    const uint8_t* b;         // n codes of this slab's columns
    const int2* top;          // [n+1] (H', h2') of row 0 (index 0 = the slab's left corner)
    const int2* left;         // [m+1] (H', h1') of the slab's left edge
    const unsigned* left_prog;  // rows of `left` available (nullptr: all)
    int2* hand;               // [nslabs][m+1] right edge of each workgroup slab
    unsigned* ticket;         // slab ticket
    unsigned* abort_word;
    uint8_t* tb;              // traceback words or nullptr
    int* out_last;            // [4]: H'(m, n_local)
    unsigned* edge_prog;      // rows of the right edge published (last slab only; may be null)
    int2* edge_out;           // right edge of the last workgroup slab (nullptr: its hand slot)
    int* full;                // FULL output (shifted M', X', Y') or nullptr
    int m, n, o, nstripes, nslabs, TC;  // TC: 16-byte traceback words per lane per stripe
    int nwc, qrows;                     // compute waves per workgroup; LDS query-profile ring rows
    int cols_per_lane;                  // T: columns per lane (a stripe is 64*T columns; 1, 2 or 4)
    unsigned spin_limit, halo_spin_limit;
    unsigned long long* dbg;  // optional timestamps: [nstripes][8] or nullptr
    int2* ckpt;               // banded traceback: (H', h2') of rows ckpt_rows, 2*ckpt_rows, ... (< m) or nullptr
    int ckpt_rows;            //   [row / ckpt_rows - 1][n + 1]; a multiple of FROWS
    // recompute checkpoints of the lane fill (nullptr: none)
    int2* colck;              // [nstripes][m + 1 + COLCK_PAD]: (H', h1') of every stripe's right edge column, rows
                              // 1..m, then 64 scratch slots of the stripe (the lean sub-chunk's lanes that carry no
                              // row store there)
    int2* stck;               // staircase lane states after step k*stck_every - 1, k = 1 .. (m - 1) / stck_every:
                              //   [k - 1][nstripes][TD + 1][64]: (H'[c], h2'[c]) for c < TD, then (h1' carry, H' diag)
    int stck_every;           //   a power of two >= 64 (pairs of 16-step sub-chunks)
    int stck_shift;           //   log2(stck_every)
    int late;                 // lane fill, score only: late edge reads (one-round chains; ga_lane.hip LATE)
    int hand_direct;          // lane fill: the last compute wave stores the hand-off rows (else the IO wave)
    // tuning overrides from the context's knobs (ga_ctx::knobs; < 0: the default): LDS floor per workgroup
    // (GA_FILL_LDS_FLOOR), lane-fill sub-chunk steps score only (GA_LANE_SUB) / with words (GA_LANE_TB_SUB)
    int lds_floor, lane_sub, lane_tb_sub;
    int asm_step;             // lane fill, score only: the lean asm sub-chunk (ga_lane_asm.h LaneSub), else the compiler's
                              // steps (GA_LANE_ASM=0)
    int io_prio;              // lane fill: s_setprio of the IO and profile waves (GA_LANE_IOPRIO; 0: none)
    int poll_win;             // lane fill: rows per hand-off poll (GA_LANE_POLLWIN, <= 192; 0: 16 while the writer is behind, else 192)
    int out_wave;             // lane fill (NWC <= 4): the out-path in a wave of its own (GA_LANE_OUTWAVE; 0: the IO wave's)
    int hand_scope;           // lane fill: workgroup hand-off polls with system-scope loads (1), and stores (2)
    int xcd_map;              // lane fill, one round of workgroups: chain neighbours on one XCD (ga_lane.hip lane_slab)
    // lane fill: the query profile of this fill's rows in HBM (launch_lane_qprof, [K][m + 4] dwords, dword r + 2 = the
    // sub' bytes of rows r .. r+3 of one column code, rows outside 1..m zero), copied into the LDS ring by the profile
    // wave; nullptr: the profile wave computes it from a and sub'
    const uint32_t* qprof;
    // lane fill, score only: the lean sub-chunk from the first step (ga_lane.hip), allowed when row 0 is uniform in the
    // shifted domain (H'(0, j) = o and h2'(0, j) = 2o for every column: the reference's boundary with 2o + GH(n) <=
    // big): lanes still above row 1 then step on zero profile bytes and keep exactly those values
    int lean0;
};

// Traceback word layout (fill -> walk): per stripe s, lane l (column 64s+l+1),
// 16-byte word q holds rows q*SPC+1 .. q*SPC+SPC (SPC = 16/CB), CB bytes per cell:
//   tb + ((s * TC + q) * 64 + l) * 16 + ((i-1) % SPC) * CB

struct WalkArgs {
    const uint8_t* tb;
    int CB, TC;
    const uint8_t* a;
    const uint8_t* b;     // this slab's columns
    const int* bnd_row;   // 3(n+1) original boundary triples
    const int* bnd_col;   // 3(m+1)
    const uint32_t* rng;  // per dispatch: level chosen for candidate set S at bits 2S (match) / 16+2S (mismatch)
    long long nrng;
    int m, n, o;          // n: this slab's columns
    int i0, j0, L0, first0, D0, h0;  // start state (j0 local); a whole problem starts at (m, n, 0, 1, 0, 0)
    int handoff;          // 1: the slab has columns to its left; reaching local column 0 ends the walk here
    int vhandoff;         // 1: a traceback band with rows above it; reaching local row 0 ends it (reason 6)
    int maxh;             // the reference's move bound m + n (global n)
    uint32_t* ops;        // out: 2-bit levels, dispatch D at bits 30 - 2*(D & 15) of word D >> 4
    int* result;          // out: [D, i, j, reason, diagnostics...]
    unsigned* dbg;        // optional: per tile need (ti, tj, D, wait ticks) x WALK_DBG entries, or nullptr
    int skip_corners;     // loaders leave the block's far off-diagonal tiles (offsets (3,0), (0,3), (3,1), (1,3))
    int nloaders;         // loader waves: 12, 13 (+ the idle wave 12) or 14 (+ wave 8, no L2 prefetcher)
    // the recompute walk (walk_rc_kernel; unused by the other walks)
    unsigned* rc_flags;        // [nbi][nbs] per 64-row block of a fill stripe: rc_ready once its words are written
    unsigned rc_ready;
    unsigned long long* rc_own;  // [RC_CACHE_I][RC_CACHE_S] the block whose words a cache slot holds (rc_slot_tag)
    int rc_nbs, rc_td;         // blocks per block row; 64-column tiles per block (the fill's TD)
    unsigned* rc_pos;          // [0] the walker's tile (ti << 16 | tj), [1] 1 once the walk has ended
    // optional (nullptr): dispatches whose levels are in `ops` (pinned host memory then), raised by the
    // helper after each flush with a system-scope release, the exact count once the walk has ended -- the
    // host decodes the alignment while the walk runs (rc_align)
    unsigned* ops_prog;
};

// The recompute walk's tile cache: block (bi, bs) (64 rows of fill stripe bs) lives at slot
// (bi mod RC_CACHE_I, bs mod RC_CACHE_S).  Candidates lie at most RC_SPAN_I - 1 = 31 block rows and RC_SPAN_S - 1
// = 7 stripes up-left of the walker's block as a worker saw it (offsets dbi * 8 + dbs in a byte), and the cache is
// twice that deep on both axes: a worker whose view of the walker is stale can then never overwrite a block the
// walker may still read (the safety argument at rc_block's cache store, ga_rcwalk.hip; ADVICE r3: with a cache
// only as deep as the candidates it could).  Deep along the rows, narrow across the stripes: a 64-row block is a
// quarter of a TD 4 stripe's width, and the path runs near the diagonal.
constexpr int RC_SPAN_I = 32;
constexpr int RC_SPAN_S = 8;
constexpr int RC_CACHE_I = 2 * RC_SPAN_I;
constexpr int RC_CACHE_S = 32;

// A cache slot's owner tag: the block whose words the slot holds, with the call's ready value, or 0 while
// a worker that claimed a block of that slot may be rewriting it.  The worker clears the tag before its first word
// store and sets it after the last, then raises the block's flag; a loader reads the tag before and after it copies
// a tile, so words another block's worker overwrote are never used, whatever the timing (the reach check's margin
// alone made that a matter of timing), and a ready flag whose slot has lost its words is reset for a recompute.
__host__ __device__ inline unsigned long long rc_slot_tag(int bi, int bs, int nbs, unsigned ready) {
    return ((unsigned long long)((unsigned)bi * (unsigned)nbs + (unsigned)bs + 1u) << 32) | ready;
}
__host__ __device__ inline int rc_slot(int bi, int bs) { return (bi % RC_CACHE_I) * RC_CACHE_S + bs % RC_CACHE_S; }

// The recompute workgroups of walk_rc_kernel (ga_rcwalk.hip): each wave recomputes 64-row
// blocks of one fill stripe (64*TD columns) from the lane fill's checkpoints, writing their traceback words.
struct RcArgs {
    const uint8_t* a;      // m codes
    const uint8_t* b;      // n codes (this slab's columns)
    const int* subp;       // K x K sub'
    int K;
    const int2* top;       // [n+1] (H', h2') of row 0
    const int2* left;      // [m+1] (H', h1') of column 0
    const int2* colck;     // [nstripes][m + 1 + COLCK_PAD] right edges (FillArgs::colck)
    const int2* stck;      // staircase states (FillArgs::stck)
    int stck_every;
    uint8_t* tb;           // traceback words (ga_device.h layout), TC 16-byte words per lane per 64-column stripe
    int TC, m, n, o;
    int TD, nstripes, nbi, nbs;  // nbs = nstripes; nbi = 64-row blocks
    unsigned* flags;       // [nbi][nbs]: < 2*epoch free, 2*epoch claimed, 2*epoch + 1 ready
    unsigned epoch;
    unsigned long long* own;  // WalkArgs::rc_own
    int tag_fault;            // test knob GA_RC_TAG_FAULT=k: each worker leaves the tag of every k-th block unset
    unsigned* pos;         // the walk's WalkArgs::rc_pos
    int tile0;             // the walk's first tile (ti << 16 | tj), until it publishes one
    int workers;           // waves per workgroup that recompute (the rest leave)
    int worker_bytes;      // LDS per worker
    unsigned spin_limit;   // idle polls before a worker gives up (the walk then reports its own timeout)
    int nwin;              // window blocks (<= 64)
    unsigned char off[64]; // window offsets (dbi << 4 | dbs) from the walker's block, likeliest first
    const uint4* jlut;     // the tie-to-tie walk's worker LUT (1024 entries, jump_lut_build), or nullptr
};

// Pipelined walks in one launch (walk_chain_kernel): walk k uses w[k % S] with rng = tab + G_k.
constexpr int WALK_CHAIN_SLOTS = 6;
struct WalkChainArgs {
    WalkArgs w[WALK_CHAIN_SLOTS];  // per slot: words, boundary, levels, result (rng / nrng set per walk)
    const uint32_t* tab;           // the continuous tie-break stream (pinned host memory, device address)
    const long long* tab_ready;    // pinned: entries of tab written so far
    unsigned* ctl;                 // pinned: [0] fills done, [1] walks done, [2] host abort, [3] wait timed out
    long long per;                 // entries one walk may read (m + n + 1)
    unsigned long long wait_limit; // s_memrealtime ticks (100 MHz) a walk may wait for its fill / entries
    int count, S;
};

void launch_boundary(hipStream_t s, const uint8_t* a, int m, const uint8_t* b, int n, const int* gh, const int* gv,
                     int o, int big, int* GVp, int* GHp, int2* top, int2* left, int* bnd_row, int* bnd_col, int* meta,
                     bool custom, int* scratch);
int boundary_scratch_ints(int m, int n);  // ints of scratch launch_boundary needs
void launch_fill(hipStream_t s, const FillArgs& p, int CB, int qbytes, bool tb, bool full);
size_t fill_lds_bytes(int nwc, int qbytes, int K, int qrows, int tb_stage_bytes_per_wave = 0);
void launch_walk(hipStream_t s, const WalkArgs& w);
void launch_walk_chain(hipStream_t s, const WalkChainArgs& a);
// the recompute walk: one walker workgroup + nserv recompute workgroups (ga_rcwalk.hip)
void launch_walk_rc(hipStream_t s, const WalkArgs& w, const RcArgs& r, int nserv);
int rc_worker_bytes(int TD, int CB, int stck_every);
// the tie-to-tie walk (ga_jump.h): the same launch with jump entries instead of traceback words
// (TD <= 4, o <= 14); r.tb is then the entry cache (RC_CACHE_I x RC_CACHE_S blocks of 4*TD 6 KB tiles)
void launch_walk_rc_jump(hipStream_t s, const WalkArgs& w, const RcArgs& r, int nserv);
int rc_jump_worker_bytes_host(int TD, int stck_every);
size_t rc_jump_lds_bytes(int TD, int stck_every);  // LDS of a workgroup with one jump worker
// The jump workers' LUT (host, ga_host.cpp): entry idx = fx | fy << 4 | (M' != H') << 8 | (a != b) << 9, fx / fy the
// cell's X'-H' / Y'-H' saturated at o+1 (o <= 14): {v_perm selectors of levels 0 | 1 << 16, of level 2 (high half
// 0x0c0c), tie words of levels 0 | 1 << 16, of level 2}
void jump_lut_build(int o, uint32_t* out4096);
// traceback words of a caller-supplied (m+1) x (n+1) x 3 cell array (dp_array_backward shim)
void launch_tb_from_cells(hipStream_t s, const int* cells, int m, int n, int o, int CB, int TC, uint8_t* tb);
// score-only anti-diagonal fill (64-column stripes; FillArgs.cols_per_lane must be 1)
void launch_fill_diag(hipStream_t s, const FillArgs& p, int qbytes, bool full);
size_t fill_diag_lds_bytes(int nwc, int qbytes, int K, int qrows);
// lane-skewed anti-diagonal fill (ga_lane.hip; FillArgs.cols_per_lane = TD in {1, 2, 4, 8}, <= 4 with
// traceback words (p.tb != nullptr, CB bytes per cell), int8 profile, K <= 32, qrows = profile rows, a power of two)
void launch_fill_lane(hipStream_t s, const FillArgs& p, int CB);
size_t fill_lane_lds_bytes(int nwc, int K, int qrows);
// the lane fill's query profile (FillArgs::qprof) of rows a[0 .. m-1]: K x (m + 4) dwords at out
void launch_lane_qprof(hipStream_t s, const uint8_t* a, int m, const int* subp, int K, uint32_t* out);

}  // namespace ga
