/*
 * globalign_amd.h -- C ABI of the MI355X affine-gap global-alignment engine.
 *
 * The reference (iamgiddyaboutgit/globalign) is pure CPython with no FFI; each
 * entry point below replaces the Python function(s) cited next to it
 * (paths relative to the reference's src/globalign/).  The Python host layer
 * (globalign_amd/_native.py) binds these with ctypes; INTEGRATION.md shows
 * the binding a globalign maintainer would add.
 *
 * Conventions: every function returns 0 on success or a negative GA_E* code;
 * ga_last_error() then describes the failure (thread-local).  Host buffers
 * are caller-owned; device buffers are owned by the context.  A context is
 * bound to one GPU and is not thread-safe (one per host thread).
 */
#ifndef GLOBALIGN_AMD_H
#define GLOBALIGN_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GA_OK 0
#define GA_E_ARG -1      /* invalid argument (maps to ValueError)          */
#define GA_E_HIP -2      /* HIP runtime failure (maps to RuntimeError)     */
#define GA_E_RANGE -3    /* int32 range / size limit exceeded               */
#define GA_E_STATE -4    /* call order violated (e.g. traceback before fill) */
#define GA_E_TIMEOUT -5  /* a device-side wait exceeded its spin bound      */
#define GA_E_NOMEM -6    /* device memory too small for the chosen path      */

/* Python-visible outcome of a traceback (dp_array_backward semantics). */
#define GA_TB_OK 0
#define GA_TB_INDEX_ERROR 1 /* the reference raises IndexError */

typedef struct ga_ctx ga_ctx;

/* Integer tables derived from the costing matrix (start.py:500-557).  Codes
 * index the alphabet in any fixed order; the gap character has a code too. */
typedef struct {
    int32_t K;              /* alphabet size including the gap code           */
    const int32_t* sub;     /* K*K: costing_mat[x][y]                         */
    const int32_t* gap_h;   /* K:   costing_mat['-'][y] (globaligner.py:347) */
    const int32_t* gap_v;   /* K:   costing_mat[x]['-'] (globaligner.py:357) */
    int32_t gap_open;       /* gap_open_cost >= 0                             */
    int32_t max_cost;       /* get_max_val(costing_mat) (start.py:488-497)   */
} ga_costs;

/* Last error message of this thread ("" if none). */
const char* ga_last_error(void);

/* Number of visible HIP devices. */
int ga_device_count(int* count);

/* Create / destroy a context on HIP device `device`.  ga_ctx_create reads the shipped GA_* environment knobs
 *  once; ga_ctx_create_opts also takes explicit options, "GA_NAME=VALUE" entries separated by ';' or
 * newlines (kernel variants for tests and tuning, fault injection, diagnostics: never read from the environment).
 * No reference counterpart: the reference has no device context. */
int ga_ctx_create(int device, ga_ctx** out);
int ga_ctx_create_opts(int device, const char* options, ga_ctx** out);
void ga_ctx_destroy(ga_ctx* ctx);

/* How the library was built: flags[0] bit 0 = an experiments build (measured-and-dropped paths compiled in). */
int ga_build_flags(int32_t* flags);

/* Load a problem: sequence codes (host), tables, optional custom boundaries.
 * Replaces make_dp_array (globaligner.py:756-821): when row0/col0 are NULL the
 * boundary is the reference's (finite sentinel big=(max_cost+1)*max(m,n));
 * otherwise row0 = 3*(n+1) and col0 = 3*(m+1) triples (M, X, Y) as in the
 * reference's own test (tests/globaligner_test.py:8-33).  Uploads to HBM. */
int ga_problem_set(ga_ctx* ctx, const uint8_t* a, int64_t m, const uint8_t* b, int64_t n, const ga_costs* costs,
                   const int32_t* row0, const int32_t* col0);

#define GA_FILL_TRACEBACK 1 /* store per-cell traceback words (needed by ga_problem_traceback) */
#define GA_FILL_FULL 2      /* also return every cell's (M, X, Y) (small problems only)       */

/* Matrix fill (dp_array_forward, globaligner.py:366-392 with
 * get_next_best_costs :317-363) on the loaded problem.  *cost_out receives
 * min(dp[m][n]) (globaligner.py:425).  With GA_FILL_FULL, full_out receives
 * 3*(m+1)*(n+1) int32 (row-major, boundary included). */
int ga_problem_fill(ga_ctx* ctx, int32_t flags, int64_t* cost_out, int32_t* full_out);

/* Traceback walk (dp_array_backward :395-593, cost_ranks_dispatcher
 * :595-685, take_* :688-753) on the last GA_FILL_TRACEBACK fill.
 * mt_state: 625 words = random.getstate()[1] in, the state after the
 * reference's random.choice calls out.  a_chr/b_chr: the upper-cased
 * sequences.  out_* need cap >= m+n+1 bytes; strings are not terminated.
 * *tb_status receives GA_TB_OK or GA_TB_INDEX_ERROR. */
int ga_problem_traceback(ga_ctx* ctx, uint32_t* mt_state, const char* a_chr, const char* b_chr, char* out_a,
                         char* out_mid, char* out_b, int64_t cap, int64_t* out_len, int32_t* tb_status);

/* Use a caller-filled cell array for the next ga_problem_traceback instead of
 * a fill: cells = 3*(m+1)*(n+1) int32 (M, X, Y), row-major, boundary
 * included (the loaded problem's row0/col0 must be its row 0 / column 0).
 * Replaces the part of dp_array_backward (globaligner.py:425-514) that reads
 * the caller's dp_array: the walk then follows THOSE cells, whatever filled
 * them.  *cost_out = min(cells[m][n]).  Small problems only. */
int ga_problem_set_cells(ga_ctx* ctx, const int32_t* cells, int64_t* cost_out);

/* fill + traceback in one call, overlapping the host-side tie-break table
 * with the device fill (the whole find_global_alignment hot path,
 * globaligner.py:258-302). */
int ga_problem_align(ga_ctx* ctx, uint32_t* mt_state, const char* a_chr, const char* b_chr, char* out_a,
                     char* out_mid, char* out_b, int64_t cap, int64_t* out_len, int32_t* tb_status,
                     int64_t* cost_out);

/* `count` consecutive alignments of the loaded pair, exactly as `count`
 * consecutive find_global_alignment calls make them: alignment k starts from
 * the random state alignment k-1 left (repeated calls sample the co-optimal
 * alignments the reference's tie-breaks reach).  The walk of alignment k runs
 * on a second stream beside the fill of alignment k+1 (double-buffered
 * traceback words; the tie-break table is one continuous MT19937 stream), so
 * the throughput is one fill per alignment.  out_a/out_mid/out_b: count*cap
 * bytes, alignment k at offset k*cap; out_len, tb_status, cost_out: count
 * entries; mt_state: in the state before the first alignment, out the state
 * after the last. */
int ga_problem_align_many(ga_ctx* ctx, int32_t count, uint32_t* mt_state, const char* a_chr, const char* b_chr,
                          char* out_a, char* out_mid, char* out_b, int64_t cap, int64_t* out_len, int32_t* tb_status,
                          int64_t* cost_out);

/* ---- multi-GPU column slabs ----------------------------------
 * A context can own the column slab [col_begin, col_end) of a larger problem
 * (global m, n and boundary).  Its left edge arrives in `halo_in`
 * ((m+1) x int2 of (H', h1') in the shifted space of DESIGN.md) guarded by
 * the progress word `halo_in_prog` (rows available, written by the host when
 * a band has arrived); its right edge is produced into `halo_out` with the
 * progress word `halo_out_prog` (rows published by the fill).  Both words are
 * HOST pointers into pinned coherent memory that the running fill reads and
 * writes, so the host can stream bands with RCCL send/recv without blocking
 * a device queue. */
int ga_problem_set_slab(ga_ctx* ctx, const uint8_t* a, int64_t m, const uint8_t* b, int64_t n, const ga_costs* costs,
                        int64_t col_begin, int64_t col_end);
int ga_slab_buffers(ga_ctx* ctx, void** halo_in, uint32_t** halo_in_prog, void** halo_out, uint32_t** halo_out_prog);
/* Use caller-owned device buffers ((m+1) x int2 each) as the slab's left-edge
 * input and right-edge output (e.g. tensors that RCCL receives into / sends
 * from); NULL keeps the context's own buffer.  Their progress goes through the context's own
 * words (ga_slab_buffers): this undoes a ga_slab_link / _export / _import. */
int ga_slab_bind_halos(ga_ctx* ctx, void* halo_in, void* halo_out);
/* Join two neighbouring slab contexts of ONE process (GlobalAligner(devices=[...])) device to device: the
 * right context allocates its left edge (m + 1 int2 rows) and a progress word in uncached device memory
 * on its own GPU, and the left context's fill writes both directly -- system-scope stores, over xGMI
 * when the contexts sit on different GPUs (peer access is enabled here) -- while the right context's
 * fill polls the word.  No host thread relays anything.  Call after ga_problem_set_slab on both
 * contexts and before either fill is launched (it zeroes the word); launch left before right.
 * Replaces the pinned-host halos + host relay of round 2 (reference: none -- the reference is
 * single-threaded CPU code). */
int ga_slab_link(ga_ctx* left, ga_ctx* right);
/* The same link between two PROCESSES (one GPU each, bench.py --gpus N): the right slab's context allocates
 * its left edge + progress word (uncached, on its GPU; zeroing the word) and exports an IPC handle
 * (HIP_IPC_HANDLE_SIZE = 64 bytes); the left slab's context maps it (hipIpcOpenMemHandle, peer access
 * enabled lazily; kept while the handle stays the same) and its fill stores the edge there directly.
 * Per problem: export on the right, hand the bytes over (any channel), import on the left, and launch
 * the left fill only after the right side's export returned (the word is zero). */
int ga_slab_link_export(ga_ctx* right, void* handle_out);
int ga_slab_link_import(ga_ctx* left, const void* handle);
/* Let `device` read and write `peer`'s memory (hipDeviceEnablePeerAccess); GA_OK if already enabled. */
int ga_enable_peer_access(int device, int peer);
/* Launch the slab fill asynchronously on the context's compute stream. */
int ga_slab_fill_launch(ga_ctx* ctx, int32_t flags);
/* Wait for the slab fill; returns H'(m, col_end) un-shifted (only meaningful on the last slab). */
int ga_slab_fill_finish(ga_ctx* ctx, int64_t* cost_out);

/* Traceback across slabs (dp_array_backward :395-593 cut at slab edges): the
 * walk starts on the slab owning column n and moves right to left; each slab
 * continues the state its right neighbour handed over. */
typedef struct {
    int64_t i, j;   /* current cell (j: global column)                        */
    int64_t D, h;   /* dispatches so far; moves after the first one            */
    int32_t L;      /* level the walk entered the cell with (0 M, 1 X, 2 Y)    */
    int32_t first;  /* 1 before the first move                                 */
    int32_t reason; /* -1 running; 0..4 ended (as the whole-problem walk);
                       5 reached this slab's left edge (continue on the left)  */
    int32_t pad;
} ga_walk_state;
/* Build the host tie-break table of the global problem from the 625-word MT
 * state (call while the fill runs). */
int ga_slab_walk_prepare(ga_ctx* ctx, const uint32_t* mt_state);
/* Walk this slab from *st (j must be the slab's right edge); writes the
 * alignment columns it produced in walk order (not reversed, no tails) and
 * updates *st.  a_chr / b_chr: the whole upper-cased sequences. */
int ga_slab_walk(ga_ctx* ctx, ga_walk_state* st, const char* a_chr, const char* b_chr, char* out_a, char* out_mid,
                 char* out_b, int64_t cap, int64_t* out_len);
/* MT state after the first D dispatches (random.getstate()[1] layout). */
int ga_slab_mt_state(ga_ctx* ctx, int64_t D, uint32_t* mt_state_out);
/* Enqueue on `stream` (a hipStream_t): wait until *prog >= value / write value to *prog. */
int ga_stream_wait_ge(void* stream, uint32_t* prog, uint32_t value);
int ga_stream_write(void* stream, uint32_t* prog, uint32_t value);
/* The context's compute stream (hipStream_t).  It is created with the
 * device's greatest stream priority, so it owns a hardware queue that no
 * normal-priority stream (torch's, RCCL's) shares: a slab fill waiting on its
 * halo never holds up the RCCL kernel that delivers it. */
void* ga_ctx_stream(ga_ctx* ctx);
/* Order the context's stream after all work enqueued so far on `stream`
 * (a hipStream_t, e.g. torch.cuda.current_stream().cuda_stream): buffers that
 * stream allocated or initialised are then safe for the next fill. */
int ga_ctx_wait_stream(ga_ctx* ctx, void* stream);
/* The priority the context's stream was created with (hipDeviceGetStreamPriorityRange units). */
int ga_ctx_stream_priority(ga_ctx* ctx, int* priority);

/* ---- measurement --------------------------------------------------------- */
/* Device time (ms, HIP events on the launch stream) of the last fill kernel
 * and of the last traceback walk kernel. */
int ga_last_kernel_ms(ga_ctx* ctx, float* fill_ms, float* walk_ms);
/* out4 = {fill kernel ms, walk kernel ms, host tie-break table ms, whole ga_problem_align wall ms}. */
int ga_last_timings(ga_ctx* ctx, float* out4);

#ifdef __cplusplus
}
#endif
#endif
