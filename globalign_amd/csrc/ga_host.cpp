// ga_host.cpp -- host side of the C ABI declared in include/globalign_amd.h.
//
// Owns device memory and the HIP stream of one context, runs the kernels of
// ga_kernels.hip, and does the two pieces of the traceback that are
// inherently host-side in the reference's semantics:
//   * the tie-break table: the reference draws 18 random.choice values per
//     dispatched traceback step from CPython's global MT19937
//     (globaligner.py:598-672); we emulate genrand_uint32 and
//     _randbelow_with_getrandbits exactly, starting from random.getstate(),
//     while the device fill runs;
//   * string assembly from the walk's per-step levels (take_* :688-753,
//     the i==0 / j==0 tails :542-581 and the final reverse :584-586).
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/globalign_amd.h"
#include "ga_device.h"
#include "ga_lane.h"
#include "ga_check.h"
#include "ga_rng.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(GA_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));              \
    } while (0)

// ------------------------------------------------------------------ buffers
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool uncached = false;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 256);
        hipError_t e = uncached ? hipExtMallocWithFlags(&p, want, hipDeviceMallocUncached) : hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

using namespace garng;
static_assert(ga::COLCK_PAD == 64, "rc_rows_fit (ga_check.h) assumes a 64-row pad");

}  // namespace

// ------------------------------------------------------------------ context
// The GA_* variables the shipped library reads from the environment (INTEGRATION.md lists them): the path choices
// and budgets an operator may want to set.  Every other option -- kernel variants for tests and tuning, fault
// injection, diagnostics -- reaches a context only through ga_ctx_create_opts, never from the environment, so a
// stray variable cannot change a production context's kernels or inject a fault.  An experiments build
// (make EXPERIMENTS=1) takes every GA_* variable.
const char* const kEnvKnobs[] = {"GA_RC",           "GA_RC_MIN_CELLS", "GA_RC_BUDGET_MB",      "GA_RC_EVERY",
                                 "GA_RC_SERVERS",   "GA_TB_BUDGET_MB", "GA_FILL_MODE",         "GA_COLS_PER_LANE",
                                 "GA_LANE_COLS_PER_LANE", "GA_PIPE_FILLS", "GA_PIPE_CHAIN",    "GA_STREAM_PRIORITY",
                                 "GA_HALO_SPIN_LIMIT", "GA_PIPE_TRACE"};
bool env_knob(const std::string& name) {
#ifdef GA_EXPERIMENTS
    return name.compare(0, 3, "GA_") == 0;
#else
    for (const char* k : kEnvKnobs)
        if (name == k) return true;
    return false;
#endif
}

struct ga_ctx {
    // GA_* tuning / diagnostic overrides, snapshotted when the context is created (ga_ctx_create_opts): the
    // environment's shipped knobs (kEnvKnobs) at that moment, then the caller's options.  A context's kernel choices
    // never change under it, whatever the process does to its environment later (nullptr: unset).
    std::map<std::string, std::string> knobs;
    const char* knob(const char* name) const {
        const auto it = knobs.find(name);
        return it == knobs.end() ? nullptr : it->second.c_str();
    }
    // knobs of paths that were measured and dropped: read only by an experiments build
    // (make EXPERIMENTS=1); the shipped library ignores them
    const char* xknob(const char* name) const {
#ifdef GA_EXPERIMENTS
        return knob(name);
#else
        (void)name;
        return nullptr;
#endif
    }
    int device = 0;
    int priority = 0;  // of `stream` (the greatest the device offers, see ga_ctx_create)
    hipStream_t stream = nullptr;
    hipEvent_t ev_dep = nullptr;  // ga_ctx_wait_stream
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // problem
    bool loaded = false, custom = false, filled_tb = false;
    int64_t m = 0, n = 0;      // local problem (slab: n = local columns)
    int64_t n_global = 0, col0 = 0;
    int K = 0, o = 0, big = 0, CB = 1, qbytes = 1;
    int64_t gh_total = 0;      // GH(n_global): the sum of the horizontal gap costs of seq_2
    int64_t gv_total = 0;      // GV(m): the sum of the vertical gap costs of seq_1
    // a streamed single call's small results in pinned, coherent host memory (no copy after the walk): [0, 16) the
    // walk's result words (it writes them there), [16, 20) the fill's H'(m, n) words, [20] its abort word (copied on
    // the upload stream while the walk runs); res_dev: the same memory as the device sees it
    int* res_pin = nullptr;
    int* res_dev = nullptr;
    hipEvent_t ev_fill = nullptr, ev_res = nullptr;
    bool rc_pos_zeroed = false;  // rc_pos was cleared on the fill's stream before the fill (rc_align)
    int nstripes = 0, nslabs = 0, TC = 0, nwc = 4, qrows = 1024, num_cu = 256;
    int T = 1, T_req = 0, nwc_req = 0;
    int diag_req = 0;          // score-only fill kernel: 0 automatic, 1 row scan, 2 anti-diagonal, 3 lane-skewed (GA_FILL_MODE)
    int lane_T_req = 0;        // columns per lane of the lane-skewed kernel (GA_LANE_COLS_PER_LANE; 0: automatic)
    bool lane = false;         // the last enqueued fill used the lane-skewed kernel
    int diag_T_req = 0;        // columns per lane of the anti-diagonal kernel (GA_DIAG_COLS_PER_LANE; 0: automatic)
    bool diag = false;         // the last enqueued fill used the anti-diagonal kernel      // columns per lane of the fill (T_req 0: automatic; GA_COLS_PER_LANE)
    int64_t GV_m = 0, GH_n = 0;
    std::vector<uint8_t> h_a, h_b;
    // device buffers
    DevBuf a, b, sub, gh, gv, qp, GVp, GHp, top, left, bnd_row, bnd_col, meta, hand, flags, tb, out_last, full, rng, bscr,
        ckpt,
        ops, result;
    DevBuf halo_in{nullptr, 0, true};
    bool slab = false;
    // slab progress words in pinned, coherent host memory: [0] halo_in rows (written by the host
    // when a band has arrived), [1] halo_out rows (written by the fill's IO wave)
    uint32_t* prog_host = nullptr;
    uint32_t* prog_dev = nullptr;
    int2* halo_in_ext = nullptr;   // caller-bound halo buffers (e.g. tensors RCCL sends from / receives into)
    int2* halo_out_ext = nullptr;
    // caller-bound progress words (device-visible; e.g. on the reading GPU, written over xGMI by the
    // writing GPU's fill): nullptr keeps prog_dev[0] / prog_dev[1]
    uint32_t* in_prog_ext = nullptr;
    uint32_t* out_prog_ext = nullptr;
    RngTable walk_rng;             // tie-break table of the global problem (slab walks)
    // pipelined repeated alignments (ga_problem_align_many): two slots of traceback words, walk
    // buffers and events; the walk runs on its own stream beside the next fill
    struct PipeSlot {
        DevBuf tb, hand, flags, out_last, rng, ops, result;
        // each pipelined alignment computes its own boundary (make_dp_array) into its slot
        DevBuf GVp, GHp, top, left, bnd_row, bnd_col, meta, bscr;
        hipEvent_t f0 = nullptr, f1 = nullptr, fdone = nullptr, w0 = nullptr, w1 = nullptr;
        uint32_t* tab_pin = nullptr;  // pinned staging of the walk's table slice
        int64_t tab_cap = 0;
    } pipe[6];
    hipStream_t wstream = nullptr, fstream[4] = {nullptr, nullptr, nullptr, nullptr};  // [0] unused: ctx->stream
    // CU-masked pipeline streams (GA_PIPE_WALK_CUS > 0): the walk keeps CUs of its own, the fills the rest
    hipStream_t mwstream = nullptr, mfstream[4] = {nullptr, nullptr, nullptr, nullptr};
    // default-priority pipeline fill streams (GA_PIPE_FILL_PRIO=normal): four fills on their own pool of
    // hardware queues, the walk stream keeping the greatest priority (it takes the next free CU)
    hipStream_t nfstream[4] = {nullptr, nullptr, nullptr, nullptr};
    int walk_cus = -1;  // CUs reserved for the walk (0: no masks; -1: not yet set up)
    int* pipe_pin = nullptr;       // pinned: per slot {out_last[4], GV(m), GH(n), abort, pad}
    int pipe_fills = 2, pipe_slots = 3;  // fills in flight (one stream each) and slots (fills + the walked one)
    int hw_queues = 4;                   // GPU_MAX_HW_QUEUES as the process first saw it (ga_ctx_create)
    int pipe_lane_td = 0, pipe_lane_nwc = 0;  // the pipeline's lane-kernel fill geometry (0: the row scan)
    RngTable many_rng;
    // chained pipeline walks (walk_chain_kernel): the tie-break stream in pinned, coherent host memory
    // and the control words {fills done, walks done, abort, timed out, entries written (8 B at [4])}
    uint32_t* chain_tab = nullptr;
    int64_t chain_tab_cap = 0;
    unsigned* chain_ctl = nullptr;
    // the chain's stream, at the LEAST priority: HIP gives each priority its own pool of hardware
    // queues, and no other stream of the process uses this pool, so no fill can ever be queued behind
    // the persistent chain on an in-order queue it shares (the chain waits for those fills)
    hipStream_t cwstream = nullptr;
    // per slot, pinned and coherent: the walk's result words and levels, written by the chain straight
    // into host memory (a hipMemcpy would wait for a CU, and the fills hold them all)
    uint8_t* chain_io = nullptr;
    size_t chain_io_cap = 0;
    bool walk_rng_ready = false;
    float fill_ms = 0.f, walk_ms = 0.f, rng_ms = 0.f, call_ms = 0.f;
    bool dbg_on = false;
    int walk_waits = 0, walk_tiles = 0, walk_t_tile = 0, walk_t_ring = 0, walk_t_total = 0, walk_c_total = 0, walk_load_ticks = 0, walk_load_count = 0;
    DevBuf dbg, wdbg;
    // the recompute walk: the score fill's checkpoints, the tile cache, the blocks' flags
    DevBuf colck, stck, rc_tb, rc_flags, rc_pos, rc_own;
    DevBuf qprof;  // the lane fill's query profile (ga::launch_lane_qprof), rebuilt by every lane fill
    int walk_jump_diag[3] = {0, 0, 0};  // the tie-to-tie walk's trips, region re-checks, ties (result[12..14])
    DevBuf jlut;           // the jump workers' LUT for gap open jlut_o (ga::jump_lut_build)
    int jlut_o = -1;
    // ga_slab_link: this slab's left edge + its progress word, uncached device memory on this GPU that
    // the left neighbour's fill writes (over xGMI when it runs on another GPU)
    DevBuf link;
    // ga_slab_link_import: the right neighbour's link buffer, mapped from another process
    void* peer_link = nullptr;
    char peer_handle[64] = {};
    unsigned rc_epoch = 0;
    bool rc_used = false;  // the last fill was the recompute path's (ga_problem_align or a slab's)
    // rc_align's walk levels in pinned host memory and the helper's progress word: decoded while the walk runs
    uint32_t* rc_ops_pin = nullptr;
    int64_t rc_ops_cap = 0;  // words
    unsigned* rc_ops_prog = nullptr;
    // rc_align's tie-break table: pinned staging, uploaded on a stream of its own while the fill runs, so that the walk
    // is queued behind the fill at once (a pageable copy on the fill's stream held the calling thread to the fill's end)
    uint32_t* up_pin = nullptr;
    int64_t up_cap = 0;  // entries
    hipStream_t ustream = nullptr;
    hipEvent_t ev_up = nullptr;
    int rc_T = 0;          // its fill stripe width (64-column tiles per block)
    bool rc_jump = false;  // the last recompute walk was the tie-to-tie walk (jump entries)
    int rc_every_used = 64;
};

namespace {

int check_ctx(ga_ctx* c) {
    if (!c) return fail(GA_E_ARG, "null context");
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return fail(GA_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    return GA_OK;
}

// Stripe geometry: T columns per lane (a stripe = one compute wave = 64*T columns).
// Blocked stripes pay the wave scan, the edge traffic and the control once per 64*T cells, but
// leave fewer stripes (waves) to fill the chip and lengthen each row's dependent chain.  A
// workgroup chains 4 waves (one per SIMD) when every stripe gets a wave that way, else 8.
void set_stripes(ga_ctx* c, int T_req, bool tb, bool full, int64_t ncols = -1) {
    const int64_t ncol = ncols < 0 ? c->n : ncols;  // a traceback band may cover a prefix of the columns
    const int64_t simds = 4 * (int64_t)c->num_cu;
    // register budget (no spills, see the code objects' vgpr_spill_count): the FULL debug output is
    // T == 1 only; traceback words T <= 2; score only T <= 8 with an int8 profile, 4 with int16
    const int cap = full ? 1 : tb ? 2 : (c->qbytes == 2 ? 4 : 8);
    int T = 1;
    if (T_req == 1 || T_req == 2 || T_req == 4 || T_req == 8) {
        T = std::min(T_req, cap);
    } else {
        // the widest stripes that still leave >= 1.5 waves per SIMD (measured: 1M columns score
        // only T = 8 > 4 > 2 > 1; 100k columns with traceback T = 1 > 2 > 4)
        for (int t = cap; t > 1; t /= 2)
            if ((ncol + 64 * t - 1) / (64 * t) * 2 >= 3 * simds) {
                T = t;
                break;
            }
    }
    // a slab with a right neighbour hands column n on: its last stripe must be whole (T == 1
    // takes the edge from any lane)
    while (T > 1 && c->col0 + c->n < c->n_global && c->n % (64 * T) != 0) T /= 2;
    c->T = T;
    c->nstripes = (int)((ncol + 64 * T - 1) / (64 * T));
    c->nwc = c->nwc_req == 4 || c->nwc_req == 8 ? c->nwc_req : c->nstripes <= 4 * c->num_cu ? 4 : 8;
    c->nslabs = (c->nstripes + c->nwc - 1) / c->nwc;
}

// Lane-skewed fill geometry: TD columns per lane, NWC compute waves per workgroup,
// every stripe resident at once (a stripe waits on its left neighbour only, so the whole chain must
// run concurrently).  The cost model is the measured step of tools/micro/lane_bench.hip (cycles per
// step per wave at one / two waves per SIMD, with the kernel's per-step LDS traffic and the DPP
// shift-register output) times the chain's length, m steps plus ~74 steps of skew per stripe.
// Returns false (row scan) when the profile table does not fit beside the rings.
bool lane_geometry(ga_ctx* c, int64_t ncol, int* qrows_out, bool tb, int force_T = 0, int force_N = 0,
                   int qrows_cap = 0) {
    if (c->qbytes != 1 || c->K > 32) return false;
    // Cycles per step per wave measured in the kernel (score only, 16-step sub-chunks; tools/lane_stamps.py,
    // tools/exp/lane_sub.sh, tools/exp/c4_pack.sh): one wave per SIMD (4-wave workgroups) 84 / 115 / 154 /
    // 239 at TD = 1 / 2 / 4 / 8; two waves per SIMD (8-wave workgroups) about 2.1x that per wave, the
    // partner's issue plus the chain coupling (C4: 243 ms against 207 for 1-wave rounds).
    static const double cyc1[4] = {84, 115, 154, 239};
    // workgroups per CU the residency check may count on (GA_LANE_WG_PER_CU, tuning: 2 needs an LDS floor
    // below 80 KB, GA_FILL_LDS_FLOOR)
    const int wpc = [c] {
        const char* e = c->knob("GA_LANE_WG_PER_CU");
        return e ? std::max(1, std::min(2, atoi(e))) : 1;
    }();
    int64_t cus = c->num_cu * wpc;
    // A slab whose edge another kernel (an RCCL receive or send) must move WHILE the fill runs: keep one CU
    // of every shader engine (8 CUs) free and every workgroup resident.  A kernel launched beside the fill
    // places each of its workgroups on a CU of one shader engine, round robin, and waits there: measured
    // (tools/exp/r3_cores.py), an RCCL-shaped kernel starts beside 224 fill workgroups on 256 CUs, not
    // beside 228.  Linked edges (ga_slab_link / _import: the fill stores them itself) need no room.
    const bool coresident = c->slab && ((c->col0 > 0 && !c->in_prog_ext) ||
                                        (c->col0 + c->n < c->n_global && !c->out_prog_ext));
    if (coresident) cus = c->num_cu - c->num_cu / 8;
    // Rounds: with 4-wave workgroups, one per CU, more stripes than 4 per CU run in rounds of workgroups.
    // A later round starts as the first finish, on left edges long written, so it runs uncoupled; the
    // chain then takes R*m + skew steps at the 1-wave step cost.  Not for a slab with a right neighbour
    // (its last stripe, in the last round, would hold the next GPU back by the earlier rounds).
    const bool right_nb = c->col0 + c->n < c->n_global;
    int bestT = 0, bestN = 0;
    double best = 0;
    for (int ti = 0; ti < 4; ti++) {
        const int T = 1 << ti;
        if (force_T ? force_T != T : c->lane_T_req && c->lane_T_req != T) continue;
        // traceback windows (register budget, ga_lane.hip lane_variant_ok): TD <= 4 with one-byte
        // words, <= 2 with two- and four-byte words (four-byte: 4 waves per workgroup)
        if (tb && T > (c->CB == 1 ? 4 : 2)) continue;
        // a slab with a right neighbour hands column n on: its last stripe must be whole
        if (right_nb && ncol % (64 * T) != 0) continue;
        const int64_t ns = (ncol + 64 * T - 1) / (64 * T);
        for (int nwc : {4, 8}) {
            if (force_N ? force_N != nwc : (c->nwc_req == 4 || c->nwc_req == 8) && nwc != c->nwc_req) continue;
            if (tb && c->CB == 4 && nwc == 8) continue;
            const int64_t rounds = (ns + nwc * cus - 1) / (nwc * cus);
            if (rounds > 1 && (nwc == 8 || right_nb || tb || coresident)) continue;  // 8-wave workgroups: all resident
            const double step = nwc == 4 ? cyc1[ti] : 2.1 * cyc1[ti];
            const double t = ((double)rounds * (double)c->m + 74.0 * (double)ns) * step;
            if (!bestT || t < best) {
                best = t;
                bestT = T;
                bestN = nwc;
            }
        }
    }
    if (!bestT) return false;
    // GA_LANE_QROWS caps the profile table (tuning: a smaller table lets two workgroups share a CU)
    const int qcap = [c] {
        const char* e = c->knob("GA_LANE_QROWS");
        return e ? atoi(e) : 4096;
    }();
    const size_t budget = 150 * 1024;
    int qr = std::max(256, std::min(4096, qrows_cap > 0 ? qrows_cap : qcap));
    while (qr > 256 && ga::fill_lane_lds_bytes(bestN, c->K, qr) > budget) qr >>= 1;
    if (ga::fill_lane_lds_bytes(bestN, c->K, qr) > budget || qr < bestN * 64 + 192) return false;
    c->T = bestT;
    c->nwc = bestN;
    c->nstripes = (int)((ncol + 64 * bestT - 1) / (64 * bestT));
    c->nslabs = (c->nstripes + c->nwc - 1) / c->nwc;
    *qrows_out = qr;
    return true;
}

int load_problem(ga_ctx* c, const uint8_t* a, int64_t m, const uint8_t* b_all, int64_t n_all, const ga_costs* cs,
                 const int32_t* row0, const int32_t* col0, int64_t cb, int64_t ce) {
    ProblemShape ps;
    std::string why;
    if (int r = check_problem(a, m, b_all, n_all, cs, row0, col0, cb, ce, ps, why)) return fail(r, why);
    const int K = cs->K;
    const int o = cs->gap_open;
    const int64_t big = ps.big;
    c->qbytes = ps.qbytes;
    c->CB = ps.CB;
    c->m = m;
    c->n = ce - cb;
    c->n_global = n_all;
    c->col0 = cb;
    c->K = K;
    c->o = o;
    c->big = (int)big;
    c->custom = row0 != nullptr || col0 != nullptr;
    c->gh_total = 0;  // GH(n) of the whole problem: the lean ramp's uniform-row-0 test (enqueue_fill), the cost
    for (int64_t j = 0; j < n_all; j++) c->gh_total += cs->gap_h[b_all[j]];
    c->gv_total = 0;  // GV(m): the cost's un-shift (cost = H'(m, n) + GV(m) + GH(n))
    for (int64_t i = 0; i < m; i++) c->gv_total += cs->gap_v[a[i]];
    // one stripe (64 columns) per compute wave; a workgroup (one per CU) chains 4 waves (one per
    // SIMD: the fastest rows) when every stripe gets a wave that way, else 8 (two per SIMD)
    set_stripes(c, c->T_req, false, false);
    c->h_a.assign(a, a + m);
    c->h_b.assign(b_all, b_all + n_all);
    HIPCHK(c->a.ensure(m));
    HIPCHK(c->b.ensure(n_all));
    HIPCHK(c->sub.ensure(sizeof(int) * K * K));
    HIPCHK(c->gh.ensure(sizeof(int) * K));
    HIPCHK(c->gv.ensure(sizeof(int) * K));
    HIPCHK(hipMemcpyAsync(c->a.p, a, m, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->b.p, b_all, n_all, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->sub.p, cs->sub, sizeof(int) * K * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->gh.p, cs->gap_h, sizeof(int) * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->gv.p, cs->gap_v, sizeof(int) * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c->bnd_row.ensure(sizeof(int) * 3 * (n_all + 1)));
    HIPCHK(c->bnd_col.ensure(sizeof(int) * 3 * (m + 1)));
    if (c->custom) {
        HIPCHK(hipMemcpyAsync(c->bnd_row.p, row0, sizeof(int) * 3 * (n_all + 1), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->bnd_col.p, col0, sizeof(int) * 3 * (m + 1), hipMemcpyHostToDevice, c->stream));
    }
    {
        // sub' = sub - gV - gH, read by the fill's IO wave into its LDS query profile
        std::vector<int> subp((size_t)K * K);
        for (int x = 0; x < K; x++)
            for (int y = 0; y < K; y++) subp[x * K + y] = cs->sub[x * K + y] - cs->gap_v[x] - cs->gap_h[y];
        HIPCHK(c->qp.ensure(sizeof(int) * K * K));
        HIPCHK(hipMemcpy(c->qp.p, subp.data(), sizeof(int) * K * K, hipMemcpyHostToDevice));
        // query-profile ring: as many rows as fit 64 KB (at least 128)
        c->qrows = 1024;
        while (c->qrows > 128 && (size_t)K * c->qrows * c->qbytes > 64 * 1024) c->qrows >>= 1;
        if (std::max(ga::fill_lds_bytes(8, c->qbytes, K, c->qrows, 8192), ga::fill_diag_lds_bytes(8, c->qbytes, K, c->qrows)) >
            160 * 1024)
            return fail(GA_E_RANGE, "alphabet too large for the LDS query profile");
    }
    HIPCHK(c->GVp.ensure(sizeof(int) * (m + 1)));
    HIPCHK(c->bscr.ensure(sizeof(int) * ga::boundary_scratch_ints((int)m, (int)n_all)));
    HIPCHK(c->GHp.ensure(sizeof(int) * (n_all + 1)));
    HIPCHK(c->top.ensure(sizeof(int2) * (n_all + 1)));
    HIPCHK(c->left.ensure(sizeof(int2) * (m + 1)));
    HIPCHK(c->meta.ensure(sizeof(int) * 8));
    HIPCHK(c->out_last.ensure(sizeof(int) * 4));
    HIPCHK(c->result.ensure(sizeof(int) * 16));
    HIPCHK(c->ops.ensure(m + n_all + 1024));  // 2-bit levels; the walk flushes whole 128-byte blocks
    HIPCHK(c->rng.ensure(sizeof(uint32_t) * (m + n_all + 2 + 64)));  // + the walk's entry look-ahead (SLD)
    HIPCHK(hipStreamSynchronize(c->stream));
    c->loaded = true;
    c->filled_tb = false;
    return GA_OK;
}

// Device memory a buffer may take: hipMemGetInfo's free bytes plus `held` (what the context's own buffers being
// resized already hold), less a 2 GB margin; GA_DEV_AVAIL_MB caps it (tests: forces the fallbacks).
int64_t dev_avail_bytes(ga_ctx* c, int64_t held) {
    int64_t avail = INT64_MAX / 4;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) avail = (int64_t)fr + held - ((int64_t)2 << 30);
    if (const char* e = c->knob("GA_DEV_AVAIL_MB")) avail = std::min<int64_t>(avail, atoll(e) << 20);
    return std::max<int64_t>(avail, 0);
}

// A band of rows of the whole problem (banded traceback): rows r0+1 .. r0+mb, its
// top row from a checkpoint (nullptr: row 0), no boundary pass; or the checkpointing pass itself.
struct Band {
    int64_t r0 = 0, mb = 0;
    int64_t nc = 0;             // columns 1..nc only (0: all): the walk enters the band at column nc
    const int2* top = nullptr;  // (H', h2') of row r0, [n+1] (column 0 = the left edge's corner)
    bool band = false;          // fill rows r0+1 .. r0+mb only (the boundary is already computed)
    // the recompute walk's score fill: the lane kernel with its checkpoints (every stripe's
    // right edge, the staircase lane states every rc_every steps) into ctx->colck / ctx->stck
    bool rc = false;
    int rc_every = 0;           // 0: chosen with the stripes' geometry (enqueue_fill)
    int2* ckpt = nullptr;       // checkpointing pass: where rows ckpt_rows, 2*ckpt_rows, ... go
    int ckpt_rows = 0;
    // pipelined alignments (align_many): a fill with buffers and a stream of its own, so that two
    // fills can run at once; the boundary is computed by the first fill only
    DevBuf* tbuf = nullptr;     // traceback words instead of ctx->tb
    DevBuf* hbuf = nullptr;     // workgroup hand-off edges instead of ctx->hand
    DevBuf* fbuf = nullptr;     // ticket / abort words instead of ctx->flags
    DevBuf* obuf = nullptr;     // H'(m, n) instead of ctx->out_last
    hipStream_t stream = nullptr;
    bool skip_boundary = false;
    // a traceback fill through the lane-skewed kernel at this geometry (TD columns per lane, NWC
    // compute waves; 0: the usual choice): the pipeline's narrow fills (align_many)
    int lane_td = 0, lane_nwc = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // fill timing events instead of ctx->ev[0 / 1]
    // boundary arrays instead of the context's (a pipeline slot's own make_dp_array output)
    DevBuf *GVp = nullptr, *GHp = nullptr, *top_b = nullptr, *left = nullptr, *bnd_row = nullptr, *bnd_col = nullptr,
           *meta = nullptr, *bscr = nullptr;
};

// Enqueue boundary + query profile + fill.  Does not synchronise.
#ifdef GA_EXPERIMENTS
constexpr bool kRcJumpDefault = false;  // the tie-to-tie walk unless GA_RC_JUMP says otherwise
#endif
// the recompute walk's block cache: the word walk's, and (experiments build) the tie-to-tie walk's entries
inline size_t rc_cache_bytes(bool jump, int TD, int CB) {
    // (+ one 64-column stripe of slack: a loader reads whole 1 KiB runs)
    return jump ? (size_t)ga::RC_CACHE_I * ga::RC_CACHE_S * 4 * TD * 6144 + 65536
                : (size_t)ga::RC_CACHE_I * ga::RC_CACHE_S * TD * 64 * 64 * CB + (size_t)64 * 64 * 4 * 4;
}
// whether the tie-to-tie walk may run (experiments build, GA_RC_JUMP): the checkpoint sizing then budgets its cache
inline bool rc_jump_requested(const ga_ctx* c) {
#ifdef GA_EXPERIMENTS
    const char* e = c->xknob("GA_RC_JUMP");
    return e ? atoi(e) != 0 : kRcJumpDefault;
#else
    (void)c;
    return false;
#endif
}

int enqueue_fill(ga_ctx* c, int32_t flags, const Band& bd = Band()) {
    int every = bd.rc_every > 0 ? bd.rc_every : 64;  // the recompute fill's checkpoint spacing (chosen below)
    if (!c->loaded) return fail(GA_E_STATE, "no problem loaded");
    const bool tb = (flags & (GA_FILL_TRACEBACK | GA_FILL_FULL)) != 0;
    const bool full = (flags & GA_FILL_FULL) != 0;
    const int64_t m = bd.band ? bd.mb : c->m, n = bd.band && bd.nc > 0 ? bd.nc : c->n;
    // 16-row chunks; CB 16-byte words per lane per chunk (ga_device.h)
    c->TC = (int)((m + ga::FROWS - 1) / ga::FROWS) * c->CB;
    // score only: the anti-diagonal kernel (64-column stripes) when asked for and its profile
    // ring is deep enough for a workgroup's skew (8 waves x 64 steps)
    // (its query-profile ring deeper than a workgroup's skew: NWC stripes x 64*TD steps)
    int qrows = c->qrows;
    c->diag = false;
    c->lane = false;
    // score only: the lane-skewed kernel when its chain's skew (~74 steps per stripe)
    // is short against the m rows every stripe walks (measured: 1M x 125k 60 ms against 107 for the row
    // scan, C4 244 against 312; 100k x 100k, whose 782 stripes add 58k steps of skew, 13.5 against 12.6)
    if (bd.rc) {
        if (tb || full || !lane_geometry(c, n, &qrows, false)) return fail(GA_E_STATE, "recompute fill needs the lane kernel");
        // the checkpointing variant runs 16-step sub-chunks (8 waves at TD = 8 would take 8-step ones)
        if (c->nwc == 8 && c->T == 8 && !lane_geometry(c, n, &qrows, false, 8, 4)) return fail(GA_E_STATE, "recompute fill geometry");
        // the recompute workers stage a block's codes in LDS (64*TD columns x the checkpoint spacing): at
        // wide stripes and wide spacings (C4: TD 8, every 256 steps, 219 KB) that exceeds the CU's LDS, so
        // the stripes narrow until a worker fits beside the walk's 128 KB torus budget
        constexpr int kRcLds = 256 * 256 * 2;  // the walk's torus (ga_walk.h TP x TP u16): the launch's dynamic LDS
        // Stripes of at most 4 columns per lane (unless GA_LANE_COLS_PER_LANE asks): a block is 64 rows of one stripe, and the walk reads ~1-2 of
        // its TD tiles, so wider blocks starve the walk (C4 on one GPU at TD 8: fill 226 ms, walk 160 ms;
        // at TD 4: 284 + 90 ms, tools/exp/r3b_c4tb3.sh, r3b_c4rc.py)
        // and 4 where the geometry model chose fewer (round 4, the lean sub-chunk): fewer, wider stripes shorten
        // the ramp as much as their slower step lengthens the rows, and the walk's blocks come cheaper (C3: fill
        // 9.69 -> 9.81 ms, walk 5.72 -> 5.42; C5 3.92 against 6.3 ms at TD = 1; tools/r4_td.sh).
        // Round 6: with the lean ramp (the first 64 steps no longer masked) and the cone-shaped recompute window
        // below, 2 columns per lane win for small alphabets whose stripes all run at once (one workgroup of four per
        // CU): C3 fill 7.61 -> 6.83 ms, walk 5.18 -> 5.03 (cone 2; 5.65 with the round-5 window), call 12.98 ->
        // 12.09; C2 1.42 -> 1.30.  The protein fill does not (C5 at TD 2: fill 1.73 -> 1.91 ms), so K > 8 keeps 4
        // (tools/exp/r6/check5.sh, check6.sh, rc_diag.py).  Behind the option GA_RC_NARROW=1 until the GPU suite has
        // run with it as the default and the roofline profiles are of that variant.
        if (!c->lane_T_req) {
            const char* nw = c->knob("GA_RC_NARROW");
            const bool td2 = nw && atoi(nw) && !c->slab && c->K <= 8 && (n + 127) / 128 <= 4 * (int64_t)c->num_cu;
            if (td2 && lane_geometry(c, n, &qrows, false, 2, 4)) {
            } else if (c->T > 4) {
                if (!lane_geometry(c, n, &qrows, false, 4, 4)) return fail(GA_E_STATE, "recompute fill geometry");
            } else if (c->T < 4) {
                (void)lane_geometry(c, n, &qrows, false, 4, 4);
            }
        }
        // The checkpoint spacing, with the stripes' geometry known: the smallest (<= 4096 steps) whose states
        // fit the memory budget (default 96 GB of the 288: C4 on one GPU, TD 4, takes 128 steps, 78 GB; 64
        // would take 156 GB and walks no faster) and whose worker fits LDS; GA_RC_EVERY fixes it (the stripes
        // narrow if it must)
        // The budget is also capped by the device memory free for it: what hipMemGetInfo reports plus
        // what this context's checkpoint buffers already hold, less the right-edge columns (8 B per row per
        // stripe), the walk's tile cache and a 2 GB margin.  A problem whose checkpoints still do not fit returns
        // GA_E_NOMEM, and ga_problem_align takes the banded traceback instead.
        int64_t budget = (int64_t)96 << 30;
        if (const char* e = c->knob("GA_RC_BUDGET_MB")) budget = atoll(e) << 20;
        const int64_t dev_avail = dev_avail_bytes(c, (int64_t)c->stck.cap + (int64_t)c->colck.cap + (int64_t)c->rc_tb.cap);
        auto ck_bytes = [&](int e) {
            const int64_t nck = std::max<int64_t>((m - 1) / e, 1);
            return nck * c->nstripes * (c->T + 1) * 512;
        };
        // (the walk's block cache as the walk that will run sizes it: ADVICE r5, the jump cache is ~6x the word one)
        auto other_bytes = [&]() {
            return (int64_t)c->nstripes * (m + 1) * 8 +
                   (int64_t)rc_cache_bytes(rc_jump_requested(c) && c->T <= 4, c->T, c->CB) +
                   ((int64_t)64 << 20);
        };
        auto fits = [&](int e) {
            return ck_bytes(e) <= std::min(budget, dev_avail - other_bytes()) &&
                   1024 + ga::rc_worker_bytes(c->T, c->CB, e) <= kRcLds;
        };
        for (;;) {
            if (bd.rc_every > 0) every = bd.rc_every;
            else
                for (every = 64; every < 4096 && !fits(every); every *= 2) {}
            if (1024 + ga::rc_worker_bytes(c->T, c->CB, every) <= kRcLds) break;
            if (c->T == 1) {
                // no spacing fits both: memory if the densest one fits LDS, else LDS
                if (1024 + ga::rc_worker_bytes(1, c->CB, 64) <= kRcLds)
                    return fail(GA_E_NOMEM, "recompute walk: the checkpoints do not fit the budget / free device memory");
                return fail(GA_E_RANGE, "recompute walk: a block's codes do not fit LDS");
            }
            if (!lane_geometry(c, n, &qrows, false, c->T / 2, 4)) return fail(GA_E_STATE, "recompute fill geometry");
        }
        if (ck_bytes(every) > std::min(budget, dev_avail - other_bytes()))
            return fail(GA_E_NOMEM, "recompute walk: the checkpoints do not fit the budget / free device memory");
        c->rc_every_used = every;
        c->lane = true;
    } else if (bd.lane_td > 0 && tb && !full && bd.ckpt == nullptr)
        c->lane = lane_geometry(c, n, &qrows, tb, bd.lane_td, bd.lane_nwc, 2048);
    else if (!full && (bd.ckpt == nullptr || !tb) && (c->diag_req == 3 || (c->diag_req == 0 && !tb)) &&
             lane_geometry(c, n, &qrows, tb) && (c->diag_req == 3 || 4 * 74 * (int64_t)c->nstripes <= m))
        c->lane = true;
    // automatic: score-only fills of tall problems on one GPU (m >= 4 n, <= 8 stripes per CU).
    // Measured (profiles/r01/diag_sweep.txt): 1M x 125k 80 ms (TD = 1) against 107 ms for the row
    // scan, 1M x 250k 126 ms (TD = 2) against 141 ms; the row scan wins on square shapes (C4 313 ms
    // against 400 ms), where the anti-diagonal skew of 64 steps per stripe costs more.  Not for a
    // slab of a multi-GPU fill: there the next rank starts when this one's last stripe does, and
    // that start (the ramp) is ~15 ms for the anti-diagonal fill against ~3 ms for the row scan.
    const int auto_td = (n + 63) / 64 <= 8 * (int64_t)c->num_cu ? 1 : 2;
    const bool auto_diag = c->diag_req == 0 && !tb && !bd.band && !c->slab && m >= 4 * n &&
                           (n + 64 * auto_td - 1) / (64 * auto_td) <= 8 * (int64_t)c->num_cu;
    if (!c->lane && (!tb || (full && c->qbytes == 1)) && (c->diag_req == 2 || auto_diag) && bd.ckpt == nullptr) {
        int td = full ? std::min(std::max(c->diag_T_req, 1), 2)
                      : c->diag_T_req == 1 || c->diag_T_req == 2 || c->diag_T_req == 4 ? c->diag_T_req
                      : auto_diag ? auto_td : 1;
        if (c->qbytes == 2) td = std::min(td, 2);  // int16 profiles at TD = 4 spill
        set_stripes(c, td, false, false, n);
        if (full) {  // the debug FULL variant is built for 4 compute waves
            c->nwc = 4;
            c->nslabs = (c->nstripes + 3) / 4;
        }
        qrows = 8192;
        while (qrows > 128 && (size_t)c->K * (qrows + 16) * c->qbytes > 64 * 1024) qrows >>= 1;
        c->diag = qrows >= c->nwc * (64 * c->T + 16) + 64 * c->T + 64;
    }
    if (!c->diag && !c->lane) {
        qrows = c->qrows;
        set_stripes(c, c->T_req, tb, full, n);
    }
    // traceback words cover T 64-column stripes per fill stripe
    DevBuf& tbb = bd.tbuf ? *bd.tbuf : c->tb;
    DevBuf& hb = bd.hbuf ? *bd.hbuf : c->hand;
    DevBuf& fb = bd.fbuf ? *bd.fbuf : c->flags;
    DevBuf& ob = bd.obuf ? *bd.obuf : c->out_last;
    hipStream_t st = bd.stream ? bd.stream : c->stream;
    HIPCHK(ob.ensure(sizeof(int) * 4));
    if (tb) HIPCHK(tbb.ensure((size_t)c->nstripes * c->T * c->TC * 1024));
    HIPCHK(hb.ensure(sizeof(int2) * (size_t)c->nslabs * (m + 1)));
    // workgroup hand-off rows read by a successor start as ga::HAND_SENT (bytes 0x80)
    if (c->nslabs > 1)
        HIPCHK(hipMemsetAsync(hb.p, 0x80, sizeof(int2) * (size_t)(c->nslabs - 1) * (m + 1), st));
    HIPCHK(fb.ensure(sizeof(unsigned) * 16));
    if (full) {
        if ((m + 1) * (n + 1) > (int64_t)64 << 20) return fail(GA_E_RANGE, "GA_FILL_FULL is for small problems");
        HIPCHK(c->full.ensure(sizeof(int) * 3 * (m + 1) * (n + 1)));
    }
    unsigned* fl = fb.as<unsigned>();
    // flags layout: [0] ticket, [1] abort
    HIPCHK(hipMemsetAsync(fl, 0, sizeof(unsigned) * 16, st));
    DevBuf& bGVp = bd.GVp ? *bd.GVp : c->GVp;
    DevBuf& bGHp = bd.GHp ? *bd.GHp : c->GHp;
    DevBuf& btop = bd.top_b ? *bd.top_b : c->top;
    DevBuf& bleft = bd.left ? *bd.left : c->left;
    DevBuf& brow = bd.bnd_row ? *bd.bnd_row : c->bnd_row;
    DevBuf& bcol = bd.bnd_col ? *bd.bnd_col : c->bnd_col;
    DevBuf& bmeta = bd.meta ? *bd.meta : c->meta;
    DevBuf& bscr = bd.bscr ? *bd.bscr : c->bscr;
    if (!bd.band && !bd.skip_boundary)
        ga::launch_boundary(st, c->a.as<uint8_t>(), (int)m, c->b.as<uint8_t>(), (int)c->n_global,
                            c->gh.as<int>(), c->gv.as<int>(), c->o, c->big, bGVp.as<int>(), bGHp.as<int>(),
                            btop.as<int2>(), bleft.as<int2>(), brow.as<int>(), bcol.as<int>(),
                            bmeta.as<int>(), c->custom, bscr.as<int>());
    ga::FillArgs p{};
    p.a = c->a.as<uint8_t>() + bd.r0;
    p.ckpt = bd.ckpt;
    p.ckpt_rows = bd.ckpt_rows;
    p.colck = nullptr;
    p.stck = nullptr;
    // one round of lane workgroups (every stripe resident): the chain's lag counts, read edges late
    p.late = c->lane && c->nslabs <= c->num_cu ? 1 : 0;
    if (const char* e = c->knob("GA_LANE_LATE")) p.late = atoi(e);
    // chain neighbours on one XCD (ga_lane.hip lane_slab; experiments build only): measured no faster, since ticket
    // order already keeps 165 of C3's 195 cross-workgroup links on one XCD (r5: 188 with the map; C3 fill 9.43 ->
    // 9.46 ms, tools/exp/r5/xcd.sh).  Only for one round of workgroups that runs alone (a pipeline's fills share
    // the device; a fill that finds its workgroups not all resident falls back to ticket order after ~40 us)
    p.xcd_map = 0;
    if (const char* e = c->xknob("GA_LANE_XCD")) p.xcd_map = c->lane && c->nslabs <= c->num_cu && bd.stream == nullptr ? atoi(e) : 0;
    p.hand_direct = 0;  // measured: C4 210 ms against 221 with the direct hand-off, 1M x 125k 52.5 against 56 (r3_c4.log)
    if (const char* e = c->knob("GA_LANE_DIRECT")) p.hand_direct = atoi(e);
    p.stck_every = every;
    p.stck_shift = 0;
    while ((1 << p.stck_shift) < every) p.stck_shift++;
    {
        const char* e = c->knob("GA_FILL_LDS_FLOOR");
        p.lds_floor = e ? atoi(e) : -1;
        e = c->knob("GA_LANE_SUB");
        p.lane_sub = e ? atoi(e) : -1;
        e = c->knob("GA_LANE_TB_SUB");
        p.lane_tb_sub = e ? atoi(e) : -1;
        e = c->knob("GA_LANE_ASM");
        p.asm_step = e ? atoi(e) : 1;
        e = c->xknob("GA_LANE_IOPRIO");
        p.io_prio = e ? atoi(e) : 0;
        e = c->xknob("GA_LANE_HANDSCOPE");
        p.hand_scope = e ? atoi(e) : 0;
        e = c->knob("GA_LANE_POLLWIN");
        p.poll_win = e ? std::min(std::max(atoi(e), 0), 192) : 0;
        e = c->knob("GA_LANE_OUTWAVE");
        p.out_wave = e ? atoi(e) : 1;
    }
    if (bd.rc) {
        const int64_t nck = std::max<int64_t>((m - 1) / every, 1);
        // An allocation that fails (the size check above passed, but the device's free memory moved) releases every
        // recompute buffer before GA_E_NOMEM, so the fallback (ga_problem_align: banded / stored words) sizes
        // itself with that memory free.  The boundary pass and the memsets enqueued above are harmless: the
        // fallback's own fill enqueues them again behind them on the same stream.  GA_RC_FAIL_ALLOC=1 (tests)
        // fails the second allocation after the first succeeded.
        const bool fail_test = c->knob("GA_RC_FAIL_ALLOC") && atoi(c->knob("GA_RC_FAIL_ALLOC")) == 1;
        int nb = 0;
        for (auto [buf, bytes] : {std::pair<DevBuf*, size_t>{&c->colck, sizeof(int2) * (size_t)c->nstripes * (m + 1 + ga::COLCK_PAD)},
                                  {&c->stck, sizeof(int2) * (size_t)nck * c->nstripes * (c->T + 1) * 64}}) {
            hipError_t e = buf->ensure(bytes);
            if (e == hipSuccess && fail_test && nb == 1) e = hipErrorOutOfMemory;
            nb++;
            if (e != hipSuccess) {
                (void)hipGetLastError();
                c->colck.release();
                c->stck.release();
                c->rc_tb.release();
                return fail(e == hipErrorOutOfMemory ? GA_E_NOMEM : GA_E_HIP,
                            std::string("recompute checkpoints: ") + hipGetErrorString(e));
            }
        }
        p.colck = c->colck.as<int2>();
        p.stck = c->stck.as<int2>();
    }
    p.subp = c->qp.as<int>();
    p.K = c->K;
    p.b = c->b.as<uint8_t>() + c->col0;
    p.top = (bd.top ? bd.top : btop.as<int2>()) + c->col0;
    if (c->slab && c->col0 > 0) {
        p.left = c->halo_in_ext ? c->halo_in_ext : c->halo_in.as<int2>();
        p.left_prog = c->in_prog_ext ? c->in_prog_ext : c->prog_dev;  // [0]: halo_in rows
    } else {
        p.left = bleft.as<int2>() + bd.r0;
        p.left_prog = nullptr;
    }
    p.hand = hb.as<int2>();
    p.ticket = fl;
    p.abort_word = fl + 1;
    p.tb = tb ? tbb.as<uint8_t>() : nullptr;
    p.out_last = ob.as<int>();
    p.edge_prog = c->slab ? (c->out_prog_ext ? c->out_prog_ext : c->prog_dev + 1) : nullptr;  // [1]: halo_out rows
    p.edge_out = c->slab ? c->halo_out_ext : nullptr;
    p.full = full ? c->full.as<int>() : nullptr;
    p.m = (int)m;
    p.n = (int)n;
    p.o = c->o;
    p.nstripes = c->nstripes;
    p.nslabs = c->nslabs;
    p.TC = c->TC;
    p.nwc = c->nwc;
    p.qrows = qrows;
    p.cols_per_lane = c->T;
    p.spin_limit = 1u << 26;        // ~seconds: only a broken hand-off can reach it
    p.halo_spin_limit = 1u << 30;  // waiting on another GPU may take long (~30 s)
    if (const char* e = c->knob("GA_HALO_SPIN_LIMIT")) p.halo_spin_limit = (unsigned)std::max(1L, atol(e));  // (tests)
    // a slab with a left neighbour: every wait of its fill is, in the end, a wait for that halo
    if (c->slab && c->col0 > 0) p.spin_limit = std::max(p.spin_limit, p.halo_spin_limit);
    if (c->dbg_on) HIPCHK(c->dbg.ensure(sizeof(unsigned long long) * ga::LK_DBG_WORDS * c->nstripes));
    if (c->dbg_on) HIPCHK(hipMemsetAsync(c->dbg.p, 0, sizeof(unsigned long long) * ga::LK_DBG_WORDS * c->nstripes, st));
    p.dbg = c->dbg_on ? c->dbg.as<unsigned long long>() : nullptr;
    // the lane fill's query profile, built on the fill's stream just before it (K x (m + 4) dwords: C5 1.9 MB, a few us).
    // Fills of one problem in flight on other streams (align_many) rewrite it with the same values.
    // the lean ramp (ga_lane.hip lean0): row 0 is the reference's boundary and uniform in the shifted domain (H' = o,
    // h2' = 2o in every column: 2o + GH(n) <= big); GA_LANE_LEAN0=0 keeps the masked ramp (A/B)
    {
        const char* e = c->knob("GA_LANE_LEAN0");
        p.lean0 = (e ? atoi(e) : 1) && c->lane && !c->custom && bd.top == nullptr && !bd.band &&
                  2 * (int64_t)c->o + c->gh_total <= (int64_t)c->big;
    }
    p.qprof = nullptr;
    if (c->lane && !c->xknob("GA_LANE_QPROF_WAVE")) {  // (experiments build: the profile wave builds it, for A/B)
        HIPCHK(c->qprof.ensure(sizeof(uint32_t) * (size_t)c->K * (size_t)(m + 4)));
        ga::launch_lane_qprof(st, p.a, (int)m, p.subp, c->K, c->qprof.as<uint32_t>());
        p.qprof = c->qprof.as<uint32_t>();
    }
    HIPCHK(hipEventRecord(bd.ev0 ? bd.ev0 : c->ev[0], st));
    if (c->lane) ga::launch_fill_lane(st, p, c->CB);
    else if (c->diag) ga::launch_fill_diag(st, p, c->qbytes, full);
    else ga::launch_fill(st, p, c->CB, c->qbytes, tb, full);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(bd.ev1 ? bd.ev1 : c->ev[1], st));
    c->filled_tb = tb;
    return GA_OK;
}

int finish_fill(ga_ctx* c, int64_t* cost_out, int32_t* full_out) {
    int last[4] = {0, 0, 0, 0}, meta[2] = {0, 0};
    unsigned abort_word = 0;
    HIPCHK(hipMemcpyAsync(last, c->out_last.p, sizeof(int) * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(meta, c->meta.p, sizeof(int) * 2, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&abort_word, c->flags.as<unsigned>() + 1, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipEventElapsedTime(&c->fill_ms, c->ev[0], c->ev[1]));
    if (abort_word) return fail(GA_E_TIMEOUT, "fill kernel hand-off wait timed out");
    c->GV_m = meta[0];
    // un-shift: cost = H'(m, n) + GV(m) + GH(column)
    int64_t gh_end = 0;
    {
        int v = 0;
        HIPCHK(hipMemcpy(&v, c->GHp.as<int>() + c->col0 + c->n, sizeof(int), hipMemcpyDeviceToHost));
        gh_end = v;
    }
    if (cost_out) *cost_out = (int64_t)last[0] + c->GV_m + gh_end;
    if (full_out) {
        const int64_t m = c->m, n = c->n, W = n + 1;
        std::vector<int> GV(m + 1), GH(n + 1);
        HIPCHK(hipMemcpy(GV.data(), c->GVp.p, sizeof(int) * (m + 1), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(GH.data(), c->GHp.p, sizeof(int) * (n + 1), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(full_out, c->full.p, sizeof(int) * 3 * (m + 1) * W, hipMemcpyDeviceToHost));
        std::vector<int> br(3 * (n + 1)), bc(3 * (m + 1));
        HIPCHK(hipMemcpy(br.data(), c->bnd_row.p, sizeof(int) * br.size(), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(bc.data(), c->bnd_col.p, sizeof(int) * bc.size(), hipMemcpyDeviceToHost));
        for (int64_t i = 0; i <= m; i++)
            for (int64_t j = 0; j <= n; j++) {
                int* f = full_out + 3 * (i * W + j);
                if (i == 0) { f[0] = br[3 * j]; f[1] = br[3 * j + 1]; f[2] = br[3 * j + 2]; }
                else if (j == 0) { f[0] = bc[3 * i]; f[1] = bc[3 * i + 1]; f[2] = bc[3 * i + 2]; }
                else {
                    const int sh = GV[i] + GH[j];
                    f[0] += sh; f[1] += sh; f[2] += sh;
                }
            }
    }
    return GA_OK;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Walk state between slab walks (the C ABI's ga_walk_state without the padding rules).
struct WalkStart {
    int64_t i, j, D, h;  // j: global column
    int L, first;
};

// Where a walk reads its words and table and leaves its levels / result, on which stream.
struct WalkBufs {
    const uint8_t* tb;
    uint32_t* rng;
    uint32_t* ops;
    int* result;
    hipStream_t stream;
    hipEvent_t ev0, ev1;
    const int* bnd_row = nullptr;  // the boundary triples (nullptr: the context's)
    const int* bnd_col = nullptr;
    unsigned* ops_prog = nullptr;  // WalkArgs::ops_prog (ops then in pinned host memory)
};
WalkBufs ctx_walk_bufs(ga_ctx* c) {
    return WalkBufs{c->tb.as<uint8_t>(), c->rng.as<uint32_t>(), c->ops.as<uint32_t>(), c->result.as<int>(), c->stream,
                    c->ev[2], c->ev[3]};
}

ga::WalkArgs walk_args(ga_ctx* c, int64_t ntab, const WalkStart& st, int64_t r0, int64_t mb, bool vhandoff,
                       const WalkBufs& wb) {
    ga::WalkArgs w{};
    w.tb = wb.tb;
    w.CB = c->CB;
    w.TC = c->TC;
    w.a = c->a.as<uint8_t>() + r0;
    w.b = c->b.as<uint8_t>() + c->col0;
    w.bnd_row = (wb.bnd_row ? wb.bnd_row : c->bnd_row.as<int>()) + 3 * c->col0;
    w.bnd_col = (wb.bnd_col ? wb.bnd_col : c->bnd_col.as<int>()) + 3 * r0;
    w.rng = wb.rng;
    w.nrng = (long long)ntab;
    w.m = (int)(mb >= 0 ? mb : c->m);
    w.n = (int)c->n;
    w.o = c->o;
    w.i0 = (int)(st.i - r0);
    w.vhandoff = vhandoff ? 1 : 0;
    w.j0 = (int)(st.j - c->col0);
    w.L0 = st.L;
    w.first0 = st.first;
    w.D0 = (int)st.D;
    w.h0 = (int)st.h;
    w.handoff = c->col0 > 0;
    w.maxh = (int)(c->m + c->n_global);
    {
        // the loaders leave the 4x4 tile block's far off-diagonal corners: 28 % fewer
        // speculative tile loads, C3 walk 6.87 -> 6.71 ms alone and 7.74 -> 7.4 ms in the pipeline, C5
        // 1.45 -> 1.27 ms (tools/exp/walk_skip.sh); GA_WALK_SKIP_CORNERS = 0 / 2 / 3 for none / more
        const char* e = c->xknob("GA_WALK_SKIP_CORNERS");
        w.skip_corners = e ? atoi(e) : 1;
        // 14 loader waves (the L2 prefetcher's and the idle wave's too): tile waits at C3 469 -> 186 us
        // alone, 921 -> 413 us in the pipeline, walk 6.81 -> 6.52 ms alone, C5 1.28 -> 1.15 ms
        // (tools/exp/walk_loaders.sh); GA_WALK_LOADERS = 12 / 13 for the former roles
        const char* nl = c->xknob("GA_WALK_LOADERS");
        w.nloaders = nl ? atoi(nl) : 14;
    }
    w.ops = wb.ops;
    w.ops_prog = wb.ops_prog;
    w.result = wb.result;
    w.dbg = nullptr;
    return w;
}

int run_walk(ga_ctx* c, const uint32_t* tab, int64_t ntab, const WalkStart& st, int64_t r0 = 0, int64_t mb = -1,
             bool vhandoff = false, bool upload_tab = true, const WalkBufs* wbp = nullptr) {
    const WalkBufs wb = wbp ? *wbp : ctx_walk_bufs(c);
    if (upload_tab) HIPCHK(hipMemcpyAsync(wb.rng, tab, sizeof(uint32_t) * ntab, hipMemcpyHostToDevice, wb.stream));
    ga::WalkArgs w = walk_args(c, ntab, st, r0, mb, vhandoff, wb);
    if (c->dbg_on) {
        HIPCHK(c->wdbg.ensure(sizeof(unsigned) * 4 * 8192));
        HIPCHK(hipMemsetAsync(c->wdbg.p, 0xff, sizeof(unsigned) * 4 * 8192, wb.stream));
    }
    w.dbg = c->dbg_on ? c->wdbg.as<unsigned>() : nullptr;
    HIPCHK(hipEventRecord(wb.ev0, wb.stream));
    ga::launch_walk(wb.stream, w);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(wb.ev1, wb.stream));
    return GA_OK;
}

inline int64_t pywrap(int64_t k, int64_t L) { return k < 0 ? k + L : k; }

// Wait for the walk; decode the levels of dispatches [st.D, D_end) into alignment columns in walk
// order starting at (st.i, st.j) (global columns).  Returns the end state through `st` and `reason`.
int decode_segment(ga_ctx* c, const int* res, WalkStart& st, int& reason, const char* a_chr, const char* b_chr,
                   char* oa, char* om, char* ob, int64_t cap, int64_t& len, const WalkBufs& wb, bool synced,
                   const uint32_t* host_ops = nullptr);

int walk_segment(ga_ctx* c, WalkStart& st, int& reason, const char* a_chr, const char* b_chr, char* oa, char* om,
                 char* ob, int64_t cap, int64_t& len, const WalkBufs* wbp = nullptr) {
    const WalkBufs wb = wbp ? *wbp : ctx_walk_bufs(c);
    int res[16];
    HIPCHK(hipMemcpyAsync(res, wb.result, sizeof(int) * 16, hipMemcpyDeviceToHost, wb.stream));
    HIPCHK(hipStreamSynchronize(wb.stream));
    return decode_segment(c, res, st, reason, a_chr, b_chr, oa, om, ob, cap, len, wb, false);
}

// The alignment columns of a finished walk (its result words already read): levels of dispatches
// [st.D, res[0]) decoded in walk order starting at (st.i, st.j).  synced: the walk is known to be
// complete, so its levels are read with a plain copy instead of on its stream (which may already
// hold the next walk).
int decode_segment(ga_ctx* c, const int* res, WalkStart& st, int& reason, const char* a_chr, const char* b_chr,
                   char* oa, char* om, char* ob, int64_t cap, int64_t& len, const WalkBufs& wb, bool synced,
                   const uint32_t* host_ops) {
    c->walk_waits = res[4];
    c->walk_tiles = res[5];
    c->walk_t_tile = res[6];
    c->walk_t_ring = res[7];
    c->walk_t_total = res[8];
    c->walk_c_total = res[9];
    c->walk_load_ticks = res[10];
    c->walk_load_count = res[11];
    for (int q = 0; q < 3; q++) c->walk_jump_diag[q] = res[12 + q];
    if (!synced) HIPCHK(hipEventElapsedTime(&c->walk_ms, wb.ev0, wb.ev1));
    const int64_t D0 = st.D, D1 = res[0];
    reason = res[3];
    // levels are packed 2 bits per dispatch, dispatch k at bits 30 - 2*(k & 15) of u32 word k >> 4
    const int64_t w0 = D0 >> 4, w1 = (D1 + 15) >> 4;
    std::vector<uint32_t> ops((size_t)std::max<int64_t>(w1 - w0, 0));
    if (host_ops) {  // the levels in pinned host memory (the walk chain writes them there)
        if (D1 > D0) std::memcpy(ops.data(), host_ops + w0, ops.size() * sizeof(uint32_t));
    } else if (synced) {
        if (D1 > D0) HIPCHK(hipMemcpy(ops.data(), wb.ops + w0, ops.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    } else {
        if (D1 > D0)
            HIPCHK(hipMemcpyAsync(ops.data(), wb.ops + w0, ops.size() * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                  wb.stream));
        HIPCHK(hipStreamSynchronize(wb.stream));
    }
    const int64_t m = c->m, n = c->n_global;
    int64_t i = st.i, j = st.j;
    int L = st.L;
    len = 0;
    auto put = [&](char x, char y, char z) {
        if (len < cap) { oa[len] = x; om[len] = y; ob[len] = z; }
        len++;
    };
    if (reason != 4) {
        for (int64_t k = D0; k < D1; k++) {
            const char ca = a_chr[pywrap(i - 1, m)], cbb = b_chr[pywrap(j - 1, n)];
            const unsigned lv = (ops[(k >> 4) - w0] >> (30 - 2 * (k & 15))) & 3u;
            if (lv == 0) { put(ca, ca == cbb ? '|' : '*', cbb); i--; j--; }
            else if (lv == 1) { put('-', ' ', cbb); j--; }
            else { put(ca, ' ', '-'); i--; }
            L = (int)lv;
        }
    }
    if (D1 > D0) {
        st.h += (D1 - D0) - (st.first ? 1 : 0);
        st.first = 0;
    }
    st.i = i;
    st.j = j;
    st.L = L;
    st.D = D1;
    if (len > cap) return fail(GA_E_ARG, "output capacity too small");
    return GA_OK;
}

// The end of a traceback: the MT state after its dispatches, the reference's tails, reversal.
int conclude_walk(const RngTable& snaps, const WalkStart& st, int reason, uint32_t* mt_state, const char* a_chr,
                  const char* b_chr, char* oa, char* om, char* ob, int64_t cap, int64_t len, int64_t* out_len,
                  int32_t* tb_status);

// Whole-problem traceback: one walk from (m, n), tails, reversal (dp_array_backward's output).
int finish_walk(ga_ctx* c, const RngTable& snaps, uint32_t* mt_state, const char* a_chr, const char* b_chr,
                char* oa, char* om, char* ob, int64_t cap, int64_t* out_len, int32_t* tb_status) {
    WalkStart st{c->m, c->n, 0, 0, 0, 1};
    int reason = 0;
    int64_t len = 0;
    if (int r = walk_segment(c, st, reason, a_chr, b_chr, oa, om, ob, cap, len)) return r;
    return conclude_walk(snaps, st, reason, mt_state, a_chr, b_chr, oa, om, ob, cap, len, out_len, tb_status);
}

int conclude_walk(const RngTable& snaps, const WalkStart& st, int reason, uint32_t* mt_state, const char* a_chr,
                  const char* b_chr, char* oa, char* om, char* ob, int64_t cap, int64_t len, int64_t* out_len,
                  int32_t* tb_status) {
    if (mt_state) state_after(snaps, st.D, mt_state);
    if (reason == 4) {  // IndexError in the reference
        *tb_status = GA_TB_INDEX_ERROR;
        *out_len = 0;
        return GA_OK;
    }
    auto put = [&](char x, char y, char z) {
        if (len < cap) { oa[len] = x; om[len] = y; ob[len] = z; }
        len++;
    };
    if (reason == 1)
        for (int64_t jj = st.j; jj > 0; jj--) put('-', ' ', b_chr[jj - 1]);
    else if (reason == 2)
        for (int64_t ii = st.i; ii > 0; ii--) put(a_chr[ii - 1], ' ', '-');
    if (len > cap) return fail(GA_E_ARG, "output capacity too small");
    std::reverse(oa, oa + len);
    std::reverse(om, om + len);
    std::reverse(ob, ob + len);
    *out_len = len;
    *tb_status = GA_TB_OK;
    return GA_OK;
}

// ---------------------------------------------------------------- banded traceback
// Traceback words take m*n*CB bytes.  Past a budget (GA_TB_BUDGET_MB, default 64 GB of the 288 GB),
// the traceback runs in bands of Bh rows: one score-only fill that also saves the
// (H', h2') row every Bh rows, then, from the bottom band up, a fill of the band's rows with
// traceback words (its top row from the checkpoint) and the walk through it, handed on at the
// band's top row (walk reason 6).  Fill work doubles; memory is one band of words.
int64_t band_rows(ga_ctx* c) {
    if (const char* e = c->knob("GA_TB_BAND_ROWS")) {  // tests: force (small) bands
        const int64_t Bh = (atoll(e) / ga::FROWS) * ga::FROWS;
        return Bh >= ga::FROWS && c->m >= 2 * Bh ? Bh : 0;
    }
    int64_t budget = (int64_t)64 << 30;
    if (const char* e = c->knob("GA_TB_BUDGET_MB")) budget = atoll(e) << 20;
    // ... and no more than the device has free for them (what this context's word buffer already holds counts as
    // free), less a 2 GB margin: a stored-words fill past it failed with GA_E_HIP instead of banding
    budget = std::min(budget, dev_avail_bytes(c, (int64_t)c->tb.cap));
    const int64_t words = ((c->n + 63) / 64) * 64 * c->CB;  // traceback bytes per row
    if (c->m * words <= budget) return 0;
    const int64_t Bh = std::max<int64_t>(64, (budget / words / ga::FROWS) * ga::FROWS);
    return c->m >= 2 * Bh ? Bh : 0;
}

int check_fill_abort(ga_ctx* c) {
    unsigned abort_word = 0;
    HIPCHK(hipMemcpy(&abort_word, c->flags.as<unsigned>() + 1, sizeof(unsigned), hipMemcpyDeviceToHost));
    if (abort_word) return fail(GA_E_TIMEOUT, "fill kernel hand-off wait timed out");
    return GA_OK;
}

int banded_align(ga_ctx* c, int64_t Bh, uint32_t* mt_state, const char* a_chr, const char* b_chr, char* oa, char* om,
                 char* ob, int64_t cap, int64_t* out_len, int32_t* tb_status, int64_t* cost_out) {
    const double t0 = now_ms();
    const int64_t m = c->m, n = c->n;
    // bands [b*Bh, b*Bh + Bh) of rows, the last one absorbing a remainder of < 16 rows
    int64_t nb = (m + Bh - 1) / Bh;
    if (nb > 1 && m - (nb - 1) * Bh < ga::FROWS) nb--;
    const int64_t nck = (m - 1) / Bh;  // checkpoint rows the fill writes (every multiple of Bh below m)
    HIPCHK(c->ckpt.ensure(sizeof(int2) * (size_t)std::max<int64_t>(nck, 1) * (n + 1)));
    int2* ck = c->ckpt.as<int2>();
    Band pass1;
    pass1.ckpt = ck;
    pass1.ckpt_rows = (int)Bh;
    if (int r = enqueue_fill(c, 0, pass1)) return r;
    RngTable R;
    const double t1 = now_ms();
    build_rng(mt_state, m + n + 1, R);
    c->rng_ms = (float)(now_ms() - t1);
    if (int r = finish_fill(c, cost_out, nullptr)) return r;
    WalkStart st{m, n, 0, 0, 0, 1};
    int reason = 6;
    int64_t len = 0;
    float walk_ms = 0.f, fill_ms = c->fill_ms;
    for (int64_t b = nb - 1; b >= 0 && reason == 6; b--) {
        Band bd;
        bd.band = true;
        bd.r0 = b * Bh;
        bd.mb = b == nb - 1 ? m - bd.r0 : Bh;
        // the path only moves up and left: this band's cells right of the column where the walk
        // enters it are never read, so the band fills columns 1..j only (on a diagonal-ish path
        // about half the refill work of full-width bands)
        bd.nc = st.j;
        if (b > 0) {
            int2* row = ck + (size_t)(b - 1) * (n + 1);
            // column 0 of the checkpoint row: the left edge's corner H'(r0, 0)
            HIPCHK(hipMemcpyAsync(row, c->left.as<int2>() + bd.r0, sizeof(int2), hipMemcpyDeviceToDevice, c->stream));
            bd.top = row;
        }
        if (int r = enqueue_fill(c, GA_FILL_TRACEBACK, bd)) return r;
        if (int r = run_walk(c, R.tab.data(), (int64_t)R.tab.size(), st, bd.r0, bd.mb, b > 0, b == nb - 1)) return r;
        int64_t seg = 0;
        if (int r = walk_segment(c, st, reason, a_chr, b_chr, oa + len, om + len, ob + len, cap - len, seg)) return r;
        if (int r = check_fill_abort(c)) return r;
        len += seg;
        walk_ms += c->walk_ms;
        float f = 0.f;
        if (hipEventElapsedTime(&f, c->ev[0], c->ev[1]) == hipSuccess) fill_ms += f;
    }
    c->walk_ms = walk_ms;
    c->fill_ms = fill_ms;
    const int rc = conclude_walk(R, st, reason, mt_state, a_chr, b_chr, oa, om, ob, cap, len, out_len, tb_status);
    c->call_ms = (float)(now_ms() - t0);
    return rc;
}

// ---------------------------------------------------------------- the recompute walk
// One find_global_alignment without stored traceback words: a score-only lane fill that leaves
// checkpoints, then one launch in which a workgroup walks while recompute workgroups write the
// traceback words of the 64-row blocks ahead of it into a small tile cache.  The fill runs at score-only
// speed and memory is O(checkpoints), not m*n words.
bool rc_eligible(ga_ctx* c) {
    const char* e = c->knob("GA_RC");  // 0: never; 1: whenever the shape allows (tests); default: large problems
    const int mode = e ? atoi(e) : -1;
    if (mode == 0 || c->slab || c->qbytes != 1 || c->K > 32) return false;
    if (c->m < 256 || c->n < 256) return false;  // (degenerate walks read cells no block ever recomputes)
    if (!rc_rows_fit(c->m)) return false;         // the lean checkpoint store's 32-bit buffer (ga_check.h)
    if (mode == 1) return true;
    // 2^26 cells and up (round 4): with the lean sub-chunk and 4-column stripes the recompute call beats the
    // stored-words one from C2 up (one call: C2 2.00 -> 1.75-1.77 ms, C5 4.12 -> 3.92, C3 15.73 -> 15.57;
    // tools/r4_td.sh, profiles/r04/single_call_td.txt); in round 3 C5's recompute fill at TD = 1 took 4.8 ms
    int64_t min_cells = (int64_t)1 << 26;
    if (const char* t = c->knob("GA_RC_MIN_CELLS")) min_cells = atoll(t);
    return c->m * c->n >= min_cells;
}

// checkpoint spacing (steps; a multiple of 32): 64 keeps a block's recompute at <= 127 + 63 steps; wider
// The checkpoint spacing trades recompute steps for checkpoint memory, (TD + 1) * 512 B per stripe per
// spacing: chosen with the geometry in enqueue_fill; GA_RC_EVERY (a power of two >= 64; rounded down) fixes it
int rc_every_req(const ga_ctx* c) {
    const char* e = c->knob("GA_RC_EVERY");  // a power of two in [64, 2^20] (checked in ga_ctx_create_opts)
    return e ? atoi(e) : 0;
}

// The score-only checkpointing fill of the loaded problem or slab.
int rc_fill(ga_ctx* c) {
    Band bd;
    bd.rc = true;
    bd.rc_every = rc_every_req(c);
    if (int r = enqueue_fill(c, 0, bd)) return r;
    c->rc_used = true;
    c->rc_T = c->T;
    return GA_OK;
}

// Launch the walk + recompute workgroups from walk state `st` on the walk buffers `wb` (its table already
// uploaded), after rc_fill.

// The tie-to-tie walk (experiments build only: it measured slower than the word walk, 7.15-7.72
// against 5.2 ms at C3) when GA_RC_JUMP asks for it and its workers fit: at most 4 columns per lane (a worker stages
// its block's 3 x 64 x 64*TD entries in LDS) and o <= 14 (X'-H', Y'-H' saturated at o+1 index a 1024-entry LUT).
bool rc_jump_wanted(ga_ctx* c, int TD) {
#ifdef GA_EXPERIMENTS
    return rc_jump_requested(c) && TD <= 4 && c->o <= 14 &&
           ga::rc_jump_lds_bytes(TD, c->rc_every_used) + 12 * 1024 <= 160 * 1024;
#else
    (void)c;
    (void)TD;
    return false;
#endif
}

int rc_walk_launch(ga_ctx* c, int64_t ntab, const WalkStart& st, WalkBufs& wb) {
    const int64_t m = c->m, n = c->n;
    const int TD = c->rc_T, CB = c->CB;
    const int nbi = (int)((m + 63) / 64), nbs = c->nstripes;
    c->rc_jump = rc_jump_wanted(c, TD);
    HIPCHK(c->rc_tb.ensure(rc_cache_bytes(c->rc_jump, TD, CB)));
    const size_t nflags = (size_t)nbi * nbs;
    // the cache slots' owner tags (ga::rc_slot_tag) carry the epoch's ready value: cleared with the flags
    const size_t nown = (size_t)ga::RC_CACHE_I * ga::RC_CACHE_S * sizeof(unsigned long long);
    if (c->rc_flags.cap < nflags * sizeof(unsigned) || c->rc_own.cap < nown || c->rc_epoch >= 0x7ffffff0u) {
        HIPCHK(c->rc_flags.ensure(nflags * sizeof(unsigned)));
        HIPCHK(hipMemsetAsync(c->rc_flags.p, 0, c->rc_flags.cap, wb.stream));
        HIPCHK(c->rc_own.ensure(nown));
        HIPCHK(hipMemsetAsync(c->rc_own.p, 0, nown, wb.stream));
        c->rc_epoch = 0;
    }
    c->rc_epoch++;
    HIPCHK(c->rc_pos.ensure(16));
    if (!c->rc_pos_zeroed) HIPCHK(hipMemsetAsync(c->rc_pos.p, 0, 16, wb.stream));
    c->rc_pos_zeroed = false;
    wb.tb = c->rc_tb.as<uint8_t>();
    ga::WalkArgs w = walk_args(c, ntab, st, 0, -1, false, wb);
    w.TC = ga::RC_CACHE_I * 4 * CB;  // 16-byte words per lane per 64-column stripe of the cache
    // 14 loaders, no L2 prefetcher (it would read blocks not yet recomputed); GA_RC_LOADERS = 12 / 13 leave
    // waves 8 and 12 / wave 8 (the walker's SIMD) idle instead
    w.nloaders = 14;
    if (const char* e = c->xknob("GA_RC_LOADERS")) w.nloaders = std::max(12, std::min(14, atoi(e)));
    w.rc_flags = c->rc_flags.as<unsigned>();
    w.rc_ready = 2u * c->rc_epoch + 1u;
    w.rc_own = c->rc_own.as<unsigned long long>();
    w.rc_nbs = nbs;
    w.rc_td = TD;
    w.rc_pos = c->rc_pos.as<unsigned>();
    ga::RcArgs r{};
    r.a = c->a.as<uint8_t>();
    r.b = c->b.as<uint8_t>() + c->col0;
    r.subp = c->qp.as<int>();
    r.K = c->K;
    r.top = c->top.as<int2>() + c->col0;
    // the slab's left edge (another GPU's right edge, landed in full by now) or column 0
    r.left = c->slab && c->col0 > 0 ? (c->halo_in_ext ? c->halo_in_ext : c->halo_in.as<int2>()) : c->left.as<int2>();
    r.colck = c->colck.as<int2>();
    r.stck = c->stck.as<int2>();
    r.stck_every = c->rc_every_used;
    r.tb = c->rc_tb.as<uint8_t>();
    r.TC = w.TC;
    r.m = (int)m;
    r.n = (int)n;
    r.o = c->o;
    r.TD = TD;
    r.nstripes = c->nstripes;
    r.nbi = nbi;
    r.nbs = nbs;
    r.flags = c->rc_flags.as<unsigned>();
    r.epoch = c->rc_epoch;
    r.own = w.rc_own;
    if (const char* e = c->knob("GA_RC_TAG_FAULT")) r.tag_fault = std::max(0, atoi(e));
    r.pos = c->rc_pos.as<unsigned>();
    r.tile0 = (int)((((st.i - 1) / 64) << 16) | ((st.j - c->col0 - 1) / 64));  // the walk's first tile
#ifdef GA_EXPERIMENTS
    r.worker_bytes = c->rc_jump ? ga::rc_jump_worker_bytes_host(TD, r.stck_every) : ga::rc_worker_bytes(TD, CB, r.stck_every);
#else
    r.worker_bytes = ga::rc_worker_bytes(TD, CB, r.stck_every);
#endif
    // one worker per workgroup (one per CU) by default: C3 blocks 14.7 us against 16.5 at three per CU,
    // the walker's tile waits 0.07 against 0.5 ms (tools/exp/r3_rc_diag.py)
    r.workers = c->rc_jump ? 1 : std::max(1, std::min(16, (int)((256 * 256 * 2 - 1024) / r.worker_bytes)));
    if (const char* e = c->knob("GA_RC_WPW")) r.workers = std::max(1, std::min(r.workers, atoi(e)));
    else r.workers = 1;
    r.spin_limit = 1u << 20;
    r.jlut = nullptr;
    if (c->rc_jump) {
        if (c->jlut_o != c->o) {
            std::vector<uint32_t> lut(4096);
            ga::jump_lut_build(c->o, lut.data());
            HIPCHK(c->jlut.ensure(sizeof(uint32_t) * lut.size()));
            HIPCHK(hipMemcpy(c->jlut.p, lut.data(), sizeof(uint32_t) * lut.size(), hipMemcpyHostToDevice));
            c->jlut_o = c->o;
        }
        r.jlut = c->jlut.as<uint4>();
    }
    {
        // the window: blocks up-left of the walker's (dbi block rows, dbs stripes), the path's likeliest
        // first: it runs near the diagonal, so the key is the tile distance plus the distance off the
        // diagonal, dbi + dbs*TD + cone*|dbi - dbs*TD| (GA_RC_CONE weighs the off-diagonal
        // distance more, which reaches further along the diagonal with the same 64 blocks).  Only the first
        // nwin are recomputed ahead (the walker's own 2 x 2 tiles always rank first); speculative blocks cost
        // the workers' time and the claims.  Candidates up to 31 block rows / 7 stripes away (offsets dbi*8 + dbs)
        // in a cache 64 x 32 deep (the safety argument is at rc_block's cache store, ga_rcwalk.hip).  Deeper
        // candidates keep the recompute ahead of a fast walker (C4, TD 4: a 28 us block against 27 us of walking
        // across 8 block rows; round 3 first searched 8 x 8, round 4 16 x 16: the default window is the same 64
        // blocks in all three).
        const int span = c->knob("GA_RC_SPAN") ? std::max(2, std::min(ga::RC_SPAN_I, atoi(c->knob("GA_RC_SPAN"))))
                                               : ga::RC_SPAN_I;
        // (cone 3 by default since round 6: the same 64 candidates reach further along the diagonal, so the walker
        // waits less on its tiles (C3 tile waits 0.31 -> 0.15 ms at TD 4, 0.70 -> 0.14 at TD 2) with fewer blocks
        // recomputed (TD 2: 16.7k -> 12.5k); cones 2 and 4 walk as fast, tools/exp/r6/check6.sh)
        const int cone = c->knob("GA_RC_CONE") ? std::max(1, std::min(8, atoi(c->knob("GA_RC_CONE")))) : 3;
        std::vector<std::pair<int, int>> off;
        for (int di = 0; di < span; di++)
            for (int dj = 0; dj < std::min(span, ga::RC_SPAN_S); dj++)
                off.push_back({di * 8 + dj, di + dj * TD + cone * std::abs(di - dj * TD)});
        // Liveness whatever the window's width: the walker waits only on tiles of its block and of the blocks
        // above it, left of it and up-left (its verified 2 x 2 tiles), so those four rank first (key -1);
        // ranked by the key alone, a 4-block window at TD = 4 held the walker's own stripe only, and one worker
        // never recomputed the stripe to its left (test_rc_worker_pools_vs_oracle[env0] timed out, round 4)
        for (auto& o : off)
            if (o.first == 0 || o.first == 1 || o.first == 8 || o.first == 9) o.second = -1;
        std::stable_sort(off.begin(), off.end(), [](const std::pair<int, int>& x, const std::pair<int, int>& y) {
            return x.second < y.second;
        });
        for (int k = 0; k < 64; k++) r.off[k] = k < (int)off.size() ? (unsigned char)off[k].first : 0;
        // 64 candidates (C3 walk 5.63 ms against 5.80 with 48 of 8 x 8, C4 with traceback 61 ms against 90:
        // tools/exp/r3b_span.sh)
        r.nwin = std::min(64, (int)off.size());
        if (const char* e = c->knob("GA_RC_WIN")) r.nwin = std::max(4, std::min(r.nwin, atoi(e)));
    }
    // recompute workgroups: with a faster walker (scalar entry loads) fewer workers keep up, and more of them
    // slow the walker's own tile loads (C3 walk 5.78 / 5.84 / 5.99 / 6.24 ms at 48 / 64 / 96 / 128 workers,
    // 6.05 at 40, 6.72 at 32: tools/exp/r3b_servers.sh); 64 keeps a margin above the cliff
    int nserv = 64;
    if (const char* e = c->knob("GA_RC_SERVERS")) nserv = std::max(1, std::min(255, atoi(e)));
    HIPCHK(hipEventRecord(wb.ev0, wb.stream));
#ifdef GA_EXPERIMENTS
    if (c->rc_jump) ga::launch_walk_rc_jump(wb.stream, w, r, nserv);
    else
#endif
        ga::launch_walk_rc(wb.stream, w, r, nserv);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(wb.ev1, wb.stream));
    return GA_OK;
}

// a slab's traceback fill (ga_slab_fill_launch): the same rule on the slab's own columns
bool rc_slab_eligible(ga_ctx* c) {
    const char* e = c->knob("GA_RC");
    const int mode = e ? atoi(e) : -1;
    if (mode == 0 || c->qbytes != 1 || c->K > 32 || c->m < 256 || c->n < 256) return false;
    if (!rc_rows_fit(c->m)) return false;  // the lean checkpoint store's 32-bit buffer (ga_check.h)
    if (mode == 1) return true;
    // C3 (10^10 cells) and up; C5 (20k x 20k protein) kept the stored-words path: its rc lane fill (313
    // stripes at TD = 1 for 20k rows) took 4.8 ms against the row scan's 1.8 (tools/exp/r3 bench_c5 logs)
    int64_t min_cells = (int64_t)1 << 32;
    if (const char* t = c->knob("GA_RC_MIN_CELLS")) min_cells = atoll(t);
    return c->m * c->n >= min_cells;
}

// One alignment's walk writing its levels to pinned host memory with a progress word (WalkArgs::ops_prog),
// so that the calling thread decodes them while the walk runs (rc_align, and the stored-words call)
int pinned_walk_levels(ga_ctx* c, WalkBufs& wb) {
    const int64_t m = c->m, n = c->n;
    const int64_t nwords = (m + n + 1 + 15) / 16 + 64;
    if (c->rc_ops_cap < nwords) {
        if (c->rc_ops_pin) HIPCHK(hipHostFree(c->rc_ops_pin));
        c->rc_ops_pin = nullptr;
        c->rc_ops_cap = 0;
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, sizeof(uint32_t) * nwords, hipHostMallocMapped | hipHostMallocCoherent));
        c->rc_ops_pin = static_cast<uint32_t*>(hp);
        c->rc_ops_cap = nwords;
    }
    if (!c->rc_ops_prog) {
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, 256, hipHostMallocMapped | hipHostMallocCoherent));
        c->rc_ops_prog = static_cast<unsigned*>(hp);
    }
    __atomic_store_n(c->rc_ops_prog, 0u, __ATOMIC_SEQ_CST);
    {
        void* dp = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dp, c->rc_ops_pin, 0));
        wb.ops = static_cast<uint32_t*>(dp);
        HIPCHK(hipHostGetDevicePointer(&dp, c->rc_ops_prog, 0));
        wb.ops_prog = static_cast<unsigned*>(dp);
    }
    // the walk's result words to pinned memory too: no hipMemcpy after the walk (round 6: the call's tail after the
    // walk held five small copies, ~0.1 ms)
    if (!c->res_pin) {
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, 64 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
        c->res_pin = static_cast<int*>(hp);
        void* dp = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dp, hp, 0));
        c->res_dev = static_cast<int*>(dp);
    }
    std::memset(c->res_pin, 0, 64 * sizeof(int));
    wb.result = c->res_dev;
    return GA_OK;
}

// The fill's result words (H'(m, n), the abort word) copied to pinned memory on the upload stream as soon as the
// fill ends, beside the walk (not on the fill's stream, where the copies would delay the walk's start), and read
// after the walk with no further copy; the cost's un-shift GV(m) + GH(n) comes from the host's own sums.
int fill_results_async(ga_ctx* c) {
    if (!c->ustream) HIPCHK(hipStreamCreateWithPriority(&c->ustream, hipStreamNonBlocking, c->priority));
    if (!c->ev_fill) HIPCHK(hipEventCreateWithFlags(&c->ev_fill, hipEventDisableTiming));
    if (!c->ev_res) HIPCHK(hipEventCreateWithFlags(&c->ev_res, hipEventDisableTiming));
    HIPCHK(hipEventRecord(c->ev_fill, c->stream));
    HIPCHK(hipStreamWaitEvent(c->ustream, c->ev_fill, 0));
    HIPCHK(hipMemcpyAsync(c->res_pin + 16, c->out_last.p, sizeof(int) * 4, hipMemcpyDeviceToHost, c->ustream));
    HIPCHK(hipMemcpyAsync(c->res_pin + 20, c->flags.as<unsigned>() + 1, sizeof(unsigned), hipMemcpyDeviceToHost,
                          c->ustream));
    HIPCHK(hipEventRecord(c->ev_res, c->ustream));
    return GA_OK;
}

int fill_results_finish(ga_ctx* c, int64_t* cost_out) {
    HIPCHK(hipEventSynchronize(c->ev_res));
    HIPCHK(hipEventElapsedTime(&c->fill_ms, c->ev[0], c->ev[1]));
    if (c->res_pin[20]) return fail(GA_E_TIMEOUT, "fill kernel hand-off wait timed out");
    c->GV_m = (int)c->gv_total;
    if (cost_out) *cost_out = (int64_t)c->res_pin[16] + c->gv_total + c->gh_total;
    return GA_OK;
}

// The calling thread's side of such a walk (launched on wb.stream after the fill): decode the levels as
// the progress word covers them, then the fill's cost, the walk's result words, the last levels, the
// tails and the final random state
int streamed_walk_finish(ga_ctx* c, const RngTable& R, const WalkBufs& wb, const WalkStart& st0, double t0,
                         uint32_t* mt_state, const char* a_chr, const char* b_chr, char* oa, char* om, char* ob,
                         int64_t cap, int64_t* out_len, int32_t* tb_status, int64_t* cost_out) {
    const int64_t m = c->m, n = c->n;
    const int64_t nwords = (m + n + 1 + 15) / 16 + 64;
    WalkStart st = st0;
    int reason = 0;
    int64_t len = 0;
    {
        // decode dispatches [D, D1) of the levels (dp_array_backward's column output, in walk order)
        const uint32_t* ops = c->rc_ops_pin;
        int64_t i = st.i, j = st.j, D = st.D;
        int L = st.L;
        auto decode_to = [&](int64_t D1) {
            for (; D < D1; D++) {
                const char ca = a_chr[pywrap(i - 1, m)], cbb = b_chr[pywrap(j - 1, n)];
                const unsigned lv = (ops[D >> 4] >> (30 - 2 * (D & 15))) & 3u;
                const int64_t k = len++;
                if (k < cap) {
                    if (lv == 0) { oa[k] = ca; om[k] = ca == cbb ? '|' : '*'; ob[k] = cbb; }
                    else if (lv == 1) { oa[k] = '-'; om[k] = ' '; ob[k] = cbb; }
                    else { oa[k] = ca; om[k] = ' '; ob[k] = '-'; }
                }
                i -= lv != 1;
                j -= lv != 2;
                L = (int)lv;
            }
        };
        const int64_t lag = [c] {
            const char* e = c->knob("GA_RC_DECODE_LAG");  // (diagnostics) blocks of 512 dispatches held back
            return e ? (int64_t)atoi(e) * 512 : (int64_t)0;
        }();
        std::vector<uint32_t> seen;  // (diagnostics) GA_RC_DECODE_CHECK: the words as decoded
        const bool check = c->knob("GA_RC_DECODE_CHECK") != nullptr;
        if (check) seen.assign((size_t)nwords, 0u);
        for (;;) {
            const unsigned pr = __atomic_load_n(c->rc_ops_prog, __ATOMIC_ACQUIRE);
            if ((int64_t)pr - lag > D) {
                if (check)
                    for (int64_t q = D >> 4; q < (((int64_t)pr - lag + 15) >> 4); q++) seen[q] = ops[q];
                decode_to((int64_t)pr - lag);
                continue;
            }
            const hipError_t q = hipStreamQuery(wb.stream);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return fail(GA_E_HIP, std::string("walk: ") + hipGetErrorString(q));
            std::this_thread::yield();
        }
        // the fill's cost and abort word (copied to pinned memory while the walk ran) and the walk's result words
        // (written to pinned memory by the walk): no copy here
        if (int rr = fill_results_finish(c, cost_out)) return rr;
        int res[16];
        std::memcpy(res, c->res_pin, sizeof(res));
        HIPCHK(hipEventElapsedTime(&c->walk_ms, wb.ev0, wb.ev1));
        c->walk_waits = res[4];
        c->walk_tiles = res[5];
        c->walk_t_tile = res[6];
        c->walk_t_ring = res[7];
        c->walk_t_total = res[8];
        c->walk_c_total = res[9];
        c->walk_load_ticks = res[10];
        c->walk_load_count = res[11];
        for (int q = 0; q < 3; q++) c->walk_jump_diag[q] = res[12 + q];
        reason = res[3];
        if (reason == 7) return fail(GA_E_TIMEOUT, "recompute walk: a tile was never recomputed");
        const int64_t D1 = res[0];
        if (D > D1) return fail(GA_E_STATE, "walk levels published past the walk's end");
        if (check) {
            int64_t bad = 0, first_bad = -1;
            for (int64_t q = 0; q < (D >> 4); q++)
                if (seen[q] != ops[q]) {
                    bad++;
                    if (first_bad < 0) first_bad = q;
                }
            if (bad)
                return fail(GA_E_STATE, "decode check: " + std::to_string(bad) + " level words changed after decode, first " +
                                            std::to_string(first_bad) + " of " + std::to_string(D >> 4) + " (D1 " +
                                            std::to_string(D1) + ")");
        }
        decode_to(D1);
        if (reason == 4) {  // (never here: such walks are degenerate, reason 7) the reference's IndexError
            len = 0;
            i = st.i;
            j = st.j;
        }
        if (D1 > st.D) {
            st.h += (D1 - st.D) - (st.first ? 1 : 0);
            st.first = 0;
        }
        st.i = i;
        st.j = j;
        st.L = L;
        st.D = D1;
        if (len > cap) return fail(GA_E_ARG, "output capacity too small");
    }
    const int rc = conclude_walk(R, st, reason, mt_state, a_chr, b_chr, oa, om, ob, cap, len, out_len, tb_status);
    c->call_ms = (float)(now_ms() - t0);
    return rc;
}

int rc_align(ga_ctx* c, uint32_t* mt_state, const char* a_chr, const char* b_chr, char* oa, char* om, char* ob,
             int64_t cap, int64_t* out_len, int32_t* tb_status, int64_t* cost_out) {
    const double t0 = now_ms();
    const int64_t m = c->m, n = c->n;
    // the walk's position words cleared before the fill (a memset between the fill and the walk delayed the walk)
    HIPCHK(c->rc_pos.ensure(16));
    HIPCHK(hipMemsetAsync(c->rc_pos.p, 0, 16, c->stream));
    if (int r = rc_fill(c)) {
        c->rc_pos_zeroed = false;
        return r;
    }
    c->rc_pos_zeroed = true;
    // the tie-break table on the host while the device fills
    RngTable R;
    const double t1 = now_ms();
    build_rng(mt_state, m + n + 1, R);
    c->rng_ms = (float)(now_ms() - t1);
    WalkBufs wb = ctx_walk_bufs(c);
    const int64_t ntab = (int64_t)R.tab.size();
    // the table goes up on a stream of its own while the fill still runs (pinned staging: the copy is asynchronous),
    // and the walk's stream waits for it: the walk launch below is then queued behind the fill at once
    if (c->up_cap < ntab) {
        if (c->up_pin) HIPCHK(hipHostFree(c->up_pin));
        c->up_pin = nullptr;
        c->up_cap = 0;
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, sizeof(uint32_t) * ntab, hipHostMallocDefault));
        c->up_pin = static_cast<uint32_t*>(hp);
        c->up_cap = ntab;
    }
    if (!c->ustream) HIPCHK(hipStreamCreateWithPriority(&c->ustream, hipStreamNonBlocking, c->priority));
    if (!c->ev_up) HIPCHK(hipEventCreateWithFlags(&c->ev_up, hipEventDisableTiming));
    // (the last call's copy out of the staging buffer has ended: its walk waited for it, and the call for its walk)
    std::memcpy(c->up_pin, R.tab.data(), sizeof(uint32_t) * ntab);
    HIPCHK(hipMemcpyAsync(wb.rng, c->up_pin, sizeof(uint32_t) * ntab, hipMemcpyHostToDevice, c->ustream));
    HIPCHK(hipEventRecord(c->ev_up, c->ustream));
    HIPCHK(hipStreamWaitEvent(wb.stream, c->ev_up, 0));
    // the walk's levels go to pinned host memory, and this thread decodes them while the walk runs
    if (int r = pinned_walk_levels(c, wb)) return r;
    // (after the table's upload on the same side stream: the copies there wait for the fill's end)
    if (int r = fill_results_async(c)) return r;
    const WalkStart st0{m, n, 0, 0, 0, 1};
    if (int r = rc_walk_launch(c, ntab, st0, wb)) return r;
    return streamed_walk_finish(c, R, wb, st0, t0, mt_state, a_chr, b_chr, oa, om, ob, cap, out_len, tb_status, cost_out);
}

// ---------------------------------------------------------------- pipelined repeated alignments
// `count` alignments of the loaded pair, each from the random state the previous one left.  Three
// slots of boundary arrays / traceback words / hand-off edges / walk buffers (every alignment runs
// the whole path: boundary, fill, table, walk, strings); fills alternate between two fill
// streams, so fill k+1 starts on the CUs fill k leaves idle (C3: one fill holds 196 of 256 CUs)
// and on those its tail frees, and walk k runs on a third stream beside them.  Walks are serial
// (alignment k's table slice starts where alignment k-1's dispatches ended); a host thread extends
// the one continuous tie-break stream ahead of them.
int pipe_setup(ga_ctx* c) {
    if (!c->wstream) HIPCHK(hipStreamCreateWithPriority(&c->wstream, hipStreamNonBlocking, c->priority));
    for (int f = 1; f < 4; f++)
        if (!c->fstream[f]) HIPCHK(hipStreamCreateWithPriority(&c->fstream[f], hipStreamNonBlocking, c->priority));
    if (c->walk_cus < 0) {
        // The walk's LDS tile torus (128 KB) needs a CU no fill workgroup occupies.  With the walk's CUs
        // masked out of the fill streams it never waits for one to drain, and two fills may share the
        // other CUs (GA_PIPE_WALK_CUS, default 0: unmasked streams)
        int wc = 0;
        if (const char* e = c->xknob("GA_PIPE_WALK_CUS")) wc = std::max(0, std::min(8, atoi(e)));
        c->walk_cus = wc;
        if (wc > 0) {
            const int nc = c->num_cu, words = (nc + 31) / 32;
            std::vector<uint32_t> fm(words, 0u), wm(words, 0u);
            for (int cu = 0; cu < nc; cu++) {
                auto& mk = cu >= nc - wc ? wm : fm;
                mk[cu >> 5] |= 1u << (cu & 31);
            }
            HIPCHK(hipExtStreamCreateWithCUMask(&c->mwstream, (uint32_t)words, wm.data()));
            for (int f = 0; f < 4; f++) HIPCHK(hipExtStreamCreateWithCUMask(&c->mfstream[f], (uint32_t)words, fm.data()));
        }
    }
    if (!c->pipe_pin) {
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, sizeof(int) * 8 * 6, hipHostMallocDefault));
        c->pipe_pin = static_cast<int*>(hp);
    }
    const int64_t per = c->m + c->n + 1;
    for (int s = 0; s < c->pipe_slots; s++) {
        auto& sl = c->pipe[s];
        for (hipEvent_t* e : {&sl.f0, &sl.f1, &sl.w0, &sl.w1})
            if (!*e) HIPCHK(hipEventCreate(e));
        if (!sl.fdone) HIPCHK(hipEventCreateWithFlags(&sl.fdone, hipEventDisableTiming));
        if (sl.tab_cap < per) {
            if (sl.tab_pin) HIPCHK(hipHostFree(sl.tab_pin));
            void* hp = nullptr;
            HIPCHK(hipHostMalloc(&hp, sizeof(uint32_t) * per, hipHostMallocDefault));
            sl.tab_pin = static_cast<uint32_t*>(hp);
            sl.tab_cap = per;
        }
        HIPCHK(sl.rng.ensure(sizeof(uint32_t) * (per + 64)));  // + the walk's entry look-ahead (SLD)
        HIPCHK(sl.ops.ensure(c->m + c->n + 1024));
        HIPCHK(sl.result.ensure(sizeof(int) * 16));
        const int64_t m = c->m, na = c->n_global;
        HIPCHK(sl.GVp.ensure(sizeof(int) * (m + 1)));
        HIPCHK(sl.GHp.ensure(sizeof(int) * (na + 1)));
        HIPCHK(sl.top.ensure(sizeof(int2) * (na + 1)));
        HIPCHK(sl.left.ensure(sizeof(int2) * (m + 1)));
        HIPCHK(sl.bnd_row.ensure(sizeof(int) * 3 * (na + 1)));
        HIPCHK(sl.bnd_col.ensure(sizeof(int) * 3 * (m + 1)));
        HIPCHK(sl.meta.ensure(sizeof(int) * 8));
        HIPCHK(sl.bscr.ensure(sizeof(int) * ga::boundary_scratch_ints((int)m, (int)na)));
        if (c->custom) {  // host-supplied boundary triples: the boundary pass reads them from the slot
            HIPCHK(hipMemcpyAsync(sl.bnd_row.p, c->bnd_row.p, sizeof(int) * 3 * (na + 1), hipMemcpyDeviceToDevice,
                                  c->stream));
            HIPCHK(hipMemcpyAsync(sl.bnd_col.p, c->bnd_col.p, sizeof(int) * 3 * (m + 1), hipMemcpyDeviceToDevice,
                                  c->stream));
        }
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return GA_OK;
}

// fill of an alignment into slot `slot` on stream `st`, then its cost inputs into pinned memory, then `fdone`
int pipe_fill(ga_ctx* c, int slot, hipStream_t st, bool row = false) {
    auto& sl = c->pipe[slot];
    Band bd;
    bd.tbuf = &sl.tb;
    bd.hbuf = &sl.hand;
    bd.fbuf = &sl.flags;
    bd.obuf = &sl.out_last;
    bd.stream = st;
    bd.ev0 = sl.f0;
    bd.ev1 = sl.f1;
    bd.GVp = &sl.GVp;
    bd.GHp = &sl.GHp;
    bd.top_b = &sl.top;
    bd.left = &sl.left;
    bd.bnd_row = &sl.bnd_row;
    bd.bnd_col = &sl.bnd_col;
    bd.meta = &sl.meta;
    bd.bscr = &sl.bscr;
    bd.lane_td = row ? 0 : c->pipe_lane_td;
    bd.lane_nwc = row ? 0 : c->pipe_lane_nwc;
    if (int r = enqueue_fill(c, GA_FILL_TRACEBACK, bd)) return r;
    int* pin = c->pipe_pin + 8 * slot;
    HIPCHK(hipMemcpyAsync(pin, sl.out_last.p, sizeof(int) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(pin + 4, sl.meta.p, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(pin + 5, sl.GHp.as<int>() + c->col0 + c->n, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(pin + 6, sl.flags.as<unsigned>() + 1, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(sl.fdone, st));
    return GA_OK;
}

// Per slot, pinned and coherent host memory for a pipelined walk's result words (256 B) and levels: the
// walk writes them there, so the host reads them without a hipMemcpy (which would wait for a CU, and
// the fills hold them all).  Returns the slot stride and the area's device address.
int pipe_io(ga_ctx* c, int S, size_t* stride, uint8_t** dev) {
    const size_t ops_bytes = (((size_t)(c->m + c->n + 1024) + 255) / 256) * 256, io_stride = 256 + ops_bytes;
    if (c->chain_io_cap < io_stride * S) {
        if (c->chain_io) HIPCHK(hipHostFree(c->chain_io));
        c->chain_io = nullptr;
        c->chain_io_cap = 0;
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, io_stride * S, hipHostMallocMapped | hipHostMallocCoherent));
        c->chain_io = static_cast<uint8_t*>(hp);
        c->chain_io_cap = io_stride * S;
    }
    void* d = nullptr;
    HIPCHK(hipHostGetDevicePointer(&d, c->chain_io, 0));
    *stride = io_stride;
    *dev = static_cast<uint8_t*>(d);
    return GA_OK;
}

// align_many with its walks chained in one walk_chain_kernel launch.  Each walk used to
// start after a host round trip (walk k's end seen by the host, its dispatch count read, walk k+1's
// table slice copied and its kernel launched: 45-55 us at C2 / C5, 0.1-0.2 ms at C3), and by then a
// queued fill workgroup could have taken the CU the walk had left (C3: a ~1 ms gap every fourth
// walk).  Now the walks keep their CU; walk k+1 starts when walk k ends, reading the tie-break stream
// from G_{k+1}, which the kernel sums itself, straight out of pinned host memory that the producer
// thread fills; the host only says which fills have ended and decodes each alignment's strings.
int align_chain(ga_ctx* c, int count, uint32_t* mt_state, const char* a_chr, const char* b_chr, char* oa, char* om,
                char* ob, int64_t cap, int64_t* out_len, int32_t* tb_status, int64_t* cost_out, double t0) {
    const int64_t m = c->m, n = c->n, per = m + n + 1;
    const int F = c->pipe_fills, S = c->pipe_slots;
    if (S > ga::WALK_CHAIN_SLOTS) return fail(GA_E_ARG, "too many pipeline slots for the walk chain");
    hipStream_t fs[4] = {c->stream, c->fstream[1], c->fstream[2], c->fstream[3]};
    if (!c->cwstream) {
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&c->cwstream, hipStreamNonBlocking, lo));
    }
    hipStream_t ws = c->cwstream;
    const int64_t need = (int64_t)count * per;
    if (c->chain_tab_cap < need) {
        if (c->chain_tab) HIPCHK(hipHostFree(c->chain_tab));
        c->chain_tab = nullptr;
        c->chain_tab_cap = 0;
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, sizeof(uint32_t) * need, hipHostMallocMapped | hipHostMallocCoherent));
        c->chain_tab = static_cast<uint32_t*>(hp);
        c->chain_tab_cap = need;
    }
    if (!c->chain_ctl) {
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent));
        c->chain_ctl = static_cast<unsigned*>(hp);
    }
    size_t io_stride = 0;
    uint8_t* io_dev = nullptr;
    if (int r = pipe_io(c, S, &io_stride, &io_dev)) return r;
    auto res_host = [&](int s) { return reinterpret_cast<int*>(c->chain_io + io_stride * s); };
    auto ops_host = [&](int s) { return reinterpret_cast<uint32_t*>(c->chain_io + io_stride * s + 256); };
    unsigned* ctl = c->chain_ctl;
    long long* tab_ready = reinterpret_cast<long long*>(ctl + 4);
    std::memset(ctl, 0, 64);
    void *tab_dev = nullptr, *ctl_dev = nullptr;
    HIPCHK(hipHostGetDevicePointer(&tab_dev, c->chain_tab, 0));
    HIPCHK(hipHostGetDevicePointer(&ctl_dev, ctl, 0));

    // the tie-break stream: a host thread extends it ahead of the walks, into pinned memory; started
    // before the fills are enqueued (C2 / C5: the first walk waited 2.1 / 4.0 ms for its entries)
    RngTable& R = c->many_rng;
    R.start(mt_state);
    R.tab.reserve((size_t)need);
    R.step_end.reserve((size_t)need + 4);
    R.acc.reserve((size_t)18 * need + 8);
    std::mutex mu;
    std::condition_variable cv;
    int64_t ready = 0;  // entries built (under mu)
    // walk k+1 may start the moment walk k ends, anywhere in [G_k + max(m, n), G_k + m + n]: the
    // entries are kept two alignments' worth ahead of the last walk known to have ended
    int64_t target = std::min<int64_t>(need, 3 * per);
    bool quit = false;
    double rng_ms = 0.0;
    std::thread producer([&] {
        for (;;) {
            int64_t want, from;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return quit || target > ready; });
                if (quit) return;
                want = std::min<int64_t>(target, need);
                from = ready;
                if (want <= ready) {
                    target = ready;
                    continue;
                }
            }
            const double t1 = now_ms();
            // in pieces of half an alignment, each published as soon as it is written: the first walk
            // waits for per entries, not for the three alignments' worth the producer starts with
            for (int64_t to = from; to < want;) {
                const int64_t nx = std::min(want, to + std::max<int64_t>(per / 2, 4096));
                R.extend(nx);
                std::memcpy(c->chain_tab + to, R.tab.data() + to, sizeof(uint32_t) * (nx - to));
                __atomic_store_n(tab_ready, (long long)nx, __ATOMIC_RELEASE);
                to = nx;
            }
            rng_ms += now_ms() - t1;
            {
                std::lock_guard<std::mutex> lk(mu);
                ready = want;
            }
            cv.notify_all();
        }
    });
    auto stop = [&](int rc) {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        cv.notify_all();
        producer.join();
        if (rc != GA_OK) __atomic_store_n(ctl + 2, 1u, __ATOMIC_RELEASE);  // the chain exits at its next wait
        (void)hipStreamSynchronize(ws);
        if (rc != GA_OK)
            for (int f = 0; f < F; f++) (void)hipStreamSynchronize(fs[f]);
        return rc;
    };
    int enqueued = 0, signalled = 0;
    auto launch_all = [&]() -> int {
        // fill 0 first (it fixes the fill geometry and so the size of every slot's traceback words), then
        // the walks' launch, so that its workgroup has a CU before the other fills take them all, then
        // fills 1 .. S-1; fill j goes into slot j % S on fill stream j % F (each computes its own boundary)
        if (int r = pipe_fill(c, 0, fs[0])) return r;
        enqueued++;
        // every slot's fill buffers at their final size now: a reallocation's hipFree while the chain runs
        // would wait for the chain, which waits for the host
        const size_t tb_bytes = (size_t)c->nstripes * c->T * c->TC * 1024;
        const size_t hand_bytes = sizeof(int2) * (size_t)c->nslabs * (m + 1);
        for (int s = 1; s < S; s++) {
            auto& sl = c->pipe[s];
            HIPCHK(sl.tb.ensure(tb_bytes));
            HIPCHK(sl.hand.ensure(hand_bytes));
            HIPCHK(sl.flags.ensure(sizeof(unsigned) * 16));
            HIPCHK(sl.out_last.ensure(sizeof(int) * 4));
        }
        ga::WalkChainArgs A{};
        for (int s = 0; s < S; s++) {
            auto& sl = c->pipe[s];
            const WalkBufs wb{sl.tb.as<uint8_t>(), nullptr, sl.ops.as<uint32_t>(), sl.result.as<int>(),
                              ws, nullptr, nullptr, sl.bnd_row.as<int>(), sl.bnd_col.as<int>()};
            A.w[s] = walk_args(c, per, WalkStart{m, n, 0, 0, 0, 1}, 0, -1, false, wb);
            A.w[s].result = reinterpret_cast<int*>(static_cast<uint8_t*>(io_dev) + io_stride * s);
            A.w[s].ops = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(io_dev) + io_stride * s + 256);
        }
        A.tab = static_cast<const uint32_t*>(tab_dev);
        A.ctl = static_cast<unsigned*>(ctl_dev);
        A.tab_ready = reinterpret_cast<const long long*>(static_cast<unsigned*>(ctl_dev) + 4);
        A.per = per;
        A.wait_limit = 100ull * 1000 * 1000 * 60;  // 60 s of s_memrealtime (100 MHz)
        A.count = count;
        A.S = S;
        HIPCHK(hipEventRecord(c->pipe[0].w0, ws));
        ga::launch_walk_chain(ws, A);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c->pipe[0].w1, ws));
        for (int k = 1; k < std::min(count, S); k++) {
            if (int r = pipe_fill(c, k, fs[k % F])) return r;
            enqueued++;
        }
        return GA_OK;
    };
    if (int r = launch_all()) return stop(r);
    FILE* trace = nullptr;
    if (const char* tp = c->knob("GA_PIPE_TRACE")) trace = fopen(tp, "a");
    const double h0 = now_ms();
    int64_t G = 0;
    float fill_sum = 0.f, walk_sum = 0.f;
    int rc = GA_OK;
    for (int k = 0; k < count && rc == GA_OK; k++) {
        auto& sl = c->pipe[k % S];
        // wait for walk k; meanwhile tell the chain which fills have ended (in order, enqueued ones only:
        // a slot's event still holds the previous fill of that slot until the next is enqueued)
        for (;;) {
            while (signalled < enqueued && hipEventQuery(c->pipe[signalled % S].fdone) == hipSuccess)
                __atomic_store_n(ctl, (unsigned)++signalled, __ATOMIC_RELEASE);
            if ((int)__atomic_load_n(ctl + 1, __ATOMIC_ACQUIRE) > k) break;
            if (__atomic_load_n(ctl + 3, __ATOMIC_ACQUIRE)) {
                rc = fail(GA_E_TIMEOUT, "chained walk waited too long for its fill or tie-break entries");
                break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        if (rc != GA_OK) break;
        int res[16];
        std::memcpy(res, res_host(k % S), sizeof(res));
        const int64_t Dk = res[0];
        {
            std::lock_guard<std::mutex> lk(mu);
            target = std::max(target, G + Dk + 2 * per + per / 8);
        }
        cv.notify_all();
        const int* pin = c->pipe_pin + 8 * (k % S);
        if (pin[6]) {
            rc = fail(GA_E_TIMEOUT, "fill kernel hand-off wait timed out");
            break;
        }
        cost_out[k] = (int64_t)pin[0] + pin[4] + pin[5];
        float f = 0.f;
        if (hipEventElapsedTime(&f, sl.f0, sl.f1) == hipSuccess) fill_sum += f;
        walk_sum += res[8] / 1.0e5f;  // the walker's own time (s_memrealtime ticks, 100 MHz)
        if (trace)
            fprintf(trace, "{\"k\": %d, \"chain\": 1, \"fill_ms\": %.3f, \"walk_ms\": %.3f, \"walk_done_host\": %.3f, "
                    "\"D\": %lld, \"tile_wait_us\": %.2f, \"tile_loads\": %d, \"chain_wait_us\": %.2f, "
                    "\"polls_fill\": %d, \"polls_tab\": %d}\n", k, f, res[8] / 1.0e5,
                    now_ms() - h0, (long long)Dk, res[6] / 100.0, res[11], res[12] / 100.0, res[13], res[14]);
        // fill k+S into slot k's buffers (walk k has read them)
        if (k + S < count) {
            if (int r = pipe_fill(c, k % S, fs[(k + S) % F])) {
                rc = r;
                break;
            }
            enqueued++;
        }
        // alignment k's strings, while walk k+1 and the fills run
        const WalkBufs wb{sl.tb.as<uint8_t>(), nullptr, sl.ops.as<uint32_t>(), sl.result.as<int>(),
                          ws, nullptr, nullptr, sl.bnd_row.as<int>(), sl.bnd_col.as<int>()};
        WalkStart st{m, n, 0, 0, 0, 1};
        int reason = 0;
        int64_t len = 0;
        char* a_k = oa + (size_t)k * cap;
        char* m_k = om + (size_t)k * cap;
        char* b_k = ob + (size_t)k * cap;
        if (int r = decode_segment(c, res, st, reason, a_chr, b_chr, a_k, m_k, b_k, cap, len, wb, true,
                                   ops_host(k % S))) {
            rc = r;
            break;
        }
        if (int r = conclude_walk(R, st, reason, nullptr, a_chr, b_chr, a_k, m_k, b_k, cap, len, &out_len[k],
                                  &tb_status[k])) {
            rc = r;
            break;
        }
        G += st.D;
    }
    if (trace) fclose(trace);
    if (int r = stop(rc)) return r;
    state_after(R, G, mt_state);  // the state the last alignment leaves (random.getstate() layout)
    c->fill_ms = fill_sum / count;
    c->walk_ms = walk_sum / count;
    c->rng_ms = (float)(rng_ms / count);
    c->call_ms = (float)(now_ms() - t0);
    c->filled_tb = false;
    return GA_OK;
}

int align_many(ga_ctx* c, int count, uint32_t* mt_state, const char* a_chr, const char* b_chr, char* oa, char* om,
               char* ob, int64_t cap, int64_t* out_len, int32_t* tb_status, int64_t* cost_out) {
    const double t0 = now_ms();
    {
        // Fill kernel and fills in flight.  A row-scan traceback fill of C3 holds 196 CUs
        // at two waves per SIMD and is issue bound there: a second fill in flight only fills the CUs it
        // leaves idle (10.4 ms per alignment in steady state), and co-resident fills gain nothing.  The
        // lane-skewed traceback fill at 4 columns per lane runs 391 stripes in 98 one-wave-per-SIMD
        // workgroups: a narrow, latency-bound fill (26 ms alone), three of which share the chip
        // (8.65 ms per alignment; tools/exp/pipe_lane2.sh).  So one-byte words of long rows (K <= 32,
        // an int8 profile) take lane fills; the rest three row-scan fills.  GA_PIPE_MODE=row|lane
        // and GA_PIPE_FILLS (2..4) override.
        const char* pm = c->knob("GA_PIPE_MODE");
        bool lane = c->CB == 1 && c->qbytes == 1 && c->K <= 32 && c->m >= 32768 && c->n >= 4 * 4 * 64 * 64 &&
                    c->diag_req != 1 && c->diag_req != 2;
        if (pm && !strcmp(pm, "row")) lane = false;
        if (pm && !strcmp(pm, "lane")) lane = c->qbytes == 1 && c->K <= 32;
        c->pipe_lane_td = lane ? (c->CB == 1 ? 4 : 2) : 0;
        c->pipe_lane_nwc = lane ? 4 : 0;
        // Lane fills: four in flight when the process has the hardware queues for them (the fill streams
        // and the walk stream share a priority's pool of GPU_MAX_HW_QUEUES queues; two streams on one
        // in-order queue serialise): C3 steady state 8.34 -> 7.81 ms per alignment, walk-bound
        // (tools/exp/pipe_queues.sh); three with HIP's default of four queues
        const int queues = c->hw_queues;
        // row-scan fills: three in flight (four streams with the walk's: HIP's default pool holds them);
        // with the faster walk C5 is no longer walk-bound (1.80 -> 1.51 ms per alignment), C2 unchanged
        int F = lane ? (queues >= 5 ? 4 : 3) : 3;
        if (const char* e = c->knob("GA_PIPE_FILLS")) F = std::max(2, std::min(4, atoi(e)));
        c->pipe_fills = F;
        // slots: fill k + S reuses walk k's buffers, so the walk chain allows one alignment per
        // (walk + fill) / S; GA_PIPE_SLOTS raises S above F + 1 (up to 6)
        int S = F + 1;
        if (const char* e = c->knob("GA_PIPE_SLOTS")) S = std::max(F + 1, std::min(6, atoi(e)));
        c->pipe_slots = S;
    }
    if (int r = pipe_setup(c)) return r;
    {
        // the walks chained in one launch (align_chain) behind row-scan fills: C2 0.908 -> 0.823 ms per
        // alignment, C5 1.522 -> 1.507.  Not behind the lane fills: C3 8.96-9.05 -> 9.47-9.55, its four
        // narrow fills (392 workgroups for 256 CUs) running 27.4 -> 29.5 ms each beside a walk that never
        // gives its CU back (tools/exp/chain_ab.sh).  Opt-in (GA_PIPE_CHAIN=1): the persistent chain polls
        // host-written words, so a device-synchronising call another thread of the process makes while it
        // runs (hipFree, hipDeviceSynchronize, a torch allocator release) would wait on it until its 60 s
        // bound; per-launch walks have no such hazard and cost C2 / C5 ~1-10 % more per alignment.
        const char* ch = c->knob("GA_PIPE_CHAIN");
        const bool fits = (int64_t)count * (c->m + c->n + 1) <= ((int64_t)256 << 20);  // 1 GB of entries
        const bool on = ch != nullptr && atoi(ch) != 0;
        if (on && fits && c->walk_cus == 0 && !c->knob("GA_PIPE_FILL_PRIO") && !c->xknob("GA_PIPE_ROW_FIRST"))
            return align_chain(c, count, mt_state, a_chr, b_chr, oa, om, ob, cap, out_len, tb_status, cost_out, t0);
    }
    const int64_t m = c->m, n = c->n, per = m + n + 1;
    const int F = c->pipe_fills, S = c->pipe_slots;
    hipStream_t fs[4] = {c->stream, c->fstream[1], c->fstream[2], c->fstream[3]};
    hipStream_t ws = c->wstream;
    if (c->walk_cus > 0) {
        for (int f = 0; f < 4; f++) fs[f] = c->mfstream[f];
        ws = c->mwstream;
    } else if (const char* fp = c->knob("GA_PIPE_FILL_PRIO"); fp && !strcmp(fp, "normal")) {
        for (int f = 0; f < 4; f++) {
            if (!c->nfstream[f]) HIPCHK(hipStreamCreateWithPriority(&c->nfstream[f], hipStreamNonBlocking, 0));
            fs[f] = c->nfstream[f];
        }
    }
    // GA_PIPE_TRACE=<file>: per alignment, GPU times (ms from the first fill's enqueue) of fill and walk
    // start / end and host times of the walk launches (a diagnostic of what bounds the pipeline)
    struct PipeTrace {  // closed on every return path
        FILE* f = nullptr;
        hipEvent_t origin = nullptr;
        ~PipeTrace() {
            if (f) fclose(f);
            if (origin) (void)hipEventDestroy(origin);
        }
    } tr;
    if (const char* tp = c->knob("GA_PIPE_TRACE"))
        if (hipEventCreate(&tr.origin) == hipSuccess && hipEventRecord(tr.origin, fs[0]) == hipSuccess)
            tr.f = fopen(tp, "a");
    FILE* const trace = tr.f;
    const hipEvent_t origin = tr.origin;
    const double h0 = now_ms();
    double walk_launch_host = 0.0;
    // experiment (GA_PIPE_ROW_FIRST=r): the first r fills through the row scan (shorter latency alone)
    int row_first = 0;
    if (const char* e = c->xknob("GA_PIPE_ROW_FIRST")) row_first = atoi(e);
    // fill j into slot j % S on fill stream j % F; each computes its own boundary.  Every fill of the
    // pipeline computes the same arrays (the same pair, boundary and words), so walk k takes whichever
    // pending slot's fill ended first, not slot k % S: in the ramp the third of four fills started at
    // once ends ~3 ms after the fourth and ~3 ms after the third walk wanted it (GA_PIPE_SLOT_ORDER=fixed
    // keeps slot k % S)
    const bool any_order = [c] {
        const char* e = c->knob("GA_PIPE_SLOT_ORDER");
        return !(e && !strcmp(e, "fixed"));
    }();
    size_t io_stride = 0;
    uint8_t* io_dev = nullptr;
    if (int r = pipe_io(c, S, &io_stride, &io_dev)) return r;
    // slot s's walk writes its result words and levels to pinned memory (pipe_io; GA_PIPE_PINNED_IO=0:
    // to the slot's device buffers, read back with hipMemcpy)
    const bool pinned_io = [c] {
        const char* e = c->knob("GA_PIPE_PINNED_IO");
        return !(e && atoi(e) == 0);
    }();
    auto walk_bufs = [&](int s) {
        auto& sl = c->pipe[s];
        return WalkBufs{sl.tb.as<uint8_t>(), sl.rng.as<uint32_t>(),
                        pinned_io ? reinterpret_cast<uint32_t*>(io_dev + io_stride * s + 256) : sl.ops.as<uint32_t>(),
                        pinned_io ? reinterpret_cast<int*>(io_dev + io_stride * s) : sl.result.as<int>(), ws, sl.w0,
                        sl.w1, sl.bnd_row.as<int>(), sl.bnd_col.as<int>()};
    };
    std::vector<int> pending;  // slots holding an enqueued fill no walk has taken, in enqueue order
    std::vector<int> walk_slot((size_t)count, -1);
    int fills_enqueued = 0;
    for (int k = 0; k < std::min(count, S); k++) {
        if (int r = pipe_fill(c, k, fs[k % F], k < row_first)) return r;
        pending.push_back(k);
        fills_enqueued++;
    }
    // the tie-break table: one continuous stream, extended by a host thread ahead of the walks (its
    // vectors are reserved up front: the walks read earlier entries while later ones are written)
    RngTable& R = c->many_rng;
    R.start(mt_state);
    R.tab.reserve((size_t)count * per);
    R.step_end.reserve((size_t)count * per + 4);
    R.acc.reserve((size_t)18 * count * per + 8);
    const uint32_t* tabp = R.tab.data();  // stable: the capacity is reserved
    std::mutex mu;
    std::condition_variable cv;
    int64_t ready = 0;         // entries available to the walks (under mu)
    // entries the producer builds up to (under mu): the first three alignments' worth while the first
    // fills run (each alignment takes about (m + n) / 1.6 dispatches), then kept ahead of the walks
    int64_t target = std::min<int64_t>((int64_t)count * per, 3 * per);
    bool quit = false;
    double rng_ms = 0.0;
    std::thread producer([&] {
        for (;;) {
            int64_t want;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return quit || target > ready; });
                if (quit) return;
                want = std::min<int64_t>(target, (int64_t)count * per);
                if (want <= ready) {
                    target = ready;  // nothing more can be built
                    continue;
                }
            }
            const double t1 = now_ms();
            R.extend(want);
            rng_ms += now_ms() - t1;
            {
                std::lock_guard<std::mutex> lk(mu);
                ready = want;
            }
            cv.notify_all();
        }
    });
    // walk k over its table slice [G, G + per), after fill k, on the walk stream
    auto start_walk = [&](int k, int64_t G) -> int {
        // the slot: the first pending one whose fill has ended; while all are still running, the host
        // waits for the first to end (the oldest is not always first: in the ramp four fills share the chip)
        size_t pick = 0;
        for (bool found = !any_order; !found;) {
            for (size_t q = 0; q < pending.size() && !found; q++)
                if (hipEventQuery(c->pipe[pending[q]].fdone) == hipSuccess) {
                    pick = q;
                    found = true;
                }
            if (!found) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        walk_slot[k] = pending[pick];
        pending.erase(pending.begin() + (long)pick);
        auto& sl = c->pipe[walk_slot[k]];
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return ready >= G + per; });
        }
        HIPCHK(hipStreamWaitEvent(ws, sl.fdone, 0));
        std::memcpy(sl.tab_pin, tabp + G, sizeof(uint32_t) * per);
        const WalkBufs wb = walk_bufs(walk_slot[k]);
        return run_walk(c, sl.tab_pin, per, WalkStart{m, n, 0, 0, 0, 1}, 0, -1, false, true, &wb);
    };
    int rc = start_walk(0, 0);
    walk_launch_host = now_ms() - h0;
    int64_t G = 0;  // global dispatches consumed by the alignments before k
    int64_t Dmax = 0;
    float fill_sum = 0.f, walk_sum = 0.f;
    for (int k = 0; k < count && rc == GA_OK; k++) {
        auto& sl = c->pipe[walk_slot[k]];
        const WalkBufs wb = walk_bufs(walk_slot[k]);
        const int* res_pin = reinterpret_cast<const int*>(c->chain_io + io_stride * walk_slot[k]);
        const uint32_t* ops_pin = reinterpret_cast<const uint32_t*>(c->chain_io + io_stride * walk_slot[k] + 256);
        auto step = [&]() -> int {
            // walk k done: its dispatch count fixes where walk k+1's table slice starts
            HIPCHK(hipEventSynchronize(sl.w1));
            int res[16];
            if (pinned_io) std::memcpy(res, res_pin, sizeof(res));
            else HIPCHK(hipMemcpy(res, sl.result.p, sizeof(int) * 16, hipMemcpyDeviceToHost));
            const int64_t Dk = res[0];
            Dmax = std::max(Dmax, Dk);
            if (trace) {
                float t[4] = {0.f, 0.f, 0.f, 0.f};
                hipEvent_t evs[4] = {sl.f0, sl.f1, sl.w0, sl.w1};
                for (int q = 0; q < 4; q++) (void)hipEventElapsedTime(&t[q], origin, evs[q]);
                // the walker's own accounting (walk_kernel result[4..11]; s_memrealtime ticks at 100 MHz)
                fprintf(trace, "{\"k\": %d, \"fill0\": %.3f, \"fill1\": %.3f, \"walk0\": %.3f, \"walk1\": %.3f, "
                        "\"walk_launch_host\": %.3f, \"walk_done_host\": %.3f, \"D\": %lld, \"tile_wait_us\": %.2f, "
                        "\"walker_us\": %.2f, \"tile_loads\": %d, \"load_us_per_tile\": %.3f}\n", k, t[0], t[1], t[2],
                        t[3], walk_launch_host, now_ms() - h0, (long long)Dk, res[6] / 100.0, res[8] / 100.0, res[11],
                        res[11] > 0 ? res[10] / 100.0 / res[11] : 0.0);
            }
            {
                // keep the producer an alignment's worth (and some) ahead of the next walk
                std::lock_guard<std::mutex> lk(mu);
                target = std::max(target, G + Dk + per + Dmax + Dmax / 8);
            }
            cv.notify_all();
            if (k + 1 < count) {
                if (int r = start_walk(k + 1, G + Dk)) return r;
                walk_launch_host = now_ms() - h0;
            }
            // alignment k's cost (fill k finished before walk k started) and walk time, before slot k's
            // pinned words and events are reused
            const int* pin = c->pipe_pin + 8 * walk_slot[k];
            if (pin[6]) return fail(GA_E_TIMEOUT, "fill kernel hand-off wait timed out");
            cost_out[k] = (int64_t)pin[0] + pin[4] + pin[5];
            float f = 0.f;
            if (hipEventElapsedTime(&f, sl.f0, sl.f1) == hipSuccess) fill_sum += f;
            float wms = 0.f;
            if (hipEventElapsedTime(&wms, sl.w0, sl.w1) == hipSuccess) walk_sum += wms;
            // the next fill into walk k's slot (walk k has read it), on its stream after the fill F before
            if (fills_enqueued < count) {
                if (int r = pipe_fill(c, walk_slot[k], fs[fills_enqueued % F])) return r;
                pending.push_back(walk_slot[k]);
                fills_enqueued++;
            }
            // alignment k's strings, while walk k+1 and the fills run
            WalkStart st{m, n, 0, 0, 0, 1};
            int reason = 0;
            int64_t len = 0;
            char* a_k = oa + (size_t)k * cap;
            char* m_k = om + (size_t)k * cap;
            char* b_k = ob + (size_t)k * cap;
            if (int r = decode_segment(c, res, st, reason, a_chr, b_chr, a_k, m_k, b_k, cap, len, wb, true,
                                       pinned_io ? ops_pin : nullptr))
                return r;
            if (int r = conclude_walk(R, st, reason, nullptr, a_chr, b_chr, a_k, m_k, b_k, cap, len, &out_len[k],
                                      &tb_status[k]))
                return r;
            G += st.D;
            return GA_OK;
        };
        rc = step();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        quit = true;
    }
    cv.notify_all();
    producer.join();
    if (rc != GA_OK) {
        for (int f = 0; f < F; f++) (void)hipStreamSynchronize(fs[f]);
        (void)hipStreamSynchronize(ws);
        return rc;
    }
    state_after(R, G, mt_state);  // the state the last alignment leaves (random.getstate() layout)
    c->fill_ms = fill_sum / count;
    c->walk_ms = walk_sum / count;
    c->rng_ms = (float)(rng_ms / count);
    c->call_ms = (float)(now_ms() - t0);
    c->filled_tb = false;  // ctx->tb does not hold the last fill's words
    return GA_OK;
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

const char* ga_last_error(void) { return g_err.c_str(); }

int ga_device_count(int* count) {
    if (!count) return fail(GA_E_ARG, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return fail(GA_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    *count = n;
    return GA_OK;
}

int ga_ctx_create(int device, ga_ctx** out) { return ga_ctx_create_opts(device, nullptr, out); }

int ga_ctx_create_opts(int device, const char* options, ga_ctx** out) {
    if (!out) return fail(GA_E_ARG, "null out");
    // the knobs, once (ga_ctx::knobs): the environment's shipped ones, then the options ("NAME=VALUE" entries
    // separated by ';' or newlines), checked before any device work
    std::map<std::string, std::string> knobs;
    for (char** e = environ; e && *e; e++)
        if (!strncmp(*e, "GA_", 3))
            if (const char* eq = strchr(*e, '=')) {
                std::string name(*e, (size_t)(eq - *e));
                if (env_knob(name)) knobs[name] = eq + 1;
            }
    if (options) {
        std::string s(options), item;
        for (size_t p = 0; p <= s.size(); p++) {
            if (p < s.size() && s[p] != ';' && s[p] != '\n') {
                item += s[p];
                continue;
            }
            if (!item.empty()) {
                const size_t eq = item.find('=');
                if (eq == std::string::npos || item.compare(0, 3, "GA_") != 0)
                    return fail(GA_E_ARG, "bad option '" + item + "' (expected GA_NAME=VALUE)");
                knobs[item.substr(0, eq)] = item.substr(eq + 1);
            }
            item.clear();
        }
    }
    {
        // GA_RC_EVERY: the checkpoint spacing is a power of two (a mask and a shift per iteration)
        const auto it = knobs.find("GA_RC_EVERY");
        if (it != knobs.end()) {
            const long v = atol(it->second.c_str());
            if (v < 64 || (v & (v - 1)) != 0 || v > (1L << 20))
                return fail(GA_E_ARG, "GA_RC_EVERY must be a power of two in [64, 2^20], not '" + it->second + "'");
        }
    }
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(GA_E_ARG, "no such HIP device");
    HIPCHK(hipSetDevice(device));
    ga_ctx* c = new ga_ctx();
    c->device = device;
    c->knobs = std::move(knobs);
    {
        // hardware queues per priority pool: what the HIP runtime read when it started, i.e. the variable
        // as the process first saw it here (a later change, e.g. a module setting it after HIP started,
        // does not change the runtime's queues)
        static const int hwq = [] {
            const char* e = getenv("GPU_MAX_HW_QUEUES");
            return e && atoi(e) > 0 ? atoi(e) : 4;
        }();
        c->hw_queues = hwq;
    }
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->num_cu = cus;
        if (const char* e = c->knob("GA_COLS_PER_LANE")) c->T_req = atoi(e);  // tuning overrides
        if (const char* e = c->knob("GA_FILL_NWC")) c->nwc_req = atoi(e);
        if (const char* e = c->knob("GA_FILL_MODE"))
            c->diag_req = !strcmp(e, "diag") ? 2 : !strcmp(e, "row") ? 1 : !strcmp(e, "lane") ? 3 : 0;
        if (const char* e = c->knob("GA_LANE_COLS_PER_LANE")) c->lane_T_req = atoi(e);
        if (const char* e = c->knob("GA_DIAG_COLS_PER_LANE")) c->diag_T_req = atoi(e);
    }
    // The fill runs on a stream of the greatest priority.  HIP keeps a separate pool of hardware
    // queues per priority (GPU_MAX_HW_QUEUES = 4 per pool and process), so no normal-priority
    // stream -- torch's, RCCL's -- is ever put behind a running fill in the same in-order queue;
    // a slab fill that waits on its halo needs the RCCL kernel that delivers it to run beside it
    // (DESIGN.md 7).  GA_STREAM_PRIORITY=normal restores a default-priority stream (experiments).
    {
        int lo = 0, hi = 0;
        const char* pe = c->knob("GA_STREAM_PRIORITY");
        const bool normal = pe && !strcmp(pe, "normal");
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
        c->priority = normal ? 0 : hi;  // 0: the default priority (lo is the LEAST, another pool)
        if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, c->priority) != hipSuccess) {
            delete c;
            return fail(GA_E_HIP, "hipStreamCreateWithPriority failed");
        }
    }
    if (hipEventCreateWithFlags(&c->ev_dep, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return fail(GA_E_HIP, "hipEventCreate failed");
    }
    for (auto& e : c->ev) {
        if (hipEventCreate(&e) != hipSuccess) {
            delete c;
            return fail(GA_E_HIP, "hipEventCreate failed");
        }
    }
    *out = c;
    return GA_OK;
}

void ga_ctx_destroy(ga_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (DevBuf* b : {&c->a, &c->b, &c->sub, &c->gh, &c->gv, &c->qp, &c->GVp, &c->GHp, &c->top, &c->left, &c->bnd_row,
                      &c->bnd_col, &c->meta, &c->hand, &c->flags, &c->tb, &c->out_last, &c->full, &c->rng, &c->ops,
                      &c->result, &c->halo_in, &c->dbg, &c->wdbg, &c->bscr, &c->ckpt, &c->colck, &c->stck,
                      &c->rc_tb, &c->rc_flags, &c->rc_pos, &c->rc_own, &c->link, &c->qprof})
        b->release();
    if (c->prog_host) (void)hipHostFree(c->prog_host);
    if (c->peer_link) (void)hipIpcCloseMemHandle(c->peer_link);
    if (c->rc_ops_pin) (void)hipHostFree(c->rc_ops_pin);
    if (c->rc_ops_prog) (void)hipHostFree(c->rc_ops_prog);
    if (c->up_pin) (void)hipHostFree(c->up_pin);
    if (c->ev_up) (void)hipEventDestroy(c->ev_up);
    if (c->res_pin) (void)hipHostFree(c->res_pin);
    if (c->ev_fill) (void)hipEventDestroy(c->ev_fill);
    if (c->ev_res) (void)hipEventDestroy(c->ev_res);
    if (c->ustream) (void)hipStreamDestroy(c->ustream);
    for (auto& sl : c->pipe) {
        for (DevBuf* b : {&sl.tb, &sl.hand, &sl.flags, &sl.out_last, &sl.rng, &sl.ops, &sl.result, &sl.GVp, &sl.GHp,
                          &sl.top, &sl.left, &sl.bnd_row, &sl.bnd_col, &sl.meta, &sl.bscr})
            b->release();
        for (hipEvent_t e : {sl.f0, sl.f1, sl.fdone, sl.w0, sl.w1})
            if (e) (void)hipEventDestroy(e);
        if (sl.tab_pin) (void)hipHostFree(sl.tab_pin);
    }
    if (c->pipe_pin) (void)hipHostFree(c->pipe_pin);
    if (c->chain_tab) (void)hipHostFree(c->chain_tab);
    if (c->chain_ctl) (void)hipHostFree(c->chain_ctl);
    if (c->chain_io) (void)hipHostFree(c->chain_io);
    if (c->wstream) (void)hipStreamDestroy(c->wstream);
    if (c->cwstream) (void)hipStreamDestroy(c->cwstream);
    if (c->mwstream) (void)hipStreamDestroy(c->mwstream);
    for (hipStream_t ms : c->mfstream)
        if (ms) (void)hipStreamDestroy(ms);
    for (hipStream_t ns : c->nfstream)
        if (ns) (void)hipStreamDestroy(ns);
    for (int f = 1; f < 4; f++)
        if (c->fstream[f]) (void)hipStreamDestroy(c->fstream[f]);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_dep) (void)hipEventDestroy(c->ev_dep);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int ga_problem_set(ga_ctx* c, const uint8_t* a, int64_t m, const uint8_t* b, int64_t n, const ga_costs* cs,
                   const int32_t* row0, const int32_t* col0) {
    if (int r = check_ctx(c)) return r;
    c->slab = false;
    return load_problem(c, a, m, b, n, cs, row0, col0, 0, n);
}

int ga_problem_fill(ga_ctx* c, int32_t flags, int64_t* cost_out, int32_t* full_out) {
    if (c) c->rc_used = false;
    if (int r = check_ctx(c)) return r;
    if (c->slab) return fail(GA_E_STATE, "slab contexts use ga_slab_fill_launch");
    if ((flags & GA_FILL_FULL) && !full_out) return fail(GA_E_ARG, "GA_FILL_FULL needs full_out");
    if (int r = enqueue_fill(c, flags)) return r;
    return finish_fill(c, cost_out, (flags & GA_FILL_FULL) ? full_out : nullptr);
}

int ga_problem_set_cells(ga_ctx* c, const int32_t* cells, int64_t* cost_out) {
    if (int r = check_ctx(c)) return r;
    if (!c->loaded) return fail(GA_E_STATE, "no problem loaded");
    if (c->slab) return fail(GA_E_STATE, "slab contexts fill their own cells");
    if (!cells || !cost_out) return fail(GA_E_ARG, "null argument");
    const int64_t m = c->m, n = c->n;
    if ((m + 1) * (n + 1) > (int64_t)64 << 20) return fail(GA_E_RANGE, "ga_problem_set_cells is for small problems");
    c->TC = (int)((m + ga::FROWS - 1) / ga::FROWS) * c->CB;
    HIPCHK(c->tb.ensure((size_t)((n + 63) / 64) * c->TC * 1024));
    HIPCHK(c->full.ensure(sizeof(int) * 3 * (m + 1) * (n + 1)));
    HIPCHK(hipMemcpyAsync(c->full.p, cells, sizeof(int) * 3 * (m + 1) * (n + 1), hipMemcpyHostToDevice, c->stream));
    ga::launch_tb_from_cells(c->stream, c->full.as<int>(), (int)m, (int)n, c->o, c->CB, c->TC, c->tb.as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    const int32_t* last = cells + 3 * (m * (n + 1) + n);
    *cost_out = std::min(std::min(last[0], last[1]), last[2]);  // min(dp_array[m][n]) (globaligner.py:425)
    c->filled_tb = true;
    return GA_OK;
}

int ga_problem_traceback(ga_ctx* c, uint32_t* mt_state, const char* a_chr, const char* b_chr, char* oa, char* om,
                         char* ob, int64_t cap, int64_t* out_len, int32_t* tb_status) {
    if (int r = check_ctx(c)) return r;
    if (!c->filled_tb) return fail(GA_E_STATE, "traceback needs a GA_FILL_TRACEBACK fill first");
    if (!mt_state || !a_chr || !b_chr || !oa || !om || !ob || !out_len || !tb_status) return fail(GA_E_ARG, "null argument");
    RngTable R;
    build_rng(mt_state, c->m + c->n + 1, R);
    if (int r = run_walk(c, R.tab.data(), (int64_t)R.tab.size(), WalkStart{c->m, c->n, 0, 0, 0, 1})) return r;
    return finish_walk(c, R, mt_state, a_chr, b_chr, oa, om, ob, cap, out_len, tb_status);
}

int ga_problem_align(ga_ctx* c, uint32_t* mt_state, const char* a_chr, const char* b_chr, char* oa, char* om,
                     char* ob, int64_t cap, int64_t* out_len, int32_t* tb_status, int64_t* cost_out) {
    if (int r = check_ctx(c)) return r;
    if (c->slab) return fail(GA_E_STATE, "slab contexts use ga_slab_fill_launch");
    if (!mt_state || !a_chr || !b_chr || !oa || !om || !ob || !out_len || !tb_status) return fail(GA_E_ARG, "null argument");
    c->rc_used = false;
    if (rc_eligible(c)) {
        const int r = rc_align(c, mt_state, a_chr, b_chr, oa, om, ob, cap, out_len, tb_status, cost_out);
        // checkpoints that do not fit this device (refused before anything was enqueued, or an allocation that
        // failed, after which the recompute buffers are released): the banded / stored-words paths below
        if (r != GA_E_NOMEM) return r;
        c->rc_used = false;
    }
    if (const int64_t Bh = band_rows(c)) return banded_align(c, Bh, mt_state, a_chr, b_chr, oa, om, ob, cap, out_len,
                                                             tb_status, cost_out);
    const double t0 = now_ms();
    if (int r = enqueue_fill(c, GA_FILL_TRACEBACK)) return r;
    // the tie-break table is built on the host while the device fills
    RngTable R;
    const double t1 = now_ms();
    build_rng(mt_state, c->m + c->n + 1, R);
    c->rng_ms = (float)(now_ms() - t1);
    if (std::min(c->m, c->n) >= 256 && !c->knob("GA_WALK_NOSTREAM")) {
        // levels to pinned host memory, decoded while the walk runs (as rc_align; degenerate walks, which
        // need a row or column of the matrix of length 1, keep the plain path)
        WalkBufs wb = ctx_walk_bufs(c);
        if (int r = pinned_walk_levels(c, wb)) return r;
        if (int r = fill_results_async(c)) return r;
        const WalkStart st0{c->m, c->n, 0, 0, 0, 1};
        if (int r = run_walk(c, R.tab.data(), (int64_t)R.tab.size(), st0, 0, -1, false, true, &wb)) return r;
        return streamed_walk_finish(c, R, wb, st0, t0, mt_state, a_chr, b_chr, oa, om, ob, cap, out_len, tb_status,
                                    cost_out);
    }
    if (int r = run_walk(c, R.tab.data(), (int64_t)R.tab.size(), WalkStart{c->m, c->n, 0, 0, 0, 1})) return r;
    if (int r = finish_fill(c, cost_out, nullptr)) return r;
    const int rc = finish_walk(c, R, mt_state, a_chr, b_chr, oa, om, ob, cap, out_len, tb_status);
    c->call_ms = (float)(now_ms() - t0);
    return rc;
}

int ga_problem_align_many(ga_ctx* c, int32_t count, uint32_t* mt_state, const char* a_chr, const char* b_chr,
                          char* oa, char* om, char* ob, int64_t cap, int64_t* out_len, int32_t* tb_status,
                          int64_t* cost_out) {
    if (int r = check_ctx(c)) return r;
    if (c->slab) return fail(GA_E_STATE, "slab contexts use ga_slab_fill_launch");
    if (count < 1) return fail(GA_E_ARG, "count must be >= 1");
    if (!mt_state || !a_chr || !b_chr || !oa || !om || !ob || !out_len || !tb_status || !cost_out)
        return fail(GA_E_ARG, "null argument");
    if (!c->loaded) return fail(GA_E_STATE, "no problem loaded");
    // up to five slots of traceback words (four lane fills in flight + the walked one; GA_PIPE_SLOTS may
    // ask for more): beyond 160 GB of them, one alignment after another
    const bool fits = (int64_t)5 * ((c->n + 63) / 64) * 64 * c->m * c->CB <= ((int64_t)160 << 30);
    if (count == 1 || band_rows(c) > 0 || !fits) {
        // one alignment, or banded tracebacks (whose band fills hold every CU): one after another
        const double t0 = now_ms();
        float fs = 0.f, ws = 0.f, rs = 0.f;
        for (int k = 0; k < count; k++) {
            if (int r = ga_problem_align(c, mt_state, a_chr, b_chr, oa + (size_t)k * cap, om + (size_t)k * cap,
                                         ob + (size_t)k * cap, cap, &out_len[k], &tb_status[k], &cost_out[k]))
                return r;
            fs += c->fill_ms;
            ws += c->walk_ms;
            rs += c->rng_ms;
        }
        c->fill_ms = fs / count;
        c->walk_ms = ws / count;
        c->rng_ms = rs / count;
        c->call_ms = (float)(now_ms() - t0);
        return GA_OK;
    }
    return align_many(c, count, mt_state, a_chr, b_chr, oa, om, ob, cap, out_len, tb_status, cost_out);
}

// ---------------------------------------------------------------- slabs
int ga_problem_set_slab(ga_ctx* c, const uint8_t* a, int64_t m, const uint8_t* b, int64_t n, const ga_costs* cs,
                        int64_t col_begin, int64_t col_end) {
    if (int r = check_ctx(c)) return r;
    c->slab = true;
    c->halo_in_ext = c->halo_out_ext = nullptr;
    c->in_prog_ext = c->out_prog_ext = nullptr;
    c->walk_rng_ready = false;
    if (int r = load_problem(c, a, m, b, n, cs, nullptr, nullptr, col_begin, col_end)) return r;
    HIPCHK(c->halo_in.ensure(sizeof(int2) * (m + 1)));
    if (!c->prog_host) {
        void* hp = nullptr;
        HIPCHK(hipHostMalloc(&hp, 256, hipHostMallocMapped | hipHostMallocCoherent));
        c->prog_host = static_cast<uint32_t*>(hp);
        void* dp = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dp, hp, 0));
        c->prog_dev = static_cast<uint32_t*>(dp);
    }
    std::memset(c->prog_host, 0, 256);
    return GA_OK;
}

int ga_slab_bind_halos(ga_ctx* c, void* halo_in, void* halo_out) {
    if (int r = check_ctx(c)) return r;
    if (!c->slab) return fail(GA_E_STATE, "not a slab context");
    c->halo_in_ext = static_cast<int2*>(halo_in);
    c->halo_out_ext = static_cast<int2*>(halo_out);
    // bound halos go with the context's own (host-relayed) progress words, not a link's
    c->in_prog_ext = c->out_prog_ext = nullptr;
    return GA_OK;
}

// the right slab's side of a link: its left edge (m + 1 int2 rows) + progress word in uncached memory on
// its own GPU, bound as its halo_in / in_prog; the word zeroed (before any writer is launched)
static int link_alloc(ga_ctx* right, uint8_t** base_out) {
    HIPCHK(hipSetDevice(right->device));
    const size_t hbytes = sizeof(int2) * (size_t)(right->m + 1);
    right->link.uncached = true;
    HIPCHK(right->link.ensure(hbytes + 256));
    uint8_t* base = right->link.as<uint8_t>();
    auto* prog = reinterpret_cast<uint32_t*>(base + hbytes);
    HIPCHK(hipMemset(prog, 0, 256));
    right->halo_in_ext = reinterpret_cast<int2*>(base);
    right->in_prog_ext = prog;
    *base_out = base;
    return GA_OK;
}

int ga_slab_link(ga_ctx* left, ga_ctx* right) {
    if (int r = check_ctx(left)) return r;
    if (int r = check_ctx(right)) return r;
    if (left == right || !left->slab || !right->slab) return fail(GA_E_STATE, "ga_slab_link needs two slab contexts");
    if (left->m != right->m || left->col0 + left->n != right->col0)
        return fail(GA_E_ARG, "ga_slab_link: the slabs are not neighbours of one problem");
    if (left->device != right->device) {
        // left's fill stores into right's memory
        if (int r = ga_enable_peer_access(left->device, right->device)) return r;
    }
    uint8_t* base = nullptr;
    if (int r = link_alloc(right, &base)) return r;
    left->halo_out_ext = reinterpret_cast<int2*>(base);
    left->out_prog_ext = reinterpret_cast<uint32_t*>(base + sizeof(int2) * (size_t)(right->m + 1));
    return GA_OK;
}

int ga_slab_link_export(ga_ctx* right, void* handle_out) {
    if (int r = check_ctx(right)) return r;
    if (!handle_out) return fail(GA_E_ARG, "null argument");
    if (!right->slab || right->col0 == 0) return fail(GA_E_STATE, "ga_slab_link_export needs a slab with a left neighbour");
    uint8_t* base = nullptr;
    if (int r = link_alloc(right, &base)) return r;
    hipIpcMemHandle_t h;
    HIPCHK(hipIpcGetMemHandle(&h, base));
    std::memcpy(handle_out, &h, sizeof(h));
    return GA_OK;
}

int ga_slab_link_import(ga_ctx* left, const void* handle) {
    if (int r = check_ctx(left)) return r;
    if (!handle) return fail(GA_E_ARG, "null argument");
    if (!left->slab || left->col0 + left->n >= left->n_global)
        return fail(GA_E_STATE, "ga_slab_link_import needs a slab with a right neighbour");
    if (!left->peer_link || std::memcmp(left->peer_handle, handle, sizeof(left->peer_handle)) != 0) {
        if (left->peer_link) (void)hipIpcCloseMemHandle(left->peer_link);
        left->peer_link = nullptr;
        hipIpcMemHandle_t h;
        std::memcpy(&h, handle, sizeof(h));
        void* p = nullptr;
        HIPCHK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        left->peer_link = p;
        std::memcpy(left->peer_handle, handle, sizeof(left->peer_handle));
    }
    auto* base = static_cast<uint8_t*>(left->peer_link);
    left->halo_out_ext = reinterpret_cast<int2*>(base);
    left->out_prog_ext = reinterpret_cast<uint32_t*>(base + sizeof(int2) * (size_t)(left->m + 1));
    return GA_OK;
}

int ga_enable_peer_access(int device, int peer) {
    if (device == peer) return GA_OK;
    int can = 0;
    HIPCHK(hipDeviceCanAccessPeer(&can, device, peer));
    if (!can) return fail(GA_E_HIP, "device " + std::to_string(device) + " cannot access device " + std::to_string(peer));
    HIPCHK(hipSetDevice(device));
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
        return fail(GA_E_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
    (void)hipGetLastError();  // clear a sticky "already enabled"
    return GA_OK;
}

int ga_slab_buffers(ga_ctx* c, void** halo_in, uint32_t** halo_in_prog, void** halo_out, uint32_t** halo_out_prog) {
    if (int r = check_ctx(c)) return r;
    if (!c->slab) return fail(GA_E_STATE, "not a slab context");
    if (halo_in) *halo_in = c->halo_in_ext ? (void*)c->halo_in_ext : c->halo_in.p;
    if (halo_in_prog) *halo_in_prog = c->prog_host;
    if (halo_out)
        *halo_out = c->halo_out_ext ? (void*)c->halo_out_ext
                                    : (void*)(c->hand.as<int2>() + (size_t)(c->nslabs - 1) * (c->m + 1));
    if (halo_out_prog) *halo_out_prog = c->prog_host + 1;
    return GA_OK;
}

int ga_slab_fill_launch(ga_ctx* c, int32_t flags) {
    if (int r = check_ctx(c)) return r;
    if (!c->slab) return fail(GA_E_STATE, "not a slab context");
    __atomic_store_n(&c->prog_host[0], 0u, __ATOMIC_SEQ_CST);
    __atomic_store_n(&c->prog_host[1], 0u, __ATOMIC_SEQ_CST);
    c->rc_used = false;
    if ((flags & GA_FILL_TRACEBACK) && rc_slab_eligible(c)) {
        // the slab's traceback by recompute: checkpoints instead of m * n words
        if (int r = rc_fill(c)) return r;
        c->filled_tb = true;
        return GA_OK;
    }
    return enqueue_fill(c, flags & GA_FILL_TRACEBACK);
}

int ga_slab_fill_finish(ga_ctx* c, int64_t* cost_out) {
    if (int r = check_ctx(c)) return r;
    return finish_fill(c, cost_out, nullptr);
}

int ga_slab_walk_prepare(ga_ctx* c, const uint32_t* mt_state) {
    if (int r = check_ctx(c)) return r;
    if (!mt_state) return fail(GA_E_ARG, "null argument");
    const double t0 = now_ms();
    build_rng(mt_state, c->m + c->n_global + 1, c->walk_rng);
    c->rng_ms = (float)(now_ms() - t0);
    c->walk_rng_ready = true;
    return GA_OK;
}

int ga_slab_walk(ga_ctx* c, ga_walk_state* st, const char* a_chr, const char* b_chr, char* oa, char* om, char* ob,
                 int64_t cap, int64_t* out_len) {
    if (int r = check_ctx(c)) return r;
    if (!st || !a_chr || !b_chr || !oa || !om || !ob || !out_len) return fail(GA_E_ARG, "null argument");
    if (!c->filled_tb) return fail(GA_E_STATE, "slab walk needs a GA_FILL_TRACEBACK fill first");
    if (!c->walk_rng_ready) return fail(GA_E_STATE, "call ga_slab_walk_prepare first");
    *out_len = 0;
    if (st->reason >= 0 && st->reason != 5) return GA_OK;  // the walk already ended to the right
    if (st->j != c->col0 + c->n) return fail(GA_E_ARG, "walk state is not at this slab's right edge");
    if (st->i < 1 || st->i > c->m) return fail(GA_E_ARG, "walk row out of range");
    WalkStart ws{st->i, st->j, st->D, st->h, st->L, st->first};
    int reason = 0;
    int64_t len = 0;
    if (c->rc_used) {
        WalkBufs wb = ctx_walk_bufs(c);
        const int64_t ntab = (int64_t)c->walk_rng.tab.size();
        HIPCHK(hipMemcpyAsync(wb.rng, c->walk_rng.tab.data(), sizeof(uint32_t) * ntab, hipMemcpyHostToDevice, wb.stream));
        if (int r = rc_walk_launch(c, ntab, ws, wb)) return r;
        if (int r = walk_segment(c, ws, reason, a_chr, b_chr, oa, om, ob, cap, len, &wb)) return r;
        if (reason == 7) return fail(GA_E_TIMEOUT, "recompute walk: a tile was never recomputed");
    } else {
        if (int r = run_walk(c, c->walk_rng.tab.data(), (int64_t)c->walk_rng.tab.size(), ws)) return r;
        if (int r = walk_segment(c, ws, reason, a_chr, b_chr, oa, om, ob, cap, len)) return r;
    }
    st->i = ws.i;
    st->j = ws.j;
    st->D = ws.D;
    st->h = ws.h;
    st->L = ws.L;
    st->first = ws.first;
    st->reason = reason;
    *out_len = len;
    return GA_OK;
}

int ga_slab_mt_state(ga_ctx* c, int64_t D, uint32_t* mt_out) {
    if (int r = check_ctx(c)) return r;
    if (!mt_out) return fail(GA_E_ARG, "null argument");
    if (!c->walk_rng_ready) return fail(GA_E_STATE, "call ga_slab_walk_prepare first");
    state_after(c->walk_rng, D, mt_out);
    return GA_OK;
}

int ga_stream_wait_ge(void* stream, uint32_t* prog, uint32_t value) {
    HIPCHK(hipStreamWaitValue32((hipStream_t)stream, prog, value, hipStreamWaitValueGte, 0xffffffffu));
    return GA_OK;
}

int ga_stream_write(void* stream, uint32_t* prog, uint32_t value) {
    HIPCHK(hipStreamWriteValue32((hipStream_t)stream, prog, value, 0));
    return GA_OK;
}

void* ga_ctx_stream(ga_ctx* c) { return c ? (void*)c->stream : nullptr; }

int ga_ctx_wait_stream(ga_ctx* c, void* stream) {
    if (int r = check_ctx(c)) return r;
    HIPCHK(hipEventRecord(c->ev_dep, (hipStream_t)stream));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_dep, 0));
    return GA_OK;
}

int ga_ctx_stream_priority(ga_ctx* c, int* priority) {
    if (!c || !priority) return fail(GA_E_ARG, "null argument");
    *priority = c->priority;
    return GA_OK;
}

int ga_last_kernel_ms(ga_ctx* c, float* fill_ms, float* walk_ms) {
    if (!c) return fail(GA_E_ARG, "null context");
    if (fill_ms) *fill_ms = c->fill_ms;
    if (walk_ms) *walk_ms = c->walk_ms;
    return GA_OK;
}

// Diagnostics (not in the public header): the walk's tile-need records (ti, tj, D, wait ticks) x 8192.
int ga_debug_walk_tiles(ga_ctx* c, unsigned* out) {
    if (!c || !out) return fail(GA_E_ARG, "null argument");
    if (!c->wdbg.p) return fail(GA_E_STATE, "no diagnostic walk ran");
    HIPCHK(hipMemcpy(out, c->wdbg.p, sizeof(unsigned) * 4 * 8192, hipMemcpyDeviceToHost));
    return GA_OK;
}

// Diagnostics (not in the public header): per-stripe s_memrealtime stamps of the next fills.
int ga_debug_stamps(ga_ctx* c, int enable, unsigned long long* out, int64_t cap) {
    if (!c) return fail(GA_E_ARG, "null context");
    c->dbg_on = enable != 0;
    if (out && c->dbg.p) {
        const int64_t nb = std::min<int64_t>(cap, ga::LK_DBG_WORDS * (int64_t)c->nstripes);
        HIPCHK(hipMemcpy(out, c->dbg.p, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost));
    }
    return GA_OK;
}

// Diagnostics: the fill geometry of the loaded problem {T, nstripes, nwc, nslabs}.
int ga_debug_geometry(ga_ctx* c, int32_t* out4) {
    if (!c || !out4) return fail(GA_E_ARG, "null argument");
    out4[0] = c->T;
    out4[1] = c->nstripes;
    out4[2] = c->nwc;
    out4[3] = c->nslabs;
    return GA_OK;
}

// Diagnostics: the kernel of the last enqueued fill (0 row scan, 1 per-column anti-diagonal, 2 lane-skewed)
// and its geometry {T, nstripes, nwc, nslabs}.
int ga_debug_fill_kind(ga_ctx* c, int32_t* out5) {
    if (!c || !out5) return fail(GA_E_ARG, "null argument");
    out5[0] = c->rc_used ? 3 : c->lane ? 2 : c->diag ? 1 : 0;  // 3: the recompute walk's lane fill
    out5[1] = c->T;
    out5[2] = c->nstripes;
    out5[3] = c->nwc;
    out5[4] = c->nslabs;
    return GA_OK;
}

// CPU-only check of the tie-break table (tests): entries for `steps` dispatches from
// the 625-word state, and the state after the first D of them.
int ga_debug_rng(const uint32_t* state, int64_t steps, uint32_t* tab_out, int64_t D, uint32_t* state_out,
                 double* ms_out) {
    if (!state || !tab_out || !state_out || D < 0 || D > steps) return fail(GA_E_ARG, "bad argument");
    RngTable R;
    const double t0 = now_ms();
    build_rng(state, steps, R);
    if (ms_out) *ms_out = now_ms() - t0;
    std::memcpy(tab_out, R.tab.data(), sizeof(uint32_t) * steps);
    state_after(R, D, state_out);
    return GA_OK;
}

// CPU-only check of the resumable table stream (tests): entries for `steps` dispatches built in
// `chunk`-sized extensions, and the state after the first D of them.
int ga_debug_rng_chunked(const uint32_t* state, int64_t steps, int64_t chunk, uint32_t* tab_out, int64_t D,
                         uint32_t* state_out) {
    if (!state || !tab_out || !state_out || D < 0 || D > steps || chunk < 1) return fail(GA_E_ARG, "bad argument");
    RngTable R;
    R.start(state);
    for (int64_t b = chunk; b < steps + chunk; b += chunk) R.extend(std::min(b, steps));
    std::memcpy(tab_out, R.tab.data(), sizeof(uint32_t) * steps);
    state_after(R, D, state_out);
    return GA_OK;
}

// out6 = {tile wait spins, tiles entered, tile-wait ticks, ring-wait ticks, walker ticks (100 MHz),
//         walker shader clocks / 16, loader busy ticks, tiles loaded}
// Diagnostics of the last recompute walk: {blocks recomputed, their summed time in 100 MHz ticks,
// recompute workers, checkpoint spacing}.
int ga_debug_rc(ga_ctx* c, unsigned* out4) {
    if (!c || !out4) return fail(GA_E_ARG, "null argument");
    if (!c->rc_pos.p) return fail(GA_E_STATE, "no recompute walk ran");
    HIPCHK(hipMemcpy(out4, c->rc_pos.p, sizeof(unsigned) * 4, hipMemcpyDeviceToHost));
    return GA_OK;
}

// How the library was built: bit 0 set in an experiments build (make EXPERIMENTS=1: the measured-and-dropped paths,
// e.g. the tie-to-tie walk, and every GA_* variable read from the environment).
int ga_build_flags(int32_t* flags) {
    if (!flags) return fail(GA_E_ARG, "null argument");
#ifdef GA_EXPERIMENTS
    flags[0] = 1;
#else
    flags[0] = 0;
#endif
    return GA_OK;
}

// diagnostics / CPU tests: the jump workers' LUT for gap open o (4096 words)
int ga_debug_jump_lut(int32_t o, uint32_t* out4096) {
    if (!out4096 || o < 0 || o > 14) return fail(GA_E_ARG, "bad argument");
    ga::jump_lut_build(o, out4096);
    return GA_OK;
}

// diagnostics: the recompute walk's tile / entry cache (rc_tb) as the last walk left it
int ga_debug_rc_cache(ga_ctx* c, void* out, int64_t bytes) {
    if (!c || !out) return fail(GA_E_ARG, "null argument");
    if (!c->rc_tb.p) return fail(GA_E_STATE, "no recompute walk ran");
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, c->rc_tb.p, std::min<size_t>((size_t)bytes, c->rc_tb.cap), hipMemcpyDeviceToHost));
    return GA_OK;
}

// which walk the last traceback ran: 0 the walk of stored words, 1 the recompute walk of traceback words, 2 the
// tie-to-tie recompute walk (jump entries)
int ga_debug_walk_kind(ga_ctx* c, int32_t* out) {
    if (!c || !out) return fail(GA_E_ARG, "null argument");
    out[0] = c->rc_used ? (c->rc_jump ? 2 : 1) : 0;
    return GA_OK;
}

int ga_debug_walk_jump(ga_ctx* c, int* out3) {
    if (!c || !out3) return fail(GA_E_ARG, "null argument");
    for (int q = 0; q < 3; q++) out3[q] = c->walk_jump_diag[q];
    return GA_OK;
}

int ga_debug_walk(ga_ctx* c, int* out5) {
    if (!c || !out5) return fail(GA_E_ARG, "null argument");
    out5[0] = c->walk_waits;
    out5[1] = c->walk_tiles;
    out5[2] = c->walk_t_tile;
    out5[3] = c->walk_t_ring;
    out5[4] = c->walk_t_total;
    out5[5] = c->walk_c_total;
    out5[6] = c->walk_load_ticks;
    out5[7] = c->walk_load_count;
    return GA_OK;
}

int ga_last_timings(ga_ctx* c, float* out4) {
    if (!c || !out4) return fail(GA_E_ARG, "null argument");
    out4[0] = c->fill_ms;
    out4[1] = c->walk_ms;
    out4[2] = c->rng_ms;
    out4[3] = c->call_ms;
    return GA_OK;
}

}  // extern "C"

namespace ga {
// The rank sets of a cell from its saturated differences (as ga_walk.h sets_from_code): per level the v_perm
// selector of the candidate its singleton move takes (bytes 4,5 of {src0, Pu} = Pd (diag), 6,7 = Pl (left), 0,1 = Pu
// (up)) or 0x0c0c (a zero half) for a tie, and the tie word ((2S - 2 + 14*(a != b)) << 2) the walker reads at a tie
void jump_lut_build(int o, uint32_t* out) {
    const unsigned uo = (unsigned)o;
    for (unsigned idx = 0; idx < 1024; idx++) {
        const unsigned fx = idx & 15u, fy = (idx >> 4) & 15u, zM = ((idx >> 8) & 1u) ^ 1u, mm = (idx >> 9) & 1u;
        const unsigned zX = fx == 0, zY = fy == 0, leX = fx <= uo, geX = fx >= uo, leY = fy <= uo, geY = fy >= uo;
        const unsigned S[3] = {zM | (zX << 1) | (zY << 2), (zM & geX) | (leX << 1) | ((zY & geX) << 2),
                               (zM & geY) | ((zX & geY) << 1) | (leY << 2)};
        unsigned sel[3], tw[3];
        for (int L = 0; L < 3; L++) {
            const unsigned x = S[L];
            sel[L] = x == 1u ? 0x0504u : x == 2u ? 0x0706u : x == 4u ? 0x0100u : 0x0c0cu;
            tw[L] = (x == 1u || x == 2u || x == 4u) ? 0u : x ? ((2u * x - 2u + 14u * mm) << 2) : 0x7cu;  // (empty: never walked)
        }
        out[4 * idx] = sel[0] | (sel[1] << 16);
        out[4 * idx + 1] = sel[2] | (0x0c0cu << 16);
        out[4 * idx + 2] = tw[0] | (tw[1] << 16);
        out[4 * idx + 3] = tw[2];
    }
}
}  // namespace ga
