// ga_check.h -- the host's checks of a problem before anything goes to the device (no HIP: built into the engine
// and into the host self-test, ga_host_selftest.cpp, under AddressSanitizer / UBSan).
//
// The reference validates its arguments in Python (start.py:150-353) and computes with unbounded ints; the device
// path computes in int32, so the host also proves that no stored value or intermediate can overflow
// and picks the widths of the query profile and of the traceback word.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "../../include/globalign_amd.h"

// the sentinel, profile and word widths of a checked problem
struct ProblemShape {
    int64_t big = 0;  // (max_cost + 1) * max(m, n) (globaligner.py:777)
    int qbytes = 1;   // query-profile entry: 1 or 2 bytes (sub' = sub - gV - gH)
    int CB = 1;       // traceback word bytes per cell: 1 / 2 / 4 for o + 1 < 8 / 128 / 32768
};

// GA_OK, or GA_E_ARG / GA_E_RANGE with the reason in err.  cb, ce: the column slab [cb, ce) of seq_2 this context
// fills (the whole problem: 0, n_all); row0 / col0: caller-supplied boundary triples (both or neither).
inline int check_problem(const uint8_t* a, int64_t m, const uint8_t* b_all, int64_t n_all, const ga_costs* cs,
                         const int32_t* row0, const int32_t* col0, int64_t cb, int64_t ce, ProblemShape& out,
                         std::string& err) {
    auto fail = [&](int code, const char* msg) {
        err = msg;
        return code;
    };
    if (!a || !b_all || !cs || !cs->sub || !cs->gap_h || !cs->gap_v) return fail(GA_E_ARG, "null argument");
    if (m < 1 || n_all < 1) return fail(GA_E_ARG, "sequences must be non-empty");
    if (cb < 0 || ce > n_all || ce <= cb) return fail(GA_E_ARG, "bad column slab");
    const int K = cs->K;
    if (K < 1 || K > 255) return fail(GA_E_ARG, "alphabet size K must be in [1,255]");
    if (cs->gap_open < 0) return fail(GA_E_ARG, "gap_open cost must be >= 0");
    if ((row0 == nullptr) != (col0 == nullptr)) return fail(GA_E_ARG, "row0 and col0 must be given together");
    for (int64_t i = 0; i < m; i++)
        if (a[i] >= K) return fail(GA_E_ARG, "seq_1 code out of range");
    for (int64_t j = 0; j < n_all; j++)
        if (b_all[j] >= K) return fail(GA_E_ARG, "seq_2 code out of range");
    // int32 range guard: every stored value, shifted or not, and every intermediate (value + o) must
    // stay far from overflow
    int64_t maxabs = 0;
    for (int q = 0; q < K * K; q++) maxabs = std::max<int64_t>(maxabs, std::llabs((long long)cs->sub[q]));
    for (int q = 0; q < K; q++) {
        maxabs = std::max<int64_t>(maxabs, std::llabs((long long)cs->gap_h[q]));
        maxabs = std::max<int64_t>(maxabs, std::llabs((long long)cs->gap_v[q]));
    }
    const int64_t big = ((int64_t)cs->max_cost + 1) * std::max(m, n_all);
    int64_t bmax = std::llabs(big);
    if (row0)
        for (int64_t q = 0; q < 3 * (n_all + 1); q++) bmax = std::max<int64_t>(bmax, std::llabs((long long)row0[q]));
    if (col0)
        for (int64_t q = 0; q < 3 * (m + 1); q++) bmax = std::max<int64_t>(bmax, std::llabs((long long)col0[q]));
    const int64_t bound = bmax + (m + n_all + 2) * (3 * maxabs + (int64_t)cs->gap_open);
    if (4 * bound >= (int64_t)INT32_MAX) return fail(GA_E_RANGE, "problem exceeds the int32 score range of the device path");
    int64_t subp_max = 0;
    for (int x = 0; x < K; x++)
        for (int y = 0; y < K; y++)
            subp_max = std::max<int64_t>(subp_max,
                                         std::llabs((long long)cs->sub[x * K + y] - cs->gap_v[x] - cs->gap_h[y]));
    out.qbytes = subp_max <= 127 ? 1 : subp_max <= 32767 ? 2 : 0;
    if (!out.qbytes) return fail(GA_E_RANGE, "substitution costs exceed the int16 query profile");
    const int o = cs->gap_open;
    out.CB = (o + 1) < 8 ? 1 : (o + 1) < 128 ? 2 : (o + 1) < 32768 ? 4 : 0;
    if (!out.CB) return fail(GA_E_RANGE, "gap_open cost too large for the traceback word");
    out.big = big;
    return GA_OK;
}

// The recompute fill's lean checkpoint store addresses a stripe's right-edge rows through a raw buffer with a 32-bit
// size, (m + 1) * 8 bytes, and drops the stores of lanes that hold no row by offsetting them to 0x7ffffff0, past the
// buffer's end (ga_lane.hip).  Both hold only while the rows (with the per-stripe pad) stay below that offset:
// m < 2^28 - 66.  Longer problems keep the stored-words or banded traceback.
inline bool rc_rows_fit(int64_t m) { return (m + 1 + 64) * 8 < (int64_t)0x7ffffff0; }
