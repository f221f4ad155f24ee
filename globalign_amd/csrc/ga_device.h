// ga_device.h -- types shared by the HIP kernels (ga_kernels.hip) and the host
// library (ga_host.cpp).  See DESIGN.md for the layouts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ga {

constexpr int QPAD = 128;        // query-profile padding (rows) on both sides
constexpr int NW = 7;            // compute waves per fill workgroup (+1 IO wave)
constexpr int RING = 512;        // rows per LDS ring between consecutive waves
constexpr int RMASK = RING - 1;
constexpr int GOUT = 16;         // rows per cross-workgroup publish
constexpr int WR = 128, WC = 128, RW = 512;  // traceback window (rows, cols, dispatches)

struct FillArgs {
    const void* qp;           // [K][qp_stride] sub' (QT)
    long long qp_stride;
    const uint8_t* b;         // n codes
    const int2* top;          // [n+1] (H', h2') of row 0
    const int2* left;         // [m+1] (H', h1') of the slab's left edge
    const unsigned* left_prog;  // rows of `left` available (nullptr: all)
    int2* hand;               // [nslabs][m+1] right edge of each slab
    unsigned* hand_prog;      // [nslabs] rows published
    unsigned* ticket;         // slab ticket
    unsigned* abort_word;
    uint8_t* tb;              // traceback words or nullptr
    int* out_last;            // [4]: H'(m, n_local) and status
    unsigned* edge_prog;      // rows of the right edge published (last slab only; may be null)
    int* full;                // FULL output (shifted M', X', Y') or nullptr
    int m, n, o, nstripes, nslabs, TC;
    unsigned spin_limit, halo_spin_limit;
};

struct WalkArgs {
    const uint8_t* tb;
    int CB, TC;
    const uint8_t* a;
    const uint8_t* b;
    const int* bnd_row;   // 3(n+1) original boundary triples
    const int* bnd_col;   // 3(m+1)
    const uint16_t* rng;  // tie-break bits per dispatch
    long long nrng;
    int m, n, o;
    uint8_t* ops;         // out: chosen level per dispatch
    int* result;          // out: [D, i, j, reason]
};

void launch_qp(hipStream_t s, const uint8_t* a, int m, const int* sub, const int* gh, const int* gv, int K, void* qp,
               long long stride, int qbytes);
void launch_boundary(hipStream_t s, const uint8_t* a, int m, const uint8_t* b, int n, const int* gh, const int* gv,
                     int o, int big, int* GVp, int* GHp, int2* top, int2* left, int* bnd_row, int* bnd_col, int* meta,
                     bool custom);
void launch_fill(hipStream_t s, const FillArgs& p, int CB, int qbytes, bool tb, bool full);
void launch_walk(hipStream_t s, const WalkArgs& w);

}  // namespace ga
