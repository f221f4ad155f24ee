// Microbenchmark: a traceback walker built on precomputed next-state words, one wave.
//
// Cells are addressed by their coordinates mod 8 (lane = (i & 7) * 8 + (j & 7)), so a window anchored
// anywhere holds each cell it covers at a fixed lane and a move never leaves the lane space.  For the
// steps of group g+3 (two steps per group), the window anchored at the walker's position at group g
// covers every reachable cell (moves 6 and 7).  Per lane and step k the word P_k holds, for each
// entering level L at byte L, the next state (next lane | L' << 6); the step is then
//     v = readlane(P_k, ix);  ix = v >> sL;  sL = (ix >> 3) & 0x18   (the last two off the chain)
// P_k = perm(F, F, perm(rec_k.hi, rec_k.lo, selw) | constw): rec_k is dispatch k's 8-byte tie record
// (the level picked for each tie set, match / mismatch), selw / constw the cell's per-level selectors
// (a LUT keyed by the cell), F the lane's three next states.  The window read (group g), the LUT read
// (g+1) and the perms (g+2) are software-pipelined so no LDS wait lands on the chain.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int TQ = 128;  // torus side (a timing stand-in for the walk's 256 x 256 tile torus)

__global__ void __launch_bounds__(64) walk_next(long long* out, unsigned* sink, int ngroups) {
    __shared__ unsigned short torus[TQ * TQ];
    __shared__ unsigned long long lut[1024];
    __shared__ unsigned long long rec[2048];
    __shared__ unsigned logb[64];
    const int lane = threadIdx.x;
    for (int q = lane; q < TQ * TQ; q += 64) torus[q] = (unsigned short)((q * 2654435761u) >> 22);
    for (int q = lane; q < 1024; q += 64) {
        unsigned long long s = 0, c = 0;
        for (int L = 0; L < 3; L++) {
            const unsigned h = (q * 7 + L * 13) * 2654435761u;
            if (h & 0x100) s |= (unsigned long long)((h >> 9) & 7) << (8 * L);  // a tie set: record byte
            else {
                s |= 12ull << (8 * L);                                  // a single level: 0x00 ...
                c |= (unsigned long long)((h >> 12) % 3) << (8 * L);    // ... OR-ed with the level
            }
        }
        s |= 12ull << 24;
        lut[q] = s | (c << 32);
    }
    for (int q = lane; q < 2048; q += 64) {
        unsigned long long v = 0;
        for (int b = 0; b < 8; b++) v |= (unsigned long long)(((q * 31 + b * 7) * 2654435761u >> 20) % 3) << (8 * b);
        rec[q] = v;
    }
    __syncthreads();
    const int rr = lane >> 3, cc = lane & 7;
    // F: next state per level (M: up-left, X: left, Y: up), level in bits 6-7
    const unsigned nM = (((rr - 1) & 7) << 3) | ((cc - 1) & 7), nX = (rr << 3) | ((cc - 1) & 7), nY = (((rr - 1) & 7) << 3) | cc;
    const unsigned F = nM | ((nX | 64u) << 8) | ((nY | 128u) << 16);
    int i = 1 << 20, j = 1 << 20;
    unsigned ix = (unsigned)(((i & 7) << 3) | (j & 7)), sL = 0, D = 0, logv = 0, slot = 0;
    // pipeline registers: the window cell read last group (LUT this group), the LUT value and the two tie
    // records read last group (P words this group, for the next group)
    unsigned cell1 = 0;
    unsigned long long lut1 = 0, r1a = 0, r1b = 0;
    unsigned P[2][2] = {{F, F}, {F, F}};
    auto window = [&](int pi, int pj) -> unsigned {
        const unsigned dr = (unsigned)((pi & 7) - rr) & 7u, dc = (unsigned)((pj & 7) - cc) & 7u;
        const unsigned a = ((unsigned)(pi - 1 - (int)dr) & (TQ - 1)) * TQ + ((unsigned)(pj - 1 - (int)dc) & (TQ - 1));
        return torus[a];
    };
    auto pword = [&](unsigned long long lv, unsigned long long r) -> unsigned {
        const unsigned Ls = __builtin_amdgcn_perm((unsigned)(r >> 32), (unsigned)r, (unsigned)lv) | (unsigned)(lv >> 32);
        return __builtin_amdgcn_perm(F, F, Ls);
    };
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int g = 0; g < ngroups; g += 2) {
#pragma unroll
        for (int u = 0; u < 2; u++) {
            // group g+u: reads for later groups (window for g+u+3, LUT of last group's window, the tie
            // records of group g+u+2), then the P words of group g+u+1 from last group's reads
            const unsigned long long lut_now = lut[cell1 & 1023u];
            const unsigned cell_now = window(i, j);
            const unsigned long long ra = rec[(D + 4) & 2047], rb = rec[(D + 5) & 2047];
            P[(u + 1) & 1][0] = pword(lut1, r1a);
            P[(u + 1) & 1][1] = pword(lut1, r1b);
            cell1 = cell_now;
            lut1 = lut_now;
            r1a = ra;
            r1b = rb;
            const unsigned ri = ix;
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const unsigned v = (unsigned)__builtin_amdgcn_readlane((int)P[u][k], (int)ix);
                const unsigned f = v >> sL;
                ix = f;
                sL = (f >> 3) & 0x18u;
                asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(logv) : "s"(ix), "s"(slot) : "m0");
                slot = (slot + 1) & 63u;
            }
            i -= (int)(((ri >> 3) - (ix >> 3)) & 7u);
            j -= (int)((ri - ix) & 7u);
            D += 2;
        }
        if (slot == 0) logb[lane] = logv;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[0] = t1 - t0;
    sink[lane] = ix + (unsigned)i + (unsigned)j + logv + logb[lane];
}

int main() {
    long long* d;
    unsigned* s;
    (void)hipMalloc(&d, 8);
    (void)hipMalloc(&s, 64 * 4);
    const int ng = 2 * 30000;
    walk_next<<<1, 64>>>(d, s, ng);
    walk_next<<<1, 64>>>(d, s, ng);
    (void)hipDeviceSynchronize();
    long long h = 0;
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("next-state walker: %.1f cyc per step (s_memtime units, as walk_chain)\n", (double)h / (2.0 * ng));
    return 0;
}
