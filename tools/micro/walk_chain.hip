// Microbenchmark: latency of the traceback walker's per-step dependent chain on gfx950 (one wave):
// v_readlane of a window cell -> scalar ops -> the next readlane's lane index.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V>
__global__ void chain(long long* out, int* sink, int n) {
    const int lane = threadIdx.x & 63;
    int win = (lane * 37 + 11) & 0x7fff;
    unsigned t = 0x9e3779b9u, idx = 0, L8 = 0, acc = 0, win2 = 0;
    if (V == 4)  // a window image in s[64:95] (the compiler is told they are clobbered)
        asm volatile(".irp r, 64,65,66,67,68,69,70,71,72,73,74,75,76,77,78,79,80,81,82,83,84,85,86,87,88,89,90,91,92,93,94,95\n\t"
                     "s_mov_b32 s\\r, 0x00030002\n\t.endr" ::: "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71",
                     "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85",
                     "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < n; k++) {
        if (V == 0) {  // the walker's step: readlane, field of the entering level, tie-break bits, move
            const unsigned v = (unsigned)__builtin_amdgcn_readlane(win, (int)(idx & 63));
            const unsigned lvl = (t >> ((v >> L8) & 31u)) & 3u;
            L8 = lvl << 3;
            idx += (0x080109u >> L8) & 0xffu;
            acc += lvl;
        } else if (V == 3) {  // table pre-shifted by 3 in 64 bits: the level's bit offset comes out masked
            const unsigned v = (unsigned)__builtin_amdgcn_readlane(win, (int)(idx & 63));
            const unsigned long long t64 = (unsigned long long)t << 3;
            L8 = (unsigned)(t64 >> ((v >> L8) & 63u)) & 0x18u;
            idx += 0x080109u >> L8;
            acc += L8;
        } else if (V == 1) {  // readlane -> one scalar add -> readlane
            const unsigned v = (unsigned)__builtin_amdgcn_readlane(win, (int)(idx & 63));
            idx += v;
        } else if (V == 4) {  // the step with the window in SGPRs s[64:95] (two 16-bit cells per dword),
            // read by s_movrels_b32 with M0 = dword index: no VALU -> SALU round trip on the chain
            unsigned v;
            asm volatile(
                "s_lshr_b32 m0, %1, 1\n\t"
                "s_movrels_b32 %0, s64\n\t"
                : "=s"(v) : "s"(idx & 63u) : "m0");
            v = (idx & 1u) ? (v >> 16) : (v & 0xffffu);
            const unsigned long long t64 = (unsigned long long)t << 3;
            L8 = (unsigned)(t64 >> ((v >> L8) & 63u)) & 0x18u;
            idx += 0x080109u >> L8;
            acc += L8;
        } else if (V == 5) {  // precomputed next-state words: readlane -> one shift -> readlane (the level's
            // field offset comes off the chain: (f >> 3) & 0x18 while the next readlane is in flight)
            const unsigned v = (unsigned)__builtin_amdgcn_readlane(win, (int)idx);
            const unsigned f = v >> L8;
            idx = f;
            L8 = (f >> 3) & 0x18u;
            acc += L8;
        } else if (V == 6) {  // V5 plus the per-step share of the next window's precompute (8 VALU, independent)
            const unsigned v = (unsigned)__builtin_amdgcn_readlane(win, (int)idx);
            unsigned x = (unsigned)win;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                x = __builtin_amdgcn_ubfe(t, x & 31u, 2u) | (x << 8);
                x = __builtin_amdgcn_perm(x, (unsigned)lane, x);
            }
            win2 ^= x;
            const unsigned f = v >> L8;
            idx = f;
            L8 = (f >> 3) & 0x18u;
            acc += L8;
            t = t * 3u + 1u;
        } else if (V == 7) {  // round 5: 64-bit table of lane deltas (up 8, left 17, diag 25) whose low 5 bits are
            // also the next cell's field offset: readlane -> field offset -> table -> index (3 SALU), the level
            // packed off the chain (bfe + lshl2_add)
            const unsigned v = (unsigned)__builtin_amdgcn_readlane(win, (int)idx);
            const unsigned s = v >> L8;
            const unsigned long long t64 = ((unsigned long long)t << 32) | t;
            const unsigned Vx = (unsigned)(t64 >> (s & 63u));
            idx += Vx;
            L8 = Vx;
            acc = acc * 4u + __builtin_amdgcn_ubfe(Vx, 3u, 2u);
        } else if (V == 2) {  // eight dependent scalar ops (no readlane)
            idx = ((idx >> 3) ^ t) + 1u;
            idx = (idx >> (idx & 7u)) & 0xffffu;
            idx = idx * 5u + 3u;
            idx = (idx >> 1) + (idx & 1u);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = (int)(idx + acc + win2);
}

template <typename F>
double run(F f) {
    long long* d; int* s;
    (void)hipMalloc(&d, 256 * 8);
    (void)hipMalloc(&s, 256 * 64 * 4);
    const int n = 1 << 16;
    f<<<1, 64>>>(d, s, n);
    f<<<1, 64>>>(d, s, n);
    (void)hipDeviceSynchronize();
    long long h = 0;
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    (void)hipFree(d); (void)hipFree(s);
    return (double)h / n;
}

int main() {
    printf("walker step (readlane + 8 SALU): %.1f cyc\n", run(chain<0>));
    printf("readlane -> s_add -> readlane : %.1f cyc\n", run(chain<1>));
    printf("walker step, 64-bit table     : %.1f cyc\n", run(chain<3>));
    printf("8 dependent SALU ops          : %.1f cyc\n", run(chain<2>));
    printf("lane-delta table (3 SALU)     : %.1f cyc\n", run(chain<7>));
    printf("walker step, SGPR window      : %.1f cyc\n", run(chain<4>));
    printf("next-state words (1 SALU)     : %.1f cyc\n", run(chain<5>));
    printf("next-state words + 8 VALU     : %.1f cyc\n", run(chain<6>));
    return 0;
}
