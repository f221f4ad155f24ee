// Microbenchmark: cycles per row of the blocked row (ga_row.h blocked_row, T columns per lane)
// in isolation (register-only inputs), score only and with traceback codes, at 1..4 waves per
// SIMD.  hipcc --offload-arch=gfx950 -O3 -I globalign_amd/csrc tools/micro/row_bench_t.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "ga_row.h"

template <int T, bool TB>
__global__ void rows(long long* out, int* sink, int nrows) {
    const int lane = threadIdx.x & 63;
    int Hprev[T], Yc[T];
    for (int k = 0; k < T; k++) { Hprev[k] = lane * T + k; Yc[k] = lane + 3 + k; }
    uint32_t acc[T][4];
    for (int k = 0; k < T; k++) for (int d = 0; d < 4; d++) acc[k][d] = 0;
    const unsigned op1 = 6;
    const int o = 5;
    int sub[T];
    for (int k = 0; k < T; k++) sub[k] = ((lane + k) & 3) ? 3 : -2;
    int oh = 0, ov = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nrows; r += 16) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
            int eh = r + u, ev = r + 2 * u;
            int a, b;
            ga::blocked_row<T, TB, 1>(Hprev, Yc, eh, ev, sub, o, op1, u, acc, a, b);
            oh += a; ov ^= b;
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    int x = oh + ov;
    for (int k = 0; k < T; k++) x += Hprev[k] + Yc[k] + (int)(acc[k][0] ^ acc[k][3]);
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <typename F>
double run(F kern, int waves, int blocks, int nrows) {
    long long* d; int* s;
    (void)hipMalloc(&d, 16 * blocks * sizeof(long long));
    (void)hipMalloc(&s, blocks * waves * 64 * sizeof(int));
    kern<<<blocks, waves * 64>>>(d, s, nrows);
    kern<<<blocks, waves * 64>>>(d, s, nrows);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * blocks);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int b = 0; b < blocks; b++) for (int w = 0; w < waves; w++) mx = std::max(mx, (double)h[b * 16 + w]);
    (void)hipFree(d); (void)hipFree(s);
    return mx / nrows;
}

int main() {
    const int nrows = 4096;
    struct K { const char* name; void (*f)(long long*, int*, int); int T; };
    std::vector<K> ks = {{"T=1 score", rows<1, false>, 1}, {"T=2 score", rows<2, false>, 2},
                         {"T=4 score", rows<4, false>, 4}, {"T=1 tb", rows<1, true>, 1},
                         {"T=2 tb", rows<2, true>, 2},     {"T=4 tb", rows<4, true>, 4},
                         {"T=8 score", rows<8, false>, 8}};
    for (auto& k : ks) {
        printf("%-10s", k.name);
        for (int w = 1; w <= 4; w++) {
            const double c = run(k.f, 4 * w, 256, nrows);
            printf("  %d w/SIMD: %6.1f cyc/row/wave %5.2f cyc/cell/SIMD", w, c, c / w / (64.0 * k.T));
        }
        printf("\n");
    }
    return 0;
}
