// Microbenchmark: cycles per row of the fill's hand-scheduled row block (ga_row.h) run in
// isolation (register-only inputs), with and without the per-4-row LDS traffic of the
// fill loop, at one and two waves per SIMD.  hipcc --offload-arch=gfx950 -I globalign_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "ga_row.h"

template <int MODE>
__global__ void rows(long long* out, int* sink, int nrows) {
    __shared__ __attribute__((aligned(16))) int lds[4096];
    const int lane = threadIdx.x & 63;
    for (int k = threadIdx.x; k < 4096; k += blockDim.x) lds[k] = k & 7;
    __syncthreads();
    int Hprev = lane, Yc = lane + 3, pM = 1, pX = 2, pY = 3, pH = 0;
    uint32_t acc = 0, qw = 0x01020304u * (lane & 3);
    int eh = 5, ev = 7;
    const unsigned op1 = 6;
    const int o = 5;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nrows; r += 4) {
        if (MODE >= 1) {
            const int4 e = reinterpret_cast<const int4*>(lds)[(r & 255) + (threadIdx.x >> 6) * 0];
            eh = e.x; ev = e.y;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            int M, X, H, Vt, Ycn;
            ga::row_asm<3, 0, false>(Hprev, Yc, eh + u, ev + u, qw, pM, pX, pY, pH, op1, o, 8u * u, acc, M, X, H, Vt, Ycn);
            pM = M; pX = X; pY = Yc; pH = H;
            Yc = Ycn; Hprev = H;
        }
        if (MODE >= 2 && lane == 0) lds[1024 + (r & 1023)] = Hprev;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = Hprev + Yc + (int)acc;
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
    const char* names[] = {"row block only", "+ per-4-row ds_read_b128 edges", "+ lane-0 ds_write per 4 rows"};
    auto fns = std::vector<void (*)(long long*, int*, int)>{rows<0>, rows<1>, rows<2>};
    for (int v = 0; v < 3; v++)
        printf("%-36s 1 wave/SIMD %6.1f cyc/row   2 waves/SIMD %6.1f cyc/row (per wave)\n", names[v],
               run(fns[v], 4, 256, nrows), run(fns[v], 8, 256, nrows));
    return 0;
}
