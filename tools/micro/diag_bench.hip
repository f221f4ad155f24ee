// Microbenchmark: cycles per step of the anti-diagonal fill's 4-step block (ga_row.h diag4_asm)
// in isolation (register-only inputs), and with the per-4-step LDS edge reads / lane-63
// publish of the kernel, at 1..4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "ga_row.h"

template <int MODE>
__global__ void steps(long long* out, int* sink, int nsteps) {
    __shared__ __attribute__((aligned(16))) int lds[4096];
    const int lane = threadIdx.x & 63;
    for (int k = threadIdx.x; k < 4096; k += blockDim.x) lds[k] = k & 7;
    __syncthreads();
    int Hd = lane, H = lane + 1, X = lane + 2, Y = lane + 3;
    uint32_t q = 0x01020304u * (lane & 3);
    int acc = 0;
    int4 e01 = make_int4(1, 2, 3, 4), e23 = make_int4(5, 6, 7, 8);
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 4) {
        int eh[4] = {e01.x, e01.z, e23.x, e23.z}, ex[4] = {e01.y, e01.w, e23.y, e23.w};
        int oH[4], oX[4];
        if (MODE >= 1) {
            const int4* e = reinterpret_cast<const int4*>(lds) + ((r & 255) + (threadIdx.x >> 6) * 0);
            e01 = e[0];
            e23 = e[1];
        }
        ga::diag4_asm<false>(eh[0], eh[1], eh[2], eh[3], ex[0], ex[1], ex[2], ex[3], Hd, H, X, Y, q, q, 5, oH, oX);
        Hd = eh[3];
        if (MODE >= 2 && lane == 63) {
            reinterpret_cast<int4*>(lds)[512 + (r & 255)] = make_int4(oH[0], oX[0], oH[1], oX[1]);
            reinterpret_cast<int4*>(lds)[513 + (r & 255)] = make_int4(oH[2], oX[2], oH[3], oX[3]);
        }
        acc ^= oH[1] + oX[2];
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = H + X + Y + acc + Hd;
}

template <typename F>
double run(F kern, int waves, int blocks, int n) {
    long long* d; int* s;
    (void)hipMalloc(&d, 16 * blocks * sizeof(long long));
    (void)hipMalloc(&s, blocks * waves * 64 * sizeof(int));
    kern<<<blocks, waves * 64>>>(d, s, n);
    kern<<<blocks, waves * 64>>>(d, s, n);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * blocks);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int b = 0; b < blocks; b++) for (int w = 0; w < waves; w++) mx = std::max(mx, (double)h[b * 16 + w]);
    (void)hipFree(d); (void)hipFree(s);
    return mx / n;
}

int main() {
    const int n = 1 << 14;
    const char* names[] = {"block only", "+ edge ds_read_b128 x2 / 4 steps", "+ lane-63 publish / 4 steps"};
    auto fns = std::vector<void (*)(long long*, int*, int)>{steps<0>, steps<1>, steps<2>};
    for (int v = 0; v < 3; v++) {
        printf("%-34s", names[v]);
        for (int w = 1; w <= 4; w++) printf("  %d w/SIMD %6.1f cyc/step/wave", w, run(fns[v], 4 * w, 256, n));
        printf("\n");
    }
    return 0;
}
