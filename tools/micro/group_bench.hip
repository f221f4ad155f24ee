// Microbenchmark: cycles per step of the group-scan fill step (ga_group.h) against the
// lane-skewed step (ga_lane.hip), one wave per SIMD and two.  Modes: 0 the steps only (registers);
// 1 + the per-16-step LDS reads of a kernel (16 edge rows broadcast, each column's 16-row profile
// window); 2 = 1 + the right edge out through two DPP shift registers and one 16-lane store per 16 steps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../globalign_amd/csrc group_bench.hip -o group_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "ga_group.h"

using namespace ga;

template <int T, int L, int MODE>
__global__ void gbench(long long* out, int* sink, int nsteps, int o) {
    __shared__ __attribute__((aligned(16))) int lds[8192];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < 8192; k += blockDim.x) lds[k] = (k * 37) & 0x03030303;
    __syncthreads();
    int H[T], Y[T];
#pragma unroll
    for (int k = 0; k < T; k++) { H[k] = lane + k; Y[k] = lane + 2 * k + 1; }
    int V = lane + 3, Hd0 = lane + 1;
    int last = (lane % L) == L - 1 ? -1 : 0;
    asm volatile("" : "+v"(last));  // an opaque mask: v_bfi_b32, not v_cndmask
    const int g = lane / L;
    uint32_t q[4][T];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int k = 0; k < T; k++) q[c][k] = 0x01020304u * ((lane + k + c) & 3);
    int4 E[8];
#pragma unroll
    for (int k = 0; k < 8; k++) E[k] = make_int4(k, k + 1, k + 2, k + 3);
    int RH = 0, RX = 0, acc = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {
        int eh[16], ex[16];
#pragma unroll
        for (int k = 0; k < 8; k++) { eh[2 * k] = E[k].x; ex[2 * k] = E[k].y; eh[2 * k + 1] = E[k].z; ex[2 * k + 1] = E[k].w; }
        uint32_t qn[4][T];
        if (MODE >= 1) {
            const int4* e4 = reinterpret_cast<const int4*>(lds) + ((r + 16 * w) & 511);
#pragma unroll
            for (int k = 0; k < 8; k++) E[k] = e4[k];
#pragma unroll
            for (int k = 0; k < T; k++) {
                const int* pk = lds + 2048 + (((r - g + 64 * k) & 1023));
                qn[0][k] = pk[0]; qn[1][k] = pk[4]; qn[2][k] = pk[8]; qn[3][k] = pk[12];
            }
        }
#pragma unroll
        for (int c = 0; c < 4; c++) {
#define GSTEP(U)                                                                                        \
    group_step<T, L, U, false>(H, Y, V, Hd0, ex[4 * c + U], eh[4 * c + U], q[c], o, last, true);          \
    if (MODE == 2) {                                                                                    \
        RH = __builtin_amdgcn_update_dpp(H[T - 1], RH, 0x130, 0xf, 0xf, false);                          \
        RX = __builtin_amdgcn_update_dpp(V, RX, 0x130, 0xf, 0xf, false);                                 \
    }
            GSTEP(0) GSTEP(1) GSTEP(2) GSTEP(3)
#undef GSTEP
        }
        if (MODE == 2 && lane >= 48) reinterpret_cast<int2*>(lds + 6144)[((r + lane + 16 * w) & 511)] = make_int2(RH, RX);
        if (MODE >= 1) {
#pragma unroll
            for (int c = 0; c < 4; c++)
#pragma unroll
                for (int k = 0; k < T; k++) q[c][k] = qn[c][k];
        }
        acc ^= H[0] + V;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    int z = V + Hd0 + acc + RH + RX;
#pragma unroll
    for (int k = 0; k < T; k++) z += H[k] + Y[k];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = z;
}

// the lane-skewed step (ga_lane.hip lane_step, score only) for comparison
template <int TD, int U>
__device__ __forceinline__ void lstep(int (&H)[TD], int (&Y)[TD], int& Xl, int& Hl, int& HLp, int eh, int ex,
                                      const uint32_t (&q)[TD], int o) {
    int X = __builtin_amdgcn_update_dpp(ex, Xl, 0x138, 0xf, 0xf, false);
    const int HLn = __builtin_amdgcn_update_dpp(eh, Hl, 0x138, 0xf, 0xf, false);
    int Hd = HLp;
#pragma unroll
    for (int k = 0; k < TD; k++) {
        const int M = Hd + (int)(int8_t)(q[k] >> (8 * U));
        const int Hn = min(min(M, X), Y[k]);
        const int Ho = Hn + o;
        X = min(X, Ho);
        Y[k] = min(Y[k], Ho);
        Hd = H[k];
        H[k] = Hn;
    }
    Xl = X;
    Hl = H[TD - 1];
    HLp = HLn;
}

template <int TD, int MODE>
__global__ void lbench(long long* out, int* sink, int nsteps, int o) {
    __shared__ __attribute__((aligned(16))) int lds[8192];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < 8192; k += blockDim.x) lds[k] = (k * 37) & 0x03030303;
    __syncthreads();
    int H[TD], Y[TD];
#pragma unroll
    for (int k = 0; k < TD; k++) { H[k] = lane + k; Y[k] = lane + 2 * k + 1; }
    int Xl = lane + 3, Hl = lane, HLp = lane + 1;
    uint32_t q[4][TD];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int k = 0; k < TD; k++) q[c][k] = 0x01020304u * ((lane + k + c) & 3);
    int4 E[8];
#pragma unroll
    for (int k = 0; k < 8; k++) E[k] = make_int4(k, k + 1, k + 2, k + 3);
    int RH = 0, RX = 0, acc = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {
        int eh[16], ex[16];
#pragma unroll
        for (int k = 0; k < 8; k++) { eh[2 * k] = E[k].x; ex[2 * k] = E[k].y; eh[2 * k + 1] = E[k].z; ex[2 * k + 1] = E[k].w; }
        uint32_t qn[4][TD];
        if (MODE >= 1) {
            const int4* e4 = reinterpret_cast<const int4*>(lds) + ((r + 16 * w) & 511);
#pragma unroll
            for (int k = 0; k < 8; k++) E[k] = e4[k];
#pragma unroll
            for (int k = 0; k < TD; k++) {
                const int* pk = lds + 2048 + (((r - lane + 64 * k) & 1023));
                qn[0][k] = pk[0]; qn[1][k] = pk[4]; qn[2][k] = pk[8]; qn[3][k] = pk[12];
            }
        }
#pragma unroll
        for (int c = 0; c < 4; c++) {
#define LSTEP(U)                                                                                        \
    lstep<TD, U>(H, Y, Xl, Hl, HLp, eh[4 * c + U], ex[4 * c + U], q[c], o);                                \
    if (MODE == 2) {                                                                                    \
        RH = __builtin_amdgcn_update_dpp(Hl, RH, 0x130, 0xf, 0xf, false);                                \
        RX = __builtin_amdgcn_update_dpp(Xl, RX, 0x130, 0xf, 0xf, false);                                \
    }
            LSTEP(0) LSTEP(1) LSTEP(2) LSTEP(3)
#undef LSTEP
        }
        if (MODE == 2 && lane >= 48) reinterpret_cast<int2*>(lds + 6144)[((r + lane + 16 * w) & 511)] = make_int2(RH, RX);
        if (MODE >= 1) {
#pragma unroll
            for (int c = 0; c < 4; c++)
#pragma unroll
                for (int k = 0; k < TD; k++) q[c][k] = qn[c][k];
        }
        acc ^= Hl + Xl;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    int z = Xl + Hl + HLp + acc + RH + RX;
#pragma unroll
    for (int k = 0; k < TD; k++) z += H[k] + Y[k];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = z;
}

// dependent-chain latencies of single forms (cycles per op, one wave per SIMD)
#define CHAIN(body) asm volatile(".rept 64\n" body ".endr\n" : "+v"(x) : "v"(y))
template <int V>
__global__ void chain(long long* out, int* sink, int, int) {
    int x = threadIdx.x, y = threadIdx.x * 3 + 1;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 16; it++) {
        if (V == 0) CHAIN("v_min_i32 %0, %0, %1\n");
        if (V == 1) CHAIN("v_add_u32 %0, %0, %1\n");
        if (V == 2) CHAIN("v_min3_i32 %0, %0, %1, %0\n");
        if (V == 3) CHAIN("v_cndmask_b32 %0, %0, %1, vcc\n");
        if (V == 4) CHAIN("v_min_i32_dpp %0, %0, %0 quad_perm:[0,0,1,2] row_mask:0xf bank_mask:0xf\ns_nop 1\n");
        if (V == 5) CHAIN("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\ns_nop 1\n");
        if (V == 6) CHAIN("v_min_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xa\ns_nop 1\n");
        if (V == 7) CHAIN("s_nop 1\n");
        if (V == 8) CHAIN("v_min_i32_dpp %0, %0, %0 quad_perm:[0,0,1,2] row_mask:0xf bank_mask:0xf\nv_min_i32 %0, %0, %1\n");
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x % 64 == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <typename F>
double run(F kern, int waves, int blocks, int n) {
    long long* d;
    int* s;
    (void)hipMalloc(&d, 16 * blocks * sizeof(long long));
    (void)hipMalloc(&s, blocks * waves * 64 * sizeof(int));
    kern<<<blocks, waves * 64>>>(d, s, n, 5);
    kern<<<blocks, waves * 64>>>(d, s, n, 5);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * blocks);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int b = 0; b < blocks; b++)
        for (int w = 0; w < waves; w++) mx = std::max(mx, (double)h[b * 16 + w]);
    (void)hipFree(d);
    (void)hipFree(s);
    return mx / n;
}

template <int T, int L>
void grow() {
    const int n = 1 << 14;
    auto fns = std::vector<void (*)(long long*, int*, int, int)>{gbench<T, L, 0>, gbench<T, L, 1>, gbench<T, L, 2>};
    const char* modes[] = {"steps only", "+ LDS reads", "+ edge out"};
    for (int v = 0; v < 3; v++) {
        printf("group T=%d L=%-2d %-12s", T, L, modes[v]);
        for (int w = 1; w <= 3; w++) {
            const double c = run(fns[v], 4 * w, 256, n);
            printf("  %d w/SIMD %6.1f cyc/step (%.3f SIMD cyc/cell)", w, c, c / w / (64.0 * T));
        }
        printf("\n");
    }
}

template <int TD>
void lrow() {
    const int n = 1 << 14;
    auto fns = std::vector<void (*)(long long*, int*, int, int)>{lbench<TD, 0>, lbench<TD, 1>, lbench<TD, 2>};
    const char* modes[] = {"steps only", "+ LDS reads", "+ edge out"};
    for (int v = 0; v < 3; v++) {
        printf("lane  TD=%d      %-12s", TD, modes[v]);
        for (int w = 1; w <= 3; w++) {
            const double c = run(fns[v], 4 * w, 256, n);
            printf("  %d w/SIMD %6.1f cyc/step (%.3f SIMD cyc/cell)", w, c, c / w / (64.0 * TD));
        }
        printf("\n");
    }
}

int main() {
    const char* cn[] = {"v_min", "v_add", "v_min3", "v_cndmask", "min_dpp quad_perm +nop1", "mov_dpp wave_shr:1 +nop1",
                        "min_dpp row_shr:4 banks +nop1", "s_nop 1", "min_dpp quad_perm + v_min"};
    auto cf = std::vector<void (*)(long long*, int*, int, int)>{chain<0>, chain<1>, chain<2>, chain<3>, chain<4>,
                                                                 chain<5>, chain<6>, chain<7>, chain<8>};
    for (int v = 0; v < (int)cf.size(); v++)
        printf("chain %-32s 1 w/SIMD %6.2f cyc/op\n", cn[v], run(cf[v], 4, 256, 1) / (16.0 * 64));
    grow<1, 4>();
    grow<1, 8>();
    grow<1, 16>();
    grow<2, 4>();
    grow<2, 8>();
    grow<2, 16>();
    grow<4, 8>();
    lrow<1>();
    lrow<2>();
    lrow<4>();
    lrow<8>();
    return 0;
}
