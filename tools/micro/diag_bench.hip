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

// the kernel's 8-step sub-chunk (fill_diag_kernel, TD = 1 fast path): edges read one sub-chunk ahead
// into ping-pong registers, the producer's counter read before the blocks and used after them, two
// 4-step blocks, lane 63's eight-row publish (exec narrowed, ds_write2_b32) and {cons, prod}
__global__ void subchunks(long long* out, int* sink, int nsteps) {
    __shared__ __attribute__((aligned(16))) int lds[4096];
    const int lane = threadIdx.x & 63;
    for (int k = threadIdx.x; k < 4096; k += blockDim.x) lds[k] = k & 7;
    __syncthreads();
    int Hd = lane, H = lane + 1, X = lane + 2, Y = lane + 3, cH = 0, cX = 0;
    uint32_t q = 0x01020304u * (lane & 3);
    int4 A[4], B[4];
    for (int k = 0; k < 4; k++) { A[k] = make_int4(k, k + 1, k + 2, k + 3); B[k] = A[k]; }
    unsigned avail = 0, pnext = 0;
    const unsigned ring = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 1024);
    const unsigned pc = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 4000);
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {
#pragma unroll
        for (int sc = 0; sc < 2; sc++) {
            int4(&C)[4] = sc ? B : A;
            int4(&N)[4] = sc ? A : B;
            int eh[8], ex[8];
            for (int k = 0; k < 4; k++) { eh[2 * k] = C[k].x; ex[2 * k] = C[k].y; eh[2 * k + 1] = C[k].z; ex[2 * k + 1] = C[k].w; }
            if ((int)avail < r + 16) avail = (unsigned)__builtin_amdgcn_readfirstlane(lds[4000]) + r + 64;  // never blocks
            const int4* e = reinterpret_cast<const int4*>(lds) + ((r + 8 * sc) & 127);
            for (int k = 0; k < 4; k++) N[k] = e[k];
            pnext = lds[4001];
            int oH[8], oX[8];
            for (int hb = 0; hb < 2; hb++) {
                int h4[4], x4[4];
                ga::diag4_asm<false>(eh[4 * hb], eh[4 * hb + 1], eh[4 * hb + 2], eh[4 * hb + 3], ex[4 * hb],
                                     ex[4 * hb + 1], ex[4 * hb + 2], ex[4 * hb + 3], Hd, H, X, Y, q, q, 5, h4, x4);
                Hd = eh[4 * hb + 3];
                for (int u = 0; u < 4; u++) { oH[4 * hb + u] = h4[u]; oX[4 * hb + u] = x4[u]; }
            }
            asm volatile("" : "+v"(pnext));
            avail = (unsigned)__builtin_amdgcn_readfirstlane((int)max(avail, pnext));
            unsigned long long saved;
            const unsigned long long m63 = 1ull << 63;
            const unsigned ra = ring + (unsigned)(((r + 8 * sc) & 127) * 8);
            typedef unsigned v2u_ __attribute__((ext_vector_type(2)));
            const v2u_ cp = {(unsigned)r, (unsigned)(r + 7)};
            asm volatile(
                "s_mov_b64 %0, exec\n\ts_mov_b64 exec, %3\n\t"
                "ds_write2_b32 %1, %4, %5 offset0:0 offset1:1\n\t"
                "ds_write2_b32 %1, %6, %7 offset0:2 offset1:3\n\t"
                "ds_write2_b32 %1, %8, %9 offset0:4 offset1:5\n\t"
                "ds_write2_b32 %1, %10, %11 offset0:6 offset1:7\n\t"
                "ds_write2_b32 %1, %12, %13 offset0:8 offset1:9\n\t"
                "ds_write2_b32 %1, %14, %15 offset0:10 offset1:11\n\t"
                "ds_write2_b32 %1, %16, %17 offset0:12 offset1:13\n\t"
                "ds_write2_b32 %1, %18, %19 offset0:14 offset1:15\n\t"
                "ds_write_b64 %2, %20\n\t"
                "s_mov_b64 exec, %0"
                : "=&s"(saved)
                : "v"(ra), "v"(pc), "s"(m63), "v"(cH), "v"(cX), "v"(oH[0]), "v"(oX[0]), "v"(oH[1]), "v"(oX[1]),
                  "v"(oH[2]), "v"(oX[2]), "v"(oH[3]), "v"(oX[3]), "v"(oH[4]), "v"(oX[4]), "v"(oH[5]), "v"(oX[5]),
                  "v"(oH[6]), "v"(oX[6]), "v"(cp)
                : "memory");
            cH = oH[7];
            cX = oX[7];
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = H + X + Y + Hd + cH + cX + (int)avail;
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
    printf("%-34s", "kernel's 8-step sub-chunk");
    for (int w = 1; w <= 4; w++) printf("  %d w/SIMD %6.1f cyc/step/wave", w, run(subchunks, 4 * w, 256, n));
    printf("\n");
    return 0;
}
