// Microbenchmark: the lean sub-chunk (LaneSub<TD, RS>, ga_lane_asm.h) as the fill runs it, one wave
// per SIMD (4-wave workgroups, 256 of them): 16 steps, the next sub-chunk's profile / counter / edge reads, lane
// 63's rows moved into lanes 48..63 and stored, and the counter check after the statement.  Cycles per step per
// wave, against the bare steps (LaneAsm<TD,0,4> x 4).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I globalign_amd/csrc tools/micro/lane_sub.hip -o tools/micro/lane_sub
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "ga_lane_asm.h"

using namespace ga;

constexpr int LDSW = 12288;

template <int TD, int MODE>
__global__ void __launch_bounds__(256) bench(long long* out, int* sink, int nsteps, int o, int never) {
    __shared__ __attribute__((aligned(16))) int lds[LDSW];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < LDSW; k += blockDim.x) lds[k] = k < 4096 ? (k * 37) & 0x03030303 : (k < 6144 ? k : 0);
    __syncthreads();
    auto la = [](const int* p) { return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const int*)p; };
    int H[TD], Y[TD];
#pragma unroll
    for (int k = 0; k < TD; k++) {
        H[k] = lane + k;
        Y[k] = lane + 2 * k + 1;
    }
    int Xl = lane + 3, HLp = lane + 1;
    uint32_t q[TD][4];
#pragma unroll
    for (int k = 0; k < TD; k++)
#pragma unroll
        for (int d = 0; d < 4; d++) q[k][d] = 0x01020304u * ((lane + k + d) & 3);
    lk_v4i E[8], E2[8];
#pragma unroll
    for (int k = 0; k < 8; k++) E[k] = lk_v4i{0, 0, 0, 0};
    uint32_t q2[TD][4];
    int acc = 0;
    const unsigned ca = la(lds + 8192 + 16 * ((w + 3) & 3));
    const unsigned scr = la(lds + 9216) + 8u * (unsigned)lane;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {
        if constexpr (MODE == 0) {
            int oh[16], ox[16];
            int eh[16], ex[16];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                eh[2 * k] = E[k].x; ex[2 * k] = E[k].y; eh[2 * k + 1] = E[k].z; ex[2 * k + 1] = E[k].w;
            }
            uint32_t qq[4][TD];
#pragma unroll
            for (int d = 0; d < 4; d++)
#pragma unroll
                for (int k = 0; k < TD; k++) qq[d][k] = q[k][d];
#pragma unroll
            for (int d = 0; d < 4; d++) LaneAsm<TD, 0, 4>::run(H, Y, Xl, HLp, eh + 4 * d, ex + 4 * d, qq[d], o, oh + 4 * d, ox + 4 * d);
            acc ^= oh[15] + ox[3];
        } else {
            // two sub-chunks per iteration, the edge / profile registers ping-ponged (no copies), as the kernel does
            auto sub = [&](int rr, const lk_v4i (&Ec)[8], const uint32_t (&qc)[TD][4], lk_v4i (&En)[8], uint32_t (&qx)[TD][4]) {
                const unsigned ea = lane == 0 ? la(lds + 4096 + 512 * w + ((2 * rr) & 255)) : la(lds + 6144);
                const unsigned qi = (unsigned)(rr + 16 - lane) & 1023u;
                unsigned qb[TD];
#pragma unroll
                for (int k = 0; k < TD; k++) qb[k] = la(lds) + 4u * (1031u * ((lane * 7 + k) & 3) + qi);
                const unsigned slot = la(lds + 4096 + 512 * ((w + 1) & 3)) + 8u * ((unsigned)(rr - 63 + lane - 48) & 255u);
                const bool hi = lane >= 48;
                const unsigned wa = hi && (lane & 4) ? slot : scr, wb = hi && !(lane & 4) ? slot : scr;
                const unsigned wc = lane == 0 ? la(lds + 8192 + 16 * w) : scr;
                unsigned cv;
                lk_v2u qn[TD][2];
                int R[4];
                LaneSub<TD, 12>::run(H, Y, Xl, HLp, Ec, qc, o, ca, ea, qb, wa, wb, wc, lk_v2u{(unsigned)rr, (unsigned)rr}, cv, En, qn, R);
                if (__builtin_expect((int)__builtin_amdgcn_readfirstlane((int)cv) == never, 0)) acc += 5;
#pragma unroll
                for (int k = 0; k < TD; k++) {
                    qx[k][0] = qn[k][0].x; qx[k][1] = qn[k][0].y; qx[k][2] = qn[k][1].x; qx[k][3] = qn[k][1].y;
                }
                if (MODE == 2 && lane >= 48 && never > 0) sink[rr + lane] = (lane & 4) ? R[0] : R[2];
                acc ^= R[1];
            };
            sub(r, E, q, E2, q2);
            sub(r + 16, E2, q2, E, q);
            r += 16;
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    int z = Xl + HLp + acc + E[0].x + E[7].w;
#pragma unroll
    for (int k = 0; k < TD; k++) z += H[k] + Y[k];
    sink[4096 + blockIdx.x * blockDim.x + threadIdx.x] = z;
}

template <typename F>
double run(F kern, int n) {
    long long* d;
    int* s;
    (void)hipMalloc(&d, 16 * 256 * sizeof(long long));
    (void)hipMalloc(&s, (4096 + 256 * 256) * sizeof(int));
    kern<<<256, 256>>>(d, s, n, 5, -1000);
    kern<<<256, 256>>>(d, s, n, 5, -1000);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * 256);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> v;
    for (int b = 0; b < 256; b++)
        for (int w = 0; w < 4; w++) v.push_back((double)h[b * 16 + w]);
    std::sort(v.begin(), v.end());
    (void)hipFree(d);
    (void)hipFree(s);
    return v[v.size() / 2] / n;
}

template <int TD>
void row() {
    const int n = 1 << 14;
    printf("TD=%d bare %6.1f  lean sub-chunk %6.1f  + store branch %6.1f cyc/step/wave\n", TD, run(bench<TD, 0>, n),
           run(bench<TD, 1>, n), run(bench<TD, 2>, n));
}

int main() {
    row<1>();
    row<2>();
    row<4>();
    row<8>();
    return 0;
}
