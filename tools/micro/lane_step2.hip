// Microbenchmark: the lane-skewed fill step with fewer VALU per step.
//
//  mode 0  the kernel's round-3 step: X / H' of the left lane by v_mov_b32_dpp with the edge as the
//          "old" operand (a copy of the edge into the destination first), lane 63's (H', h1') into
//          DPP shift registers (another copy + DPP each), 16 edge rows per 16 steps by ds_read_b128
//  mode 1  the left lane's values by ONE v_add_u32_dpp each: shr:1 with bound_ctrl (lane 0 gets 0)
//          plus an edge register that is 0 in lanes 1..63 (lane 0 loads the ring, the others a zero
//          block), so no copy; output as in mode 0
//  mode 2  mode 1, and lane 63's (H', h1') straight to the LDS ring every step: one ds_write2_b32 from
//          every lane (lane 63 at the ring slot, lanes 0..62 at a scratch area), no shift registers
// Cycles per step per wave at one and two waves per SIMD, 256 workgroups.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int TD>
struct St {
    int H[TD], Y[TD];
    int Xl, HLp;
};

template <int TD, int U, int MODE>
__device__ __forceinline__ void lstep(St<TD>& s, int eh, int ex, const uint32_t (&q)[TD], int o) {
    int X, HLn;
    if constexpr (MODE == 0) {
        X = __builtin_amdgcn_update_dpp(ex, s.Xl, 0x138, 0xf, 0xf, false);
        HLn = __builtin_amdgcn_update_dpp(eh, s.H[TD - 1], 0x138, 0xf, 0xf, false);
    } else {
        X = __builtin_amdgcn_update_dpp(0, s.Xl, 0x138, 0xf, 0xf, true) + ex;
        HLn = __builtin_amdgcn_update_dpp(0, s.H[TD - 1], 0x138, 0xf, 0xf, true) + eh;
    }
    int Hd = s.HLp;
#pragma unroll
    for (int k = 0; k < TD; k++) {
        const int sb = (int)(int8_t)(q[k] >> (8 * U));
        const int M = Hd + sb;
        const int Hn = min(min(M, X), s.Y[k]);
        const int Ho = Hn + o;
        X = min(X, Ho);
        s.Y[k] = min(s.Y[k], Ho);
        Hd = s.H[k];
        s.H[k] = Hn;
    }
    s.Xl = X;
    s.HLp = HLn;
}

template <int TD, int MODE>
__global__ void __launch_bounds__(512) bench(long long* out, int* sink, int nsteps, int o) {
    __shared__ __attribute__((aligned(16))) int lds[8192 + 2048];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < 8192 + 2048; k += blockDim.x) lds[k] = k < 8192 ? (k * 37) & 0x03030303 : 0;
    __syncthreads();
    St<TD> s;
#pragma unroll
    for (int k = 0; k < TD; k++) { s.H[k] = lane + k; s.Y[k] = lane + 2 * k + 1; }
    s.Xl = lane + 3; s.HLp = lane + 1;
    uint32_t q[4][TD];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int k = 0; k < TD; k++) q[c][k] = 0x01020304u * ((lane + k + c) & 3);
    int4 E[8];
#pragma unroll
    for (int k = 0; k < 8; k++) E[k] = make_int4(k, k + 1, k + 2, k + 3);
    int RH = 0, RX = 0, acc = 0;
    // mode 2 output: lane 63 -> ring [w][256] int2 at lds + 4096 (as int), lanes 0..62 -> scratch past 8192
    int* ring = lds + 4096 + w * 512;
    int* scratch = lds + 8192 + w * 160;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {
        int eh[16], ex[16];
#pragma unroll
        for (int k = 0; k < 8; k++) { eh[2 * k] = E[k].x; ex[2 * k] = E[k].y; eh[2 * k + 1] = E[k].z; ex[2 * k + 1] = E[k].w; }
        uint32_t qn[4][TD];
        {
            // edges: mode 0 every lane the ring rows (broadcast); modes 1-2 lane 0 the ring rows, the
            // others a zero block
            const int4* e4 = reinterpret_cast<const int4*>(lds) + ((r + 16 * w) & 511);
            const int4* z4 = reinterpret_cast<const int4*>(lds + 8192 + 8 * 160);  // zeros
            const int4* src = (MODE == 0 || lane == 0) ? e4 : z4;
#pragma unroll
            for (int k = 0; k < 8; k++) E[k] = src[k];
#pragma unroll
            for (int k = 0; k < TD; k++) {
                const int* pk = lds + 2048 + (((r - lane + 64 * k) & 1023));
                qn[0][k] = pk[0]; qn[1][k] = pk[4]; qn[2][k] = pk[8]; qn[3][k] = pk[12];
            }
        }
        // mode 2: this lane's output base (lane 63 the ring slot of this sub-chunk's first row)
        int* ob = lane == 63 ? ring + 2 * ((r + 1) & 255 & ~15) : scratch + 2 * lane;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            auto out = [&](int u) {
                if constexpr (MODE == 2) {
                    ob[2 * u] = s.H[TD - 1];
                    ob[2 * u + 1] = s.Xl;
                } else {
                    RH = __builtin_amdgcn_update_dpp(s.H[TD - 1], RH, 0x130, 0xf, 0xf, false);
                    RX = __builtin_amdgcn_update_dpp(s.Xl, RX, 0x130, 0xf, 0xf, false);
                }
            };
            lstep<TD, 0, MODE>(s, eh[4 * c + 0], ex[4 * c + 0], q[c], o); out(4 * c + 0);
            lstep<TD, 1, MODE>(s, eh[4 * c + 1], ex[4 * c + 1], q[c], o); out(4 * c + 1);
            lstep<TD, 2, MODE>(s, eh[4 * c + 2], ex[4 * c + 2], q[c], o); out(4 * c + 2);
            lstep<TD, 3, MODE>(s, eh[4 * c + 3], ex[4 * c + 3], q[c], o); out(4 * c + 3);
        }
        if (MODE != 2 && lane >= 48) reinterpret_cast<int2*>(ring)[((r + lane) & 255)] = make_int2(RH, RX);
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int k = 0; k < TD; k++) q[c][k] = qn[c][k];
        acc ^= s.Xl;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    int z = s.Xl + s.HLp + acc + RH + RX + ring[lane];
#pragma unroll
    for (int k = 0; k < TD; k++) z += s.H[k] + s.Y[k];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = z;
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

template <int TD>
void row() {
    const int n = 1 << 14;
    auto fns = std::vector<void (*)(long long*, int*, int, int)>{bench<TD, 0>, bench<TD, 1>, bench<TD, 2>};
    const char* modes[] = {"r3 step (copies, DPP shift out)", "add-DPP in, DPP shift out", "add-DPP in, LDS out/step"};
    for (int v = 0; v < 3; v++) {
        printf("TD=%d %-34s", TD, modes[v]);
        for (int w = 1; w <= 2; w++) {
            const double c = run(fns[v], 4 * w, 256, n);
            printf("  %d w/SIMD %6.1f cyc/step/wave (%.3f SIMD cyc/cell)", w, c, c / w / (64.0 * TD));
        }
        printf("\n");
    }
}

int main() {
    row<1>();
    row<2>();
    row<4>();
    row<8>();
    return 0;
}
