// Microbenchmark: cycles per step of a "lane-skewed" anti-diagonal fill block:
// lane l owns TD adjacent columns and works on row t - l at step t, so a lane's TD columns are one
// in-register row segment (h1' chained through them) and only the lane-to-lane hand-over is
// skewed.  Modes: 0 block only (registers), 1 + the per-16-step LDS traffic of a kernel (edge rows
// broadcast, the lane's profile window), 2 = 1 + right edge out through a DPP shift register and
// one 16-lane store per 16 steps, 3 = 1 + right edge out as lane 63's 16-byte stores per 4 steps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int TD>
struct St {
    int H[TD], Y[TD];
    int Xl, Hl, HLp;
};

// one step; u = the step's byte within the profile dwords (compile time)
template <int TD, int U>
__device__ __forceinline__ void lstep(St<TD>& s, int eh, int ex, const uint32_t (&q)[TD], int o) {
    int X = __builtin_amdgcn_update_dpp(ex, s.Xl, 0x138, 0xf, 0xf, false);
    const int HLn = __builtin_amdgcn_update_dpp(eh, s.Hl, 0x138, 0xf, 0xf, false);
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
    s.Hl = s.H[TD - 1];
    s.HLp = HLn;
}

template <int TD, int MODE>
__global__ void bench(long long* out, int* sink, int nsteps, int o) {
    __shared__ __attribute__((aligned(16))) int lds[8192];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < 8192; k += blockDim.x) lds[k] = (k * 37) & 0x03030303;
    __syncthreads();
    St<TD> s;
#pragma unroll
    for (int k = 0; k < TD; k++) { s.H[k] = lane + k; s.Y[k] = lane + 2 * k + 1; }
    s.Xl = lane + 3; s.Hl = lane; s.HLp = lane + 1;
    uint32_t q[4][TD];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int k = 0; k < TD; k++) q[c][k] = 0x01020304u * ((lane + k + c) & 3);
    int4 E[8];
#pragma unroll
    for (int k = 0; k < 8; k++) E[k] = make_int4(k, k + 1, k + 2, k + 3);
    int RH = 0, RX = 0, acc = 0;
    const unsigned prof = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 2048);
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
            // the lane's 16-row profile window of each column: two ds_read2_b32 from a table whose
            // dword r holds rows r..r+3 (any start row is dword aligned)
#pragma unroll
            for (int k = 0; k < TD; k++) {
                const int* pk = lds + 2048 + (((r - lane + 64 * k) & 1023));
                qn[0][k] = pk[0]; qn[1][k] = pk[4]; qn[2][k] = pk[8]; qn[3][k] = pk[12];
            }
        }
        int oH[16], oX[16];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            lstep<TD, 0>(s, eh[4 * c + 0], ex[4 * c + 0], q[c], o); oH[4 * c + 0] = s.Hl; oX[4 * c + 0] = s.Xl;
            if (MODE == 2) { RH = __builtin_amdgcn_update_dpp(s.Hl, RH, 0x130, 0xf, 0xf, false); RX = __builtin_amdgcn_update_dpp(s.Xl, RX, 0x130, 0xf, 0xf, false); }
            lstep<TD, 1>(s, eh[4 * c + 1], ex[4 * c + 1], q[c], o); oH[4 * c + 1] = s.Hl; oX[4 * c + 1] = s.Xl;
            if (MODE == 2) { RH = __builtin_amdgcn_update_dpp(s.Hl, RH, 0x130, 0xf, 0xf, false); RX = __builtin_amdgcn_update_dpp(s.Xl, RX, 0x130, 0xf, 0xf, false); }
            lstep<TD, 2>(s, eh[4 * c + 2], ex[4 * c + 2], q[c], o); oH[4 * c + 2] = s.Hl; oX[4 * c + 2] = s.Xl;
            if (MODE == 2) { RH = __builtin_amdgcn_update_dpp(s.Hl, RH, 0x130, 0xf, 0xf, false); RX = __builtin_amdgcn_update_dpp(s.Xl, RX, 0x130, 0xf, 0xf, false); }
            lstep<TD, 3>(s, eh[4 * c + 3], ex[4 * c + 3], q[c], o); oH[4 * c + 3] = s.Hl; oX[4 * c + 3] = s.Xl;
            if (MODE == 2) { RH = __builtin_amdgcn_update_dpp(s.Hl, RH, 0x130, 0xf, 0xf, false); RX = __builtin_amdgcn_update_dpp(s.Xl, RX, 0x130, 0xf, 0xf, false); }
            if (MODE == 3 && lane == 63) {
                int4* d = reinterpret_cast<int4*>(lds + 6144) + ((2 * (r + 4 * c) + 16 * w) & 255);
                d[0] = make_int4(oH[4 * c], oX[4 * c], oH[4 * c + 1], oX[4 * c + 1]);
                d[1] = make_int4(oH[4 * c + 2], oX[4 * c + 2], oH[4 * c + 3], oX[4 * c + 3]);
            }
        }
        if (MODE == 2 && lane >= 48) reinterpret_cast<int2*>(lds + 6144)[((r + lane + 16 * w) & 511)] = make_int2(RH, RX);
        if (MODE >= 1) {
#pragma unroll
            for (int c = 0; c < 4; c++)
#pragma unroll
                for (int k = 0; k < TD; k++) q[c][k] = qn[c][k];
        }
        acc ^= oH[5] + oX[9];
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    int z = s.Xl + s.Hl + s.HLp + acc + RH + RX;
#pragma unroll
    for (int k = 0; k < TD; k++) z += s.H[k] + s.Y[k];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = z;
}

template <typename F>
double run(F kern, int waves, int blocks, int n) {
    long long* d; int* s;
    (void)hipMalloc(&d, 16 * blocks * sizeof(long long));
    (void)hipMalloc(&s, blocks * waves * 64 * sizeof(int));
    kern<<<blocks, waves * 64>>>(d, s, n, 5);
    kern<<<blocks, waves * 64>>>(d, s, n, 5);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * blocks);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int b = 0; b < blocks; b++) for (int w = 0; w < waves; w++) mx = std::max(mx, (double)h[b * 16 + w]);
    (void)hipFree(d); (void)hipFree(s);
    return mx / n;
}

template <int TD>
void row(const char* name) {
    const int n = 1 << 14;
    auto fns = std::vector<void (*)(long long*, int*, int, int)>{bench<TD, 0>, bench<TD, 1>, bench<TD, 2>, bench<TD, 3>};
    const char* modes[] = {"block only", "+ edge/profile LDS reads", "+ DPP shift-register out", "+ lane-63 b128 out"};
    for (int v = 0; v < 4; v++) {
        printf("TD=%d %-28s", TD, modes[v]);
        for (int w = 1; w <= 2; w++) {
            const double c = run(fns[v], 4 * w, 256, n);
            printf("  %d w/SIMD %6.1f cyc/step/wave (%.3f SIMD cyc/cell)", w, c, c / w / (64.0 * TD));
        }
        printf("\n");
    }
}

int main() {
    row<1>("");
    row<2>("");
    row<4>("");
    row<8>("");
    return 0;
}
