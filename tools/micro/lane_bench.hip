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

// Packed 16-bit variant: two stripes per wave in the halves of each register,
// TD columns of each; per column pair: a v_perm for the two stripes' profile halves, then the
// recurrence in v_pk_add_i16 (clamp) / v_pk_min_i16.  Cycles per step cover 2 x TD columns.
typedef short s2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s2v as_s2(int x) { return __builtin_bit_cast(s2v, x); }
__device__ __forceinline__ int as_i(s2v x) { return __builtin_bit_cast(int, x); }
template <int TD>
struct St16 {
    s2v H[TD], Y[TD];
    int Xl, Hl, HLp;
};
template <int TD, int U>
__device__ __forceinline__ void lstep16(St16<TD>& s, int eh, int ex, const uint32_t (&qa)[TD], const uint32_t (&qb)[TD],
                                        s2v o2) {
    s2v X = as_s2(__builtin_amdgcn_update_dpp(ex, s.Xl, 0x138, 0xf, 0xf, false));
    const int HLn = __builtin_amdgcn_update_dpp(eh, s.Hl, 0x138, 0xf, 0xf, false);
    s2v Hd = as_s2(s.HLp);
    constexpr unsigned sel = (U & 1) ? 0x07060302u : 0x05040100u;  // the step's int16 of each stripe's dword
#pragma unroll
    for (int k = 0; k < TD; k++) {
        const s2v sb = as_s2((int)__builtin_amdgcn_perm(qb[k], qa[k], sel));
        const s2v M = __builtin_elementwise_add_sat(Hd, sb);
        const s2v Hn = __builtin_elementwise_min(__builtin_elementwise_min(M, X), s.Y[k]);
        const s2v Ho = __builtin_elementwise_add_sat(Hn, o2);
        X = __builtin_elementwise_min(X, Ho);
        s.Y[k] = __builtin_elementwise_min(s.Y[k], Ho);
        Hd = s.H[k];
        s.H[k] = Hn;
    }
    s.Xl = as_i(X);
    s.Hl = as_i(s.H[TD - 1]);
    s.HLp = HLn;
}

template <int TD, int MODE>
__global__ void bench16(long long* out, int* sink, int nsteps, int o) {
    __shared__ __attribute__((aligned(16))) int lds[8192];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < 8192; k += blockDim.x) lds[k] = (k * 37) & 0x00030003;
    __syncthreads();
    St16<TD> s;
#pragma unroll
    for (int k = 0; k < TD; k++) { s.H[k] = s2v{(short)(lane + k), (short)(lane - k)}; s.Y[k] = s2v{(short)(lane + 2 * k + 1), (short)(lane + 3)}; }
    s.Xl = lane + 3; s.Hl = lane; s.HLp = lane + 1;
    const s2v o2 = s2v{(short)o, (short)o};
    // profile: int16 entries, a dword = two rows; 16 steps = 8 dwords per column per stripe
    uint32_t qa[8][TD], qb[8][TD];
#pragma unroll
    for (int c = 0; c < 8; c++)
#pragma unroll
        for (int k = 0; k < TD; k++) { qa[c][k] = 0x00010002u * ((lane + k + c) & 3); qb[c][k] = 0x00020001u * ((lane + k + 2 * c) & 3); }
    int4 E[8];
#pragma unroll
    for (int k = 0; k < 8; k++) E[k] = make_int4(k, k + 1, k + 2, k + 3);
    int acc = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {
        int eh[16], ex[16];
#pragma unroll
        for (int k = 0; k < 8; k++) { eh[2 * k] = E[k].x; ex[2 * k] = E[k].y; eh[2 * k + 1] = E[k].z; ex[2 * k + 1] = E[k].w; }
        uint32_t qan[8][TD], qbn[8][TD];
        if (MODE >= 1) {
            const int4* e4 = reinterpret_cast<const int4*>(lds) + ((r + 16 * w) & 511);
#pragma unroll
            for (int k = 0; k < 8; k++) E[k] = e4[k];
#pragma unroll
            for (int k = 0; k < TD; k++) {
                const int* pa = lds + 2048 + (((r - lane + 64 * k) & 1023));
                const int* pb = lds + 4096 + (((r - lane + 64 * k + 40) & 1023));
#pragma unroll
                for (int c = 0; c < 8; c++) { qan[c][k] = pa[c]; qbn[c][k] = pb[c]; }
            }
        }
        int oH[16];
#pragma unroll
        for (int c = 0; c < 8; c++) {
            lstep16<TD, 0>(s, eh[2 * c + 0], ex[2 * c + 0], qa[c], qb[c], o2); oH[2 * c + 0] = s.Hl;
            lstep16<TD, 1>(s, eh[2 * c + 1], ex[2 * c + 1], qa[c], qb[c], o2); oH[2 * c + 1] = s.Hl;
        }
        if (MODE >= 1) {
#pragma unroll
            for (int c = 0; c < 8; c++)
#pragma unroll
                for (int k = 0; k < TD; k++) { qa[c][k] = qan[c][k]; qb[c][k] = qbn[c][k]; }
        }
        acc ^= oH[5] + oH[9];
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    int z = s.Xl + s.Hl + s.HLp + acc;
#pragma unroll
    for (int k = 0; k < TD; k++) z += as_i(s.H[k]) + as_i(s.Y[k]);
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

template <int TD>
void row16() {
    const int n = 1 << 14;
    auto fns = std::vector<void (*)(long long*, int*, int, int)>{bench16<TD, 0>, bench16<TD, 1>};
    const char* modes[] = {"packed block only", "packed + LDS reads"};
    for (int v = 0; v < 2; v++) {
        printf("TD=%d x2 %-24s", TD, modes[v]);
        for (int w = 1; w <= 2; w++) {
            const double c = run(fns[v], 4 * w, 256, n);
            printf("  %d w/SIMD %6.1f cyc/step/wave (%.3f SIMD cyc/cell)", w, c, c / w / (128.0 * TD));
        }
        printf("\n");
    }
}

int main() {
    row16<1>();
    row16<2>();
    row16<4>();
    row16<8>();
    row<1>("");
    row<2>("");
    row<4>("");
    row<8>("");
    return 0;
}
