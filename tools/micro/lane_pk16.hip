// Microbenchmark: what a packed 16-bit encoding of the lane fill's step would
// cost at one column per lane.  The step (ga_lane.h lane_step, TD = 1):
//     X = h1'(left) (DPP wave_shr:1), HLn = H'(left) (DPP), M = Hd + sub', H = min3(M, X, Y), T = H + o,
//     X = min(X, T), Y = min(Y, T)
// Variants, cycles per step per wave (s_memtime), 256 workgroups:
//   0: int32, one stripe per wave, 4-wave workgroups (one wave per SIMD)
//   1: int32, 8-wave workgroups (two waves per SIMD: the issue-bound regime of ~2 stripes per SIMD at N = 8)
//   2: two stripes packed in the 16-bit halves of each register (v_pk_add_u16 / v_pk_min_i16), one wave per SIMD,
//      no range bookkeeping: the best a packed encoding could do
//   3: variant 2 plus what an exact encoding needs: int16 holds only differences (H' grows to 2.45e6 at C4), so a
//      lane keeps its values relative to a base of its own; the two values taken from the left lane are rebased
//      (one v_pk_add each, the base difference) and every 16 steps the lane rebases itself (a v_pk_sub per value)
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short s2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int as_i(s2 v) { return __builtin_bit_cast(int, v); }
__device__ __forceinline__ s2 as_s2(int v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ s2 pmin(s2 a, s2 b) { return __builtin_elementwise_min(a, b); }

template <int V>
__global__ void steps(long long* out, int* sink, int n, int qseed) {
    const int lane = threadIdx.x & 63;
    const int o = 6;
    long long t0 = 0;
    if (V <= 1) {
        int X = lane, Hl = lane * 3, HLp = lane, Y = lane * 2 + 5, H = lane;
        const int ex = lane == 0 ? 7 : 0, eh = lane == 0 ? 3 : 0;
        unsigned q = (unsigned)(qseed * 2654435761u) ^ lane;
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
        for (int k = 0; k < n; k++) {
            X = __builtin_amdgcn_update_dpp(ex, X, 0x138, 0xf, 0xf, false);
            const int HLn = __builtin_amdgcn_update_dpp(eh, Hl, 0x138, 0xf, 0xf, false);
            const int M = HLp + (int)(signed char)(q >> (8 * (k & 3)));
            H = min(min(M, X), Y);
            const int T = H + o;
            X = min(X, T);
            Y = min(Y, T);
            Hl = H;
            HLp = HLn;
            if ((k & 3) == 3) q = q * 1664525u + 1013904223u;
        }
        sink[blockIdx.x * blockDim.x + threadIdx.x] = X + Y + H;
    } else {
        s2 X = {(short)lane, (short)(lane + 1)}, Y = {(short)(2 * lane), (short)(lane + 5)}, H = X, Hl = X, HLp = X;
        const s2 o2 = {(short)o, (short)o};
        s2 base = {0, 0};  // (V3) the lane's rebase amount, and the left lane's
        const int ex = lane == 0 ? 7 : 0, eh = lane == 0 ? 3 : 0;
        unsigned q = (unsigned)(qseed * 2654435761u) ^ lane;
        t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
        for (int k = 0; k < n; k++) {
            s2 Xn = as_s2(__builtin_amdgcn_update_dpp(ex, as_i(X), 0x138, 0xf, 0xf, false));
            const s2 HLn = as_s2(__builtin_amdgcn_update_dpp(eh, as_i(Hl), 0x138, 0xf, 0xf, false));
            if (V == 3) {
                const s2 bl = as_s2(__builtin_amdgcn_update_dpp(0, as_i(base), 0x138, 0xf, 0xf, false));
                Xn = Xn + (bl - base);  // the left lane's values in this lane's frame
            }
            const unsigned qq = q >> (8 * (k & 3));
            const s2 sub = {(short)(signed char)qq, (short)(signed char)(qq >> 4)};
            const s2 M = HLp + sub;
            H = pmin(pmin(M, Xn), Y);
            const s2 T = H + o2;
            X = pmin(Xn, T);
            Y = pmin(Y, T);
            Hl = H;
            HLp = HLn;
            if ((k & 3) == 3) q = q * 1664525u + 1013904223u;
            if (V == 3 && (k & 15) == 15) {  // rebase: subtract the lane's own H from everything it holds
                X = X - H;
                Y = Y - H;
                HLp = HLp - H;
                base = base + H;
                Hl = H - H;
                H = Hl;
            }
        }
        sink[blockIdx.x * blockDim.x + threadIdx.x] = as_i(X) + as_i(Y) + as_i(H);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <typename F>
double run(F f, int waves) {
    long long* d;
    int* s;
    (void)hipMalloc(&d, 256 * 16 * 8);
    (void)hipMalloc(&s, 256 * 1024 * 4);
    const int n = 1 << 15;
    f<<<256, 64 * waves>>>(d, s, n, 1);
    f<<<256, 64 * waves>>>(d, s, n, 2);
    (void)hipDeviceSynchronize();
    long long h[256 * 16];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int b = 0; b < 256; b++)
        for (int w = 0; w < waves; w++) sum += (double)h[b * 16 + w];
    (void)hipFree(d);
    (void)hipFree(s);
    return sum / (256.0 * waves) / n;
}

int main() {
    const double c0 = run(steps<0>, 4), c1 = run(steps<1>, 8), c2 = run(steps<2>, 4), c3 = run(steps<3>, 4);
    printf("int32, 1 wave/SIMD        : %6.1f cycles per step per wave, %5.1f per stripe-step\n", c0, c0);
    printf("int32, 2 waves/SIMD       : %6.1f cycles per step per wave, %5.1f per stripe-step (SIMD view)\n", c1, c1 / 2);
    printf("packed x2, 1 wave/SIMD    : %6.1f cycles per step per wave, %5.1f per stripe-step\n", c2, c2 / 2);
    printf("packed x2 + rebasing      : %6.1f cycles per step per wave, %5.1f per stripe-step\n", c3, c3 / 2);
    return 0;
}
