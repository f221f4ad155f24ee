// Microbenchmark: what each part of the lane fill's sub-chunk machinery (ga_lane.hip) costs on
// top of the bare asm step, one wave per SIMD (4-wave workgroups, 256 of them), 16-step sub-chunks.
// Cycles per step per wave:
//   0  bare: LaneAsm<TD,0,4> x 4
//   1  + 8 ds_read_b128 edge reads per sub-chunk (lane 0 its ring rows, lanes 1..63 one zero block), used next
//   2  + the same with every lane at lane 0's ring address (a broadcast)
//   3  + 2 ds_read_b128 per 4-step block (lane 0 ring, others zero block), used next block
//   4  + profile gathers: TD x 4 dwords per lane per sub-chunk at code-dependent rows (the kernel's table)
//   5  + a sequence window instead: 4 dwords per lane per sub-chunk (row-consecutive, conflict-free), and per
//        block TD v_perm_b32 from an 8-entry per-column byte table (K <= 8)
//   6  + lane 63's 16 rows per sub-chunk from registers under an exec mask (lk_store_rows)
//   7  + per step two DPP shift-register updates, one ds_write_b64 from lanes 48..63 per sub-chunk (exec mask)
//   8  + one counter check per sub-chunk: readfirstlane of a value loaded a sub-chunk ago, compare, branch
//   9  + one counter check per block (the value loaded after the block's first step)
//  10  1 + 4 + 6 + 8: the round-3 asm sub-chunk with its profile and check
//  11  1 + 5 + 6 + 8: the same with the sequence-window profile
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I globalign_amd/csrc tools/micro/lane_parts.hip -o tools/micro/lane_parts
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "ga_lane_asm.h"

using namespace ga;

constexpr int LDSW = 12288;  // ints: [0,4096) profile table, [4096,6144) rings, [6144,8192) zero block, rest scratch

template <int TD, int MODE>
__global__ void __launch_bounds__(512) bench(long long* out, int* sink, int nsteps, int o, int never) {
    __shared__ __attribute__((aligned(16))) int lds[LDSW];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < LDSW; k += blockDim.x) lds[k] = k < 4096 ? (k * 37) & 0x03030303 : (k < 6144 ? k : 0);
    __syncthreads();
    int H[TD], Y[TD];
#pragma unroll
    for (int k = 0; k < TD; k++) {
        H[k] = lane + k;
        Y[k] = lane + 2 * k + 1;
    }
    int Xl = lane + 3, HLp = lane + 1;
    uint32_t q[4][TD];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int k = 0; k < TD; k++) q[c][k] = 0x01020304u * ((lane + k + c) & 3);
    // per-column 8-entry sub' byte tables (mode 5, 11)
    uint32_t tlo[TD], thi[TD];
#pragma unroll
    for (int k = 0; k < TD; k++) {
        tlo[k] = 0x03020100u + (unsigned)(lane + k);
        thi[k] = 0x07060504u + (unsigned)(lane * 3 + k);
    }
    uint32_t sq[4] = {0x01000302u, 0x02010003u, 0x03020100u, 0x00030201u};  // sequence code dwords
    int4 E[8];
#pragma unroll
    for (int k = 0; k < 8; k++) E[k] = make_int4(0, 0, 0, 0);
    int acc = 0, RH = 0, RX = 0;
    unsigned cnt_v = 0;
    int4* ringw = reinterpret_cast<int4*>(lds + 4096 + 512 * (w & 3));
    const int4* zero4 = reinterpret_cast<const int4*>(lds + 6144);
    const unsigned outb = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 4096 + 512 * ((w + 1) & 3));
    const unsigned pc = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 8192 + 16 * (w & 3));
    int ohs[16], oxs[16];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {
        constexpr bool EREAD = MODE == 1 || MODE == 10 || MODE == 11;
        constexpr bool PROF = MODE == 4 || MODE == 10;
        constexpr bool SEQ = MODE == 5 || MODE == 11;
        constexpr bool OUT16 = MODE == 6 || MODE == 10 || MODE == 11;
        constexpr bool CHK = MODE == 8 || MODE == 10 || MODE == 11;
        int eh[16], ex[16];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            eh[2 * k] = E[k].x; ex[2 * k] = E[k].y; eh[2 * k + 1] = E[k].z; ex[2 * k + 1] = E[k].w;
        }
        if constexpr (CHK) {
            if (__builtin_expect((int)__builtin_amdgcn_readfirstlane((int)cnt_v) == never, 0)) acc += 5;
        }
        uint32_t qn[4][TD];
        uint32_t sqn[4];
        int4 En[8];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            int h4[4], x4[4];
            uint32_t qq[TD];
#pragma unroll
            for (int k = 0; k < TD; k++) qq[k] = SEQ ? __builtin_amdgcn_perm(thi[k], tlo[k], sq[d]) : q[d][k];
            if constexpr (MODE == 7) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    LaneAsm<TD, 0, 1>::run(H, Y, Xl, HLp, eh + 4 * d + u, ex + 4 * d + u, qq, o, h4 + u, x4 + u);
                    RH = __builtin_amdgcn_update_dpp(h4[u], RH, 0x130, 0xf, 0xf, false);
                    RX = __builtin_amdgcn_update_dpp(x4[u], RX, 0x130, 0xf, 0xf, false);
                }
            } else {
                LaneAsm<TD, 0, 1>::run(H, Y, Xl, HLp, eh + 4 * d, ex + 4 * d, qq, o, h4, x4);
                if (d == 0) {
                    asm volatile("" ::: "memory");
                    if constexpr (EREAD || MODE == 2) {
                        const int4* src = (MODE == 2 || lane == 0) ? ringw + ((r >> 1) & 63) : zero4;
#pragma unroll
                        for (int k = 0; k < 8; k++) En[k] = src[k];
                    }
                    if constexpr (PROF) {
#pragma unroll
                        for (int k = 0; k < TD; k++) {
                            const int* pk = lds + ((((r + 16 - lane) & 1023) + 1031 * ((lane * 7 + k) & 3)) & 4095);
                            qn[0][k] = pk[0]; qn[1][k] = pk[4]; qn[2][k] = pk[8]; qn[3][k] = pk[12];
                        }
                    }
                    if constexpr (SEQ) {
                        const int* pk = lds + ((r + 16 - lane) & 4095);
                        sqn[0] = pk[0]; sqn[1] = pk[4]; sqn[2] = pk[8]; sqn[3] = pk[12];
                    }
                    if constexpr (CHK || MODE == 8) cnt_v = lds[8192 + 16 * ((w + 3) & 3)];
                    if constexpr (MODE == 12) {  // edge reads from lane 0 only (exec mask), no zero-block returns
                        const unsigned ea = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int4*)(ringw + ((r >> 1) & 63));
                        unsigned long long saved;
                        typedef int v4i __attribute__((ext_vector_type(4)));
                        v4i a0, a1, a2, a3, a4, a5, a6, a7;
                        asm volatile("s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, 1\n\t"
                                     "ds_read_b128 %[a0], %[ea]\n\tds_read_b128 %[a1], %[ea] offset:16\n\t"
                                     "ds_read_b128 %[a2], %[ea] offset:32\n\tds_read_b128 %[a3], %[ea] offset:48\n\t"
                                     "ds_read_b128 %[a4], %[ea] offset:64\n\tds_read_b128 %[a5], %[ea] offset:80\n\t"
                                     "ds_read_b128 %[a6], %[ea] offset:96\n\tds_read_b128 %[a7], %[ea] offset:112\n\t"
                                     "s_mov_b64 exec, %[sv]\n\ts_waitcnt lgkmcnt(0)"
                                     : [sv] "=&s"(saved), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3),
                                       [a4] "=&v"(a4), [a5] "=&v"(a5), [a6] "=&v"(a6), [a7] "=&v"(a7)
                                     : [ea] "v"(ea) : "memory");
                        En[0] = make_int4(a0.x, a0.y, a0.z, a0.w); En[1] = make_int4(a1.x, a1.y, a1.z, a1.w);
                        En[2] = make_int4(a2.x, a2.y, a2.z, a2.w); En[3] = make_int4(a3.x, a3.y, a3.z, a3.w);
                        En[4] = make_int4(a4.x, a4.y, a4.z, a4.w); En[5] = make_int4(a5.x, a5.y, a5.z, a5.w);
                        En[6] = make_int4(a6.x, a6.y, a6.z, a6.w); En[7] = make_int4(a7.x, a7.y, a7.z, a7.w);
                    }
                    asm volatile("" ::: "memory");
                }
                if constexpr (MODE == 3) {
                    asm volatile("" ::: "memory");
                    const int4* src = lane == 0 ? ringw + ((r + 4 * d) & 63) : zero4;
                    En[2 * d] = src[0];
                    En[2 * d + 1] = src[1];
                    asm volatile("" ::: "memory");
                }
                if constexpr (MODE == 9) {
                    asm volatile("" ::: "memory");
                    cnt_v = lds[8192 + 16 * ((w + 3) & 3) + d];
                    asm volatile("" ::: "memory");
                }
                LaneAsm<TD, 1, 3>::run(H, Y, Xl, HLp, eh + 4 * d + 1, ex + 4 * d + 1, qq, o, h4 + 1, x4 + 1);
                if constexpr (MODE == 9) {
                    if (__builtin_expect((int)__builtin_amdgcn_readfirstlane((int)cnt_v) == never, 0)) acc += 5;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                ohs[4 * d + u] = h4[u];
                oxs[4 * d + u] = x4[u];
            }
        }
        if constexpr (OUT16) lk_store_rows(outb + 8 * (r & 63), outb + 8 * (r & 63) + 120, pc, lk_v2u{(unsigned)r, 0u}, ohs, oxs);
        if constexpr (MODE == 7) {
            unsigned long long saved;
            const unsigned oaddr = outb + 8u * (unsigned)((r + lane) & 127);
            typedef int v2i_t __attribute__((ext_vector_type(2)));
            const v2i_t hx = {RH, RX};
            asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, %3\n\tds_write_b64 %1, %2\n\ts_mov_b64 exec, %0\n\ts_nop 4"
                         : "=&s"(saved) : "v"(oaddr), "v"(hx), "s"(0xffff000000000000ull) : "memory");
        }
        if constexpr (EREAD || MODE == 2 || MODE == 3 || MODE == 12) {
#pragma unroll
            for (int k = 0; k < 8; k++) E[k] = En[k];
        } else {
            acc ^= ohs[3];
        }
        if constexpr (PROF) {
#pragma unroll
            for (int c = 0; c < 4; c++)
#pragma unroll
                for (int k = 0; k < TD; k++) q[c][k] = qn[c][k];
        }
        if constexpr (SEQ) {
#pragma unroll
            for (int c = 0; c < 4; c++) sq[c] = sqn[c];
        }
        acc ^= oxs[15];
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    int z = Xl + HLp + acc + E[0].x + E[7].w + RH + RX;
#pragma unroll
    for (int k = 0; k < TD; k++) z += H[k] + Y[k];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = z;
}

template <typename F>
double run(F kern, int blocks, int n, int threads = 256) {
    long long* d;
    int* s;
    (void)hipMalloc(&d, 16 * blocks * sizeof(long long));
    (void)hipMalloc(&s, blocks * threads * sizeof(int));
    kern<<<blocks, threads>>>(d, s, n, 5, -1000);
    kern<<<blocks, threads>>>(d, s, n, 5, -1000);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * blocks);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> v;
    for (int b = 0; b < blocks; b++)
        for (int w = 0; w < threads / 64; w++) v.push_back((double)h[b * 16 + w]);
    std::sort(v.begin(), v.end());
    (void)hipFree(d);
    (void)hipFree(s);
    return v[v.size() / 2] / n;  // median wave
}

template <int TD>
void row() {
    const int n = 1 << 14;
    auto fns = std::vector<void (*)(long long*, int*, int, int, int)>{
        bench<TD, 0>, bench<TD, 1>, bench<TD, 2>, bench<TD, 3>, bench<TD, 4>, bench<TD, 5>,
        bench<TD, 6>, bench<TD, 7>, bench<TD, 8>, bench<TD, 9>, bench<TD, 10>, bench<TD, 11>};
    const char* modes[] = {"bare steps", "+ 8 b128 edge reads / 16", "+ 8 b128 broadcast / 16", "+ 2 b128 per block",
                           "+ profile gathers", "+ sequence window + v_perm", "+ lane-63 16-row store",
                           "+ DPP shift regs + b64 store", "+ 1 check / sub-chunk", "+ 1 check / block",
                           "r3: edges+prof+store+check", "r3 with seq window + v_perm"};
    for (size_t v = 0; v < fns.size(); v++) printf("TD=%d %-30s %6.1f cyc/step/wave\n", TD, modes[v], run(fns[v], 256, n));
    printf("TD=%d %-30s %6.1f cyc/step/wave\n", TD, "+ exec-masked edge reads (wait)", run(bench<TD, 12>, 256, n));
    printf("TD=%d %-30s %6.1f cyc/step/wave (2 waves/SIMD)\n", TD, "bare steps", run(bench<TD, 0>, 256, n, 512));
    printf("TD=%d %-30s %6.1f cyc/step/wave (2 waves/SIMD)\n", TD, "r3: edges+prof+store+check", run(bench<TD, 10>, 256, n, 512));
}

int main() {
    row<1>();
    row<2>();
    row<4>();
    return 0;
}
