// Microbenchmark: what the fine-grained edge hand-over (ga_lane.hip) adds to the lane step.
// Cycles per step per wave, one wave per SIMD (4-wave workgroups, 256 of them), 16-step sub-chunks of four
// 4-step blocks, the kernel's own asm (ga_lane_asm.h):
//   0  LaneAsm<TD,0,4> x 4: the bare steps
//   1  LaneBlk x 4: the steps with the counter + edge reads after each block's first step and the wait
//   2  1 + the counter check (v_readfirstlane, compare, a branch never taken)
//   3  2 + the publish (lk_store_rows4: 4 rows + counters from lane 63 under an exec mask)
//   4  3 + a uniform branch around a skipped region per block (the kernel's hand_direct test)
//   5  3 with the publish's counter store only at the sub-chunk's last block
//   6  3 without the publish's trailing s_nop (exec restored first)
//   7  the round-3 asm path: 16 steps, edge reads after step 12, one 16-row store per sub-chunk
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I globalign_amd/csrc tools/micro/lane_fine.hip -o tools/micro/lane_fine
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "ga_lane_asm.h"

using namespace ga;

template <int TD, int MODE>
__global__ void __launch_bounds__(384) bench(long long* out, int* sink, int nsteps, int o, int never) {
    __shared__ __attribute__((aligned(16))) int lds[8192 + 2048];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < 8192 + 2048; k += blockDim.x) lds[k] = k < 4096 ? (k * 37) & 0x03030303 : 0;
    __syncthreads();
    if (w >= 4) {  // mode 13's aux wave: poll an LDS word with s_sleep 1 until the compute waves finish
        unsigned spins = 0;
        while (__hip_atomic_load(&lds[8192 + 2040], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4 && spins < (1u << 22)) {
            __builtin_amdgcn_s_sleep(1);
            spins++;
        }
        return;
    }
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
    lk_v4i E0 = {1, 2, 3, 4}, E1 = {5, 6, 7, 8};
    int acc = 0;
    const unsigned ring_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 4096);
    const unsigned zero_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 8192);
    const unsigned ebase = lane == 0 ? ring_lds : zero_lds;
    const unsigned ca = ring_lds + 2048 * 4 - 64 + 8 * w;  // a counter slot (0 / never reached)
    const unsigned outb = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 4096 + 512 * w);
    const unsigned pc = ca;
    // a scratch area of 80 bytes per lane (the non-63 lanes' writes of the all-lanes publish)
    const unsigned scr = (unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)(lds + 8192 + 512) + 8u * (unsigned)lane;
    int ohs[16], oxs[16];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {
        if constexpr (MODE == 12 || MODE == 13 || MODE == 14 || MODE == 15 || MODE == 16) {
            // 14: only the profile gathers, 15: only the three checks, 16: only the skipped store region
            constexpr bool QL = MODE != 15 && MODE != 16, CK = MODE != 14 && MODE != 16, SK = MODE != 14 && MODE != 15;
            // the round-3 asm sub-chunk with the kernel's per-sub-chunk extras: profile gathers for the next
            // sub-chunk, the producer counter read and checks, a uniform branch around skipped stores (flush_pend),
            // the ring-space check; 13: and an idle-polling aux wave (blockDim 320: wave 4 spins on an LDS word)
            int eh[16], ex[16];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                eh[u] = u & 1 ? E0.z : E0.x;
                ex[u] = u & 1 ? E1.w : E1.y;
            }
            if (CK && (int)__builtin_amdgcn_readfirstlane(acc) == never) acc += 3;  // a wait check, never taken
            LaneAsm<TD, 0, 4>::run(H, Y, Xl, HLp, eh, ex, q[0], o, ohs, oxs);
            uint32_t qn[4][TD];
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < TD; k++) {
                if (QL) {
                    const int* pk = lds + ((((r + 16 - lane) & 1023) + 1031 * ((lane * 7 + k) & 3)) & 4095);
                    qn[0][k] = pk[0]; qn[1][k] = pk[4]; qn[2][k] = pk[8]; qn[3][k] = pk[12];
                } else {
                    qn[0][k] = q[1][k]; qn[1][k] = q[2][k]; qn[2][k] = q[3][k]; qn[3][k] = q[0][k];
                }
            }
            asm volatile("" ::: "memory");
            if (SK && never > 0 && r > never) {  // flush_pend's store region, skipped
                if (lane < 16) sink[r + lane] = Xl;
            }
            LaneAsm<TD, 0, 4>::run(H, Y, Xl, HLp, eh + 4, ex + 4, q[1], o, ohs + 4, oxs + 4);
            LaneAsm<TD, 0, 4>::run(H, Y, Xl, HLp, eh + 8, ex + 8, q[2], o, ohs + 8, oxs + 8);
            LaneAsm<TD, 0, 1>::run(H, Y, Xl, HLp, eh + 12, ex + 12, q[3], o, ohs + 12, oxs + 12);
            asm volatile("" ::: "memory");
            if (CK && (int)__builtin_amdgcn_readfirstlane(acc) == never + 1) acc += 5;  // the edge wait check
            const int4* src = reinterpret_cast<const int4*>(lds + 4096 + ((r * 8) & 1023));
            int4 n[8];
#pragma unroll
            for (int k = 0; k < 8; k++) n[k] = src[k];
            const int pn = lds[4096 + 2040 + w];
            asm volatile("" ::: "memory");
            LaneAsm<TD, 1, 3>::run(H, Y, Xl, HLp, eh + 13, ex + 13, q[3], o, ohs + 13, oxs + 13);
            if (CK && (int)__builtin_amdgcn_readfirstlane(pn) == never + 2) acc += 7;  // the ring-space check
            lk_store_rows(outb + 8 * (r & 63), outb + 8 * (r & 63) + 120, pc, lk_v2u{(unsigned)r, 0u}, ohs, oxs);
            E0 = lk_v4i{n[0].x, n[0].y, n[0].z, n[0].w};
            E1 = lk_v4i{n[1].x, n[1].y, n[1].z, n[1].w};
            acc ^= n[7].x;
#pragma unroll
            for (int c = 0; c < 4; c++)
#pragma unroll
                for (int k = 0; k < TD; k++) q[c][k] = qn[c][k];
        } else if constexpr (MODE == 7) {
            int eh[16], ex[16];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                eh[u] = u & 1 ? E0.z : E0.x;
                ex[u] = u & 1 ? E1.w : E1.y;
            }
            LaneAsm<TD, 0, 4>::run(H, Y, Xl, HLp, eh, ex, q[0], o, ohs, oxs);
            LaneAsm<TD, 0, 4>::run(H, Y, Xl, HLp, eh + 4, ex + 4, q[1], o, ohs + 4, oxs + 4);
            LaneAsm<TD, 0, 4>::run(H, Y, Xl, HLp, eh + 8, ex + 8, q[2], o, ohs + 8, oxs + 8);
            LaneAsm<TD, 0, 1>::run(H, Y, Xl, HLp, eh + 12, ex + 12, q[3], o, ohs + 12, oxs + 12);
            asm volatile("" ::: "memory");
            const int4* src = reinterpret_cast<const int4*>(lds + 4096 + ((r * 8) & 1023));
            int4 n[8];
#pragma unroll
            for (int k = 0; k < 8; k++) n[k] = src[k];
            asm volatile("" ::: "memory");
            LaneAsm<TD, 1, 3>::run(H, Y, Xl, HLp, eh + 13, ex + 13, q[3], o, ohs + 13, oxs + 13);
            lk_store_rows(outb + 8 * (r & 63), outb + 8 * (r & 63) + 120, pc, lk_v2u{(unsigned)r, 0u}, ohs, oxs);
            E0 = lk_v4i{n[0].x, n[0].y, n[0].z, n[0].w};
            E1 = lk_v4i{n[1].x, n[1].y, n[1].z, n[1].w};
            acc ^= n[7].x;
        } else {
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const int eh4[4] = {E0.x, E0.z, E1.x, E1.z}, ex4[4] = {E0.y, E0.w, E1.y, E1.w};
                int h4[4], x4[4];
                if constexpr (MODE == 0) {
                    LaneAsm<TD, 0, 4>::run(H, Y, Xl, HLp, eh4, ex4, q[d], o, h4, x4);
                    E0.x ^= h4[0];
                } else {
                    unsigned cv;
                    lk_v4i N0, N1;
                    LaneBlk<TD>::run(H, Y, Xl, HLp, eh4, ex4, q[d], o, h4, x4, ca, ebase + (unsigned)((r + 4 * d) & 255) * 8u,
                                     cv, N0, N1);
                    if constexpr (MODE >= 2) {
                        if (__builtin_expect((int)__builtin_amdgcn_readfirstlane((int)cv) < never, 0)) {
                            acc += __builtin_amdgcn_readfirstlane(N0.x);
                            asm volatile("s_sleep 1" ::: "memory");
                        }
                    }
                    if constexpr (MODE >= 8) {
                        // publish variants: 8 no trailing s_nop; 9 exec juggling only; 10 every lane writes (lane 63 the
                        // ring, the others a scratch row of their own), no exec change; 11 = 10 without the counter
                        const unsigned b1 = outb + 8u * (unsigned)(r & 63);
                        if constexpr (MODE == 8) {
                            unsigned long long saved;
                            asm volatile(
                                "s_mov_b64 %[saved], exec\n\ts_mov_b64 exec, %[m63]\n\t"
                                "ds_write2_b32 %[b1], %[h0], %[x0] offset0:0 offset1:1\n\t"
                                "ds_write2_b32 %[b1], %[h1], %[x1] offset0:2 offset1:3\n\t"
                                "ds_write2_b32 %[b1], %[h2], %[x2] offset0:4 offset1:5\n\t"
                                "ds_write2_b32 %[b1], %[h3], %[x3] offset0:6 offset1:7\n\t"
                                "ds_write_b64 %[pc], %[cp]\n\ts_mov_b64 exec, %[saved]"
                                : [saved] "=&s"(saved)
                                : [b1] "v"(b1), [pc] "v"(pc), [cp] "v"(lk_v2u{(unsigned)r, (unsigned)r}), [m63] "s"(1ull << 63),
                                  [h0] "v"(h4[0]), [h1] "v"(h4[1]), [h2] "v"(h4[2]), [h3] "v"(h4[3]), [x0] "v"(x4[0]),
                                  [x1] "v"(x4[1]), [x2] "v"(x4[2]), [x3] "v"(x4[3])
                                : "memory");
                        } else if constexpr (MODE == 9) {
                            unsigned long long saved;
                            asm volatile("s_mov_b64 %[saved], exec\n\ts_mov_b64 exec, %[m63]\n\ts_mov_b64 exec, %[saved]\n\ts_nop 4"
                                         : [saved] "=&s"(saved) : [m63] "s"(1ull << 63) : "memory");
                        } else {
                            const unsigned wa = lane == 63 ? b1 : scr;
                            if constexpr (MODE == 10)
                                asm volatile(
                                    "ds_write2_b32 %[b1], %[h0], %[x0] offset0:0 offset1:1\n\t"
                                    "ds_write2_b32 %[b1], %[h1], %[x1] offset0:2 offset1:3\n\t"
                                    "ds_write2_b32 %[b1], %[h2], %[x2] offset0:4 offset1:5\n\t"
                                    "ds_write2_b32 %[b1], %[h3], %[x3] offset0:6 offset1:7\n\t"
                                    "ds_write_b64 %[pc], %[cp]"
                                    :
                                    : [b1] "v"(wa), [pc] "v"(lane == 63 ? pc : scr + 64), [cp] "v"(lk_v2u{(unsigned)r, (unsigned)r}),
                                      [h0] "v"(h4[0]), [h1] "v"(h4[1]), [h2] "v"(h4[2]), [h3] "v"(h4[3]), [x0] "v"(x4[0]),
                                      [x1] "v"(x4[1]), [x2] "v"(x4[2]), [x3] "v"(x4[3])
                                    : "memory");
                            else
                                asm volatile(
                                    "ds_write2_b32 %[b1], %[h0], %[x0] offset0:0 offset1:1\n\t"
                                    "ds_write2_b32 %[b1], %[h1], %[x1] offset0:2 offset1:3\n\t"
                                    "ds_write2_b32 %[b1], %[h2], %[x2] offset0:4 offset1:5\n\t"
                                    "ds_write2_b32 %[b1], %[h3], %[x3] offset0:6 offset1:7"
                                    :
                                    : [b1] "v"(wa), [h0] "v"(h4[0]), [h1] "v"(h4[1]), [h2] "v"(h4[2]), [h3] "v"(h4[3]),
                                      [x0] "v"(x4[0]), [x1] "v"(x4[1]), [x2] "v"(x4[2]), [x3] "v"(x4[3])
                                    : "memory");
                        }
                    } else if constexpr (MODE >= 3) {
                        const unsigned b1 = outb + 8u * (unsigned)(r & 63);
                        if constexpr (MODE == 5) {
                            if (d == 3) {
                                if (d == 3) lk_store_rows4<3>(b1, b1 + 120, pc, lk_v2u{(unsigned)r, (unsigned)r}, h4, x4);
                            }
                        } else {
                            switch (d) {
                                case 0: lk_store_rows4<0>(b1, b1 + 120, pc, lk_v2u{(unsigned)r, (unsigned)r}, h4, x4); break;
                                case 1: lk_store_rows4<1>(b1, b1 + 120, pc, lk_v2u{(unsigned)r, (unsigned)r}, h4, x4); break;
                                case 2: lk_store_rows4<2>(b1, b1 + 120, pc, lk_v2u{(unsigned)r, (unsigned)r}, h4, x4); break;
                                default: lk_store_rows4<3>(b1, b1 + 120, pc, lk_v2u{(unsigned)r, (unsigned)r}, h4, x4); break;
                            }
                        }
                    }
                    if constexpr (MODE == 4) {
                        if (never == 12345 && lane == 63) sink[r] = h4[0];
                    }
                    E0 = N0;
                    E1 = N1;
                }
            }
        }
        acc ^= Xl;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    if (lane == 0) __hip_atomic_fetch_add(&lds[8192 + 2040], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    int z = Xl + HLp + acc + E0.x + E1.y;
#pragma unroll
    for (int k = 0; k < TD; k++) z += H[k] + Y[k];
    sink[4096 + blockIdx.x * blockDim.x + threadIdx.x] = z;
}

template <typename F>
double run(F kern, int blocks, int n, int threads = 256) {
    long long* d;
    int* s;
    (void)hipMalloc(&d, 16 * blocks * sizeof(long long));
    (void)hipMalloc(&s, (4096 + blocks * 256) * sizeof(int));
    kern<<<blocks, threads>>>(d, s, n, 5, -1000);
    kern<<<blocks, threads>>>(d, s, n, 5, -1000);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * blocks);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int b = 0; b < blocks; b++)
        for (int w = 0; w < 4; w++) mx = std::max(mx, (double)h[b * 16 + w]);
    (void)hipFree(d);
    (void)hipFree(s);
    return mx / n;
}

template <int TD>
void row() {
    const int n = 1 << 14;
    auto fns = std::vector<void (*)(long long*, int*, int, int, int)>{
        bench<TD, 0>, bench<TD, 1>, bench<TD, 2>, bench<TD, 3>, bench<TD, 4>, bench<TD, 5>, bench<TD, 7>,
        bench<TD, 8>, bench<TD, 9>, bench<TD, 10>, bench<TD, 11>};
    const char* modes[] = {"bare asm steps", "+ reads/wait per block", "+ counter check", "+ publish per block",
                           "+ skipped uniform branch", "publish only last block", "round-3 asm sub-chunk",
                           "check + publish, no s_nop", "check + exec juggling only", "check + all-lane publish",
                           "check + all-lane rows only"};
    for (size_t v = 0; v < fns.size(); v++) printf("TD=%d %-28s %6.1f cyc/step/wave\n", TD, modes[v], run(fns[v], 256, n));
    printf("TD=%d %-28s %6.1f cyc/step/wave\n", TD, "r3 + kernel extras", run(bench<TD, 12>, 256, n));
    printf("TD=%d %-28s %6.1f cyc/step/wave\n", TD, "r3 + profile gathers", run(bench<TD, 14>, 256, n));
    printf("TD=%d %-28s %6.1f cyc/step/wave\n", TD, "r3 + 3 checks", run(bench<TD, 15>, 256, n));
    printf("TD=%d %-28s %6.1f cyc/step/wave\n", TD, "r3 + skipped store region", run(bench<TD, 16>, 256, n));
    printf("TD=%d %-28s %6.1f cyc/step/wave\n", TD, "r3 + extras + 1 aux wave", run(bench<TD, 13>, 256, n, 320));
    printf("TD=%d %-28s %6.1f cyc/step/wave\n", TD, "r3 + extras + 2 aux waves", run(bench<TD, 13>, 256, n, 384));
}

int main() {
    row<1>();
    row<2>();
    row<4>();
    return 0;
}
