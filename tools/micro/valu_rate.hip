// Microbenchmark: issue throughput (cycles per wave64 instruction, s_memtime) of
// VALU forms the fill could use; 4 independent chains, one and two waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define OPS4(op) ".rept 64\n" op " %0, %0, %4\n" op " %1, %1, %4\n" op " %2, %2, %4\n" op " %3, %3, %4\n.endr\n"
#define OPS4_S(op, suf) ".rept 64\n" op " %0, %4, %0 " suf "\n" op " %1, %4, %1 " suf "\n" op " %2, %4, %2 " suf "\n" op " %3, %4, %3 " suf "\n.endr\n"
#define OPS4_M(op, suf) ".rept 64\n" op " %0, %4 " suf "\n" op " %1, %4 " suf "\n" op " %2, %4 " suf "\n" op " %3, %4 " suf "\n.endr\n"
#define OPS4_3(op) ".rept 64\n" op " %0, %0, %4, %1\n" op " %1, %1, %4, %2\n" op " %2, %2, %4, %3\n" op " %3, %3, %4, %0\n.endr\n"

template <int V>
__global__ void indep(long long* out, int* sink) {
    int a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3, y = a * 3 + 7;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 16; it++) {
#define R(str) asm volatile(str : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(y))
        if (V == 0) R(OPS4("v_min_i32"));
        if (V == 1) R(OPS4("v_min_u32"));
        if (V == 2) R(OPS4("v_sub_u32"));
        if (V == 3) R(OPS4("v_max_i32"));
        if (V == 4) R(OPS4_3("v_med3_i32"));
        if (V == 5) R(OPS4_3("v_lshl_or_b32"));
        if (V == 6) R(OPS4_3("v_or3_b32"));
        if (V == 7) R(OPS4("v_pk_min_i16"));
        if (V == 8) R(OPS4("v_pk_add_u16"));
        if (V == 9) R(OPS4("v_cvt_pk_u16_u32"));
        if (V == 10) R(OPS4_3("v_perm_b32"));
        if (V == 11) R(OPS4_3("v_add3_u32"));
        if (V == 12) R(OPS4_3("v_bfe_i32"));
        if (V == 13) R(OPS4("v_and_b32"));
        if (V == 14) R(OPS4("v_or_b32"));
        if (V == 15) R(OPS4("v_lshlrev_b32"));
        if (V == 16) R(OPS4_3("v_min3_i32"));
        if (V == 17) R(OPS4("v_pk_min_u16"));
        if (V == 18) R(OPS4("v_min_i16"));
        if (V == 19) R(OPS4("v_sub_i32"));
        if (V == 20) R(OPS4("v_add_co_u32"));
        if (V == 21) R(OPS4_3("v_add_lshl_u32"));
        if (V == 22) R(OPS4("v_pk_max_i16"));
        if (V == 23) R(OPS4_3("v_min3_u32"));
        // forms the fill's hot loop uses (tools/valu_mix.py); the DPP / SDWA source is the
        // loop-invariant %4, so no VALU->DPP hazard applies
        if (V == 24) R(OPS4_S("v_min_i32_dpp", "row_shr:1 row_mask:0xf bank_mask:0xf"));
        if (V == 25) R(OPS4_M("v_mov_b32_dpp", "row_shr:1 row_mask:0xf bank_mask:0xf"));
        if (V == 26) R(OPS4_M("v_mov_b32", ""));
        if (V == 27) R(OPS4_S("v_add_u32_sdwa", "dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"));
        if (V == 28) R(OPS4_S("v_min_i32_dpp", "row_bcast:15 row_mask:0xa bank_mask:0xf"));
#undef R
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x % 64 == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}

template <typename F>
double run(F kern, int waves, int blocks) {
    long long* d; int* s;
    (void)hipMalloc(&d, 16 * blocks * sizeof(long long));
    (void)hipMalloc(&s, blocks * waves * 64 * sizeof(int));
    kern<<<blocks, waves * 64>>>(d, s);
    kern<<<blocks, waves * 64>>>(d, s);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * blocks);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int b = 0; b < blocks; b++) for (int w = 0; w < waves; w++) mx = std::max(mx, (double)h[b * 16 + w]);
    (void)hipFree(d); (void)hipFree(s);
    return mx;
}

int main() {
    const char* names[] = {"v_min_i32", "v_min_u32", "v_sub_u32", "v_max_i32", "v_med3_i32", "v_lshl_or_b32",
                           "v_or3_b32", "v_pk_min_i16", "v_pk_add_u16", "v_cvt_pk_u16_u32", "v_perm_b32", "v_add3_u32",
                           "v_bfe_i32", "v_and_b32", "v_or_b32", "v_lshlrev_b32", "v_min3_i32", "v_pk_min_u16",
                           "v_min_i16", "v_sub_i32", "v_add_co_u32", "v_add_lshl_u32", "v_pk_max_i16", "v_min3_u32", "v_min_i32_dpp", "v_mov_b32_dpp", "v_mov_b32",
                           "v_add_u32_sdwa", "v_min_i32_dpp bcast15"};
    auto fns = std::vector<void (*)(long long*, int*)>{
        indep<0>, indep<1>, indep<2>, indep<3>, indep<4>, indep<5>, indep<6>, indep<7>, indep<8>, indep<9>, indep<10>,
        indep<11>, indep<12>, indep<13>, indep<14>, indep<15>, indep<16>, indep<17>, indep<18>, indep<19>, indep<20>,
        indep<21>, indep<22>, indep<23>, indep<24>, indep<25>, indep<26>, indep<27>, indep<28>};
    const double n = 16.0 * 64 * 4;
    for (int v = 0; v < (int)fns.size(); v++) {
        double c1 = run(fns[v], 4, 256) / n, c2 = run(fns[v], 8, 256) / n;
        printf("%-18s 1 wave/SIMD %5.2f cyc/op   2 waves/SIMD %5.2f cyc/op (per wave)\n", names[v], c1, c2);
    }
    return 0;
}
