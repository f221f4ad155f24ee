// Microbenchmark: latency of the walker's step chain (v_readlane -> SALU ops -> lane
// index -> v_readlane), one wave alone on its SIMD.  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V>
__global__ void chain(long long* out, unsigned* sink) {
    unsigned win = (threadIdx.x * 7u) & 63u;
    unsigned s = 3, t = 0x9e3779b9u;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long t0 = __builtin_amdgcn_s_memtime();
    long long r0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int it = 0; it < 4096; it++) {
        if (V == 0)  // readlane + 8 SALU (the current walker step)
            asm volatile(".rept 16\n"
                         "v_readlane_b32 %0, %1, %0\n"
                         "s_lshr_b32 %0, %0, 1\n s_lshr_b32 %0, %2, %0\n s_and_b32 %0, %0, 3\n s_lshl_b32 %0, %0, 3\n"
                         "s_lshr_b32 %0, 0x80109, %0\n s_and_b32 %0, %0, 9\n s_add_u32 %0, %0, 5\n s_and_b32 %0, %0, 63\n"
                         ".endr" : "+s"(s) : "v"(win), "s"(t) : "memory");
        if (V == 1)  // 8 dependent SALU only
            asm volatile(".rept 16\n"
                         "s_lshr_b32 %0, %0, 1\n s_lshr_b32 %0, %2, %0\n s_and_b32 %0, %0, 3\n s_lshl_b32 %0, %0, 3\n"
                         "s_lshr_b32 %0, 0x80109, %0\n s_and_b32 %0, %0, 9\n s_add_u32 %0, %0, 5\n s_and_b32 %0, %0, 63\n"
                         ".endr" : "+s"(s) : "v"(win), "s"(t) : "memory");
        if (V == 2)  // readlane + 1 SALU
            asm volatile(".rept 16\nv_readlane_b32 %0, %1, %0\ns_and_b32 %0, %0, 63\n.endr" : "+s"(s) : "v"(win), "s"(t) : "memory");
        if (V == 3)  // readlane + 3 SALU
            asm volatile(".rept 16\nv_readlane_b32 %0, %1, %0\ns_lshr_b32 %0, %0, 1\ns_lshr_b32 %0, %2, %0\ns_and_b32 %0, %0, 63\n.endr"
                         : "+s"(s) : "v"(win), "s"(t) : "memory");
        if (V == 4)  // s_bfe + readlane
            asm volatile(".rept 16\nv_readlane_b32 %0, %1, %0\ns_bfe_u32 %0, %0, 0x60000\n.endr" : "+s"(s) : "v"(win), "s"(t) : "memory");
        if (V == 5)  // VALU dependent chain (reference: 8 v_min)
            asm volatile(".rept 16\nv_min_i32 %0, %0, %1\nv_min_i32 %0, %0, %1\nv_min_i32 %0, %0, %1\nv_min_i32 %0, %0, %1\n"
                         "v_min_i32 %0, %0, %1\nv_min_i32 %0, %0, %1\nv_min_i32 %0, %0, %1\nv_min_i32 %0, %0, %1\n.endr"
                         : "+v"(win) : "v"(t) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long t1 = __builtin_amdgcn_s_memtime();
    long long r1 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    long long* d; unsigned* s; long long h[4];
    (void)hipMalloc(&d, 64 * sizeof(long long));
    (void)hipMalloc(&s, 64 * 64 * sizeof(unsigned));
    const char* names[] = {"readlane + 8 SALU", "8 SALU only", "readlane + 1 SALU", "readlane + 3 SALU", "readlane + s_bfe",
                           "8 v_min (VALU ref)"};
    void (*fns[])(long long*, unsigned*) = {chain<0>, chain<1>, chain<2>, chain<3>, chain<4>, chain<5>};
    for (int v = 0; v < 6; v++) {
        fns[v]<<<1, 64>>>(d, s);
        fns[v]<<<1, 64>>>(d, s);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, d, 2 * sizeof(long long), hipMemcpyDeviceToHost);
        const double ns = h[1] * 10.0 / (4096.0 * 16);  // s_memrealtime: 100 MHz
        printf("%-22s %.2f ns per step (%.1f cycles at 2.4 GHz); memtime ticks per step %.1f\n", names[v], ns, ns * 2.4,
               h[0] / (4096.0 * 16));
    }
    return 0;
}
