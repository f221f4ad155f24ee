// Microbenchmark: dependent-chain latency (cycles, s_memtime) of the VALU / DPP
// forms the row-scan fill uses, one wave per SIMD and two.  hipcc --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define REP 64
#define CHAIN(body) asm volatile(".rept 64\n" body ".endr\n" : "+v"(x) : "v"(y))

template <int V>
__global__ void chain(long long* out, int* sink) {
    int x = threadIdx.x, y = threadIdx.x * 3 + 1;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 16; it++) {
        if (V == 0) CHAIN("v_min_i32 %0, %0, %1\n");
        if (V == 1) CHAIN("v_min_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\ns_nop 1\n");
        if (V == 2) CHAIN("v_min_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\ns_nop 1\n");
        if (V == 3) CHAIN("v_min_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\ns_nop 1\n");
        if (V == 4) CHAIN("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\ns_nop 1\n");
        if (V == 5) CHAIN("v_add_u32 %0, %0, %1\n");
        if (V == 6) CHAIN("v_min3_i32 %0, %0, %1, %0\n");
        if (V == 7) CHAIN("v_min_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\ns_nop 4\n");
        if (V == 8) CHAIN("v_min_i32_dpp %0, %0, %0 quad_perm:[0,0,1,2] row_mask:0xf bank_mask:0xf\ns_nop 1\n");
        if (V == 9) CHAIN("v_min_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\ns_nop 1\nv_min_i32 %0, %0, %1\n");
        if (V == 10) CHAIN("v_permlane32_swap_b32 %0, %1\n");
        if (V == 11) CHAIN("s_nop 1\n");
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x % 64 == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// independent: 4 chains interleaved (throughput)
template <int V>
__global__ void indep(long long* out, int* sink) {
    int a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3, y = a * 3;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 16; it++) {
        if (V == 0)
            asm volatile(".rept 64\nv_min_i32 %0, %0, %4\nv_min_i32 %1, %1, %4\nv_min_i32 %2, %2, %4\nv_min_i32 %3, %3, %4\n.endr\n"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(y));
        if (V == 1)
            asm volatile(".rept 64\nv_min_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\nv_min_i32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf\nv_min_i32_dpp %2, %2, %2 row_shr:1 row_mask:0xf bank_mask:0xf\nv_min_i32_dpp %3, %3, %3 row_shr:1 row_mask:0xf bank_mask:0xf\n.endr\n"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(y));
        if (V == 2)
            asm volatile(".rept 64\nv_min_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\nv_min_i32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\nv_min_i32_dpp %2, %2, %2 row_bcast:31 row_mask:0xc bank_mask:0xf\nv_min_i32_dpp %3, %3, %3 row_bcast:31 row_mask:0xc bank_mask:0xf\n.endr\n"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(y));
        if (V == 3)
            asm volatile(".rept 64\nv_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n.endr\n"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(y));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x % 64 == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}

// LDS round trip between two waves of one workgroup: ping-pong on a counter
__global__ void pingpong(long long* out, int iters) {
    __shared__ unsigned flag[2];
    const int w = threadIdx.x >> 6;
    if (threadIdx.x < 2) flag[threadIdx.x] = 0;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 1; k <= iters; k++) {
        if (w == 0) {
            __hip_atomic_store(&flag[0], (unsigned)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            while (__hip_atomic_load(&flag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)k) {}
        } else {
            while (__hip_atomic_load(&flag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)k) {}
            __hip_atomic_store(&flag[1], (unsigned)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

// LDS read latency (dependent chain of ds_read_b32)
__global__ void ldslat(long long* out) {
    __shared__ int buf[1024];
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) buf[k] = (k + 1) & 1023;
    __syncthreads();
    int p = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 256; k++) p = buf[p];
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = p; }
}

template <typename F>
double run(F kern, int waves, int blocks) {
    long long* d; int* s;
    hipMalloc(&d, 16 * blocks * sizeof(long long));
    hipMalloc(&s, blocks * waves * 64 * sizeof(int));
    kern<<<blocks, waves * 64>>>(d, s);
    kern<<<blocks, waves * 64>>>(d, s);
    hipDeviceSynchronize();
    std::vector<long long> h(16 * blocks);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int b = 0; b < blocks; b++) for (int w = 0; w < waves; w++) mx = std::max(mx, (double)h[b * 16 + w]);
    hipFree(d); hipFree(s);
    return mx;
}

int main() {
    const char* names[] = {"v_min", "min_dpp row_shr:1 +nop1", "min_dpp row_bcast:15 +nop1", "min_dpp row_bcast:31 +nop1",
                           "mov_dpp wave_shr:1 +nop1", "v_add", "v_min3", "min_dpp row_shr:1 +nop4",
                           "min_dpp quad_perm +nop1", "min_dpp row_shr:1 +nop1 + v_min", "v_permlane32_swap", "s_nop 1"};
    auto fns = std::vector<void (*)(long long*, int*)>{chain<0>, chain<1>, chain<2>, chain<3>, chain<4>, chain<5>,
                                                        chain<6>, chain<7>, chain<8>, chain<9>, chain<10>, chain<11>};
    const double n = 16.0 * 64;
    for (int v = 0; v < (int)fns.size(); v++) {
        double c1 = run(fns[v], 4, 256) / n, c2 = run(fns[v], 8, 256) / n;
        printf("chain %-36s  1 wave/SIMD %6.2f cyc/op   2 waves/SIMD %6.2f cyc/op\n", names[v], c1, c2);
    }
    const char* inames[] = {"v_min x4", "min_dpp row_shr:1 x4", "min_dpp row_bcast:31 x4", "mov_dpp wave_shr:1 x4"};
    auto ifs = std::vector<void (*)(long long*, int*)>{indep<0>, indep<1>, indep<2>, indep<3>};
    for (int v = 0; v < 4; v++) {
        double c1 = run(ifs[v], 4, 256) / (n * 4), c2 = run(ifs[v], 8, 256) / (n * 4);
        printf("indep %-36s  1 wave/SIMD %6.2f cyc/op   2 waves/SIMD %6.2f cyc/op\n", inames[v], c1, c2);
    }
    long long* d; hipMalloc(&d, 64);
    long long h[2];
    pingpong<<<1, 128>>>(d, 1000); pingpong<<<1, 128>>>(d, 1000); hipDeviceSynchronize();
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("LDS ping-pong round trip: %.1f cyc\n", h[0] / 1000.0);
    ldslat<<<1, 64>>>(d); ldslat<<<1, 64>>>(d); hipDeviceSynchronize();
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("ds_read_b32 dependent latency: %.1f cyc\n", h[0] / 256.0);
    // clock: s_memtime vs s_memrealtime
    return 0;
}
