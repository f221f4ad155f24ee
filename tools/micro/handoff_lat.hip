// Hand-off latency between two workgroups through global memory: a ping-pong of one dword
// between workgroup 0 and workgroup P (P = 8: the same XCD under round-robin dispatch, P = 1: another XCD;
// each reports its XCC id), with relaxed atomic loads / stores at agent scope (what the lane fill's hand-off
// uses) or system scope, one lane polling.  Prints the one-way latency (half the round trip) in ns.
//
//     hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/handoff_lat.hip -o tools/micro/handoff_lat
#include <hip/hip_runtime.h>

#include <cstdio>

template <int SCOPE>
__device__ __forceinline__ unsigned ld(unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, SCOPE);
}
template <int SCOPE>
__device__ __forceinline__ void st(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, SCOPE);
}

template <int SCOPE>
__global__ void __launch_bounds__(64) pingpong(unsigned* flags, unsigned long long* out, int iters, int partner) {
    const int b = blockIdx.x;
    if (b != 0 && b != partner) return;
    if (threadIdx.x != 0) return;
    unsigned* ping = flags;       // written by 0
    unsigned* pong = flags + 64;  // written by the partner (another 256-byte line)
    const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20) & 15u;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long bound = 0;
    for (int i = 1; i <= iters && bound <= (1ull << 26); i++) {
        if (b == 0) {
            st<SCOPE>(ping, (unsigned)i);
            while (ld<SCOPE>(pong) != (unsigned)i)
                if (++bound > (1ull << 26)) break;
        } else {
            while (ld<SCOPE>(ping) != (unsigned)i)
                if (++bound > (1ull << 26)) break;
            st<SCOPE>(pong, (unsigned)i);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    out[b == 0 ? 0 : 1] = t1 - t0;
    out[b == 0 ? 2 : 3] = xcc;
}

template <int SCOPE>
static void run(const char* name, int partner) {
    unsigned* f;
    unsigned long long* o;
    (void)hipMalloc(&f, 4096);
    (void)hipMalloc(&o, 64);
    (void)hipMemset(f, 0, 4096);
    const int iters = 20000;
    hipLaunchKernelGGL(pingpong<SCOPE>, dim3(partner + 1), dim3(64), 0, 0, f, o, iters, partner);
    (void)hipDeviceSynchronize();
    unsigned long long h[4];
    (void)hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
    // s_memrealtime: 100 MHz
    printf("%-8s partner %d  xcc %llu -> %llu  one-way %.0f ns\n", name, partner, h[2], h[3],
           (double)h[0] * 10.0 / (2.0 * iters));
    (void)hipFree(f);
    (void)hipFree(o);
}

int main() {
    for (int partner : {8, 1, 16, 3}) {
        run<__HIP_MEMORY_SCOPE_AGENT>("agent", partner);
        run<__HIP_MEMORY_SCOPE_SYSTEM>("system", partner);
    }
    return 0;
}
