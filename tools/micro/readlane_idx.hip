#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out, const unsigned* idx, int n) {
    const int lane = threadIdx.x;
    const int v = 1000 + lane;
    for (int q = 0; q < n; q++) {
        unsigned s = __builtin_amdgcn_readfirstlane(idx[q]);
        unsigned r;
        asm volatile("v_readlane_b32 %0, %1, %2" : "=s"(r) : "v"(v), "s"(s));
        unsigned long long t = 0x0123456789abcdefull;
        unsigned long long x;
        asm volatile("s_lshr_b64 %0, %1, %2" : "=s"(x) : "s"(t), "s"(s));
        unsigned y;
        asm volatile("s_lshr_b32 %0, %1, %2" : "=s"(y) : "s"(0x89abcdefu), "s"(s));
        if (lane == 0) { out[3 * q] = r; out[3 * q + 1] = (unsigned)x; out[3 * q + 2] = y; }
    }
}
int main() {
    const unsigned h[8] = {5, 69, 133, 0x12345, 0x80000005u, 64, 0x7fffffc5u, 63};
    unsigned *di, *dout, ho[24];
    hipMalloc(&di, 32); hipMalloc(&dout, 96);
    hipMemcpy(di, h, 32, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dout, di, 8);
    hipMemcpy(ho, dout, 96, hipMemcpyDeviceToHost);
    for (int q = 0; q < 8; q++)
        printf("idx 0x%x: readlane -> %u (lane %u), lshr64 -> 0x%08x (expect low6 %u), lshr32 -> 0x%08x\n", h[q], ho[3*q], ho[3*q]-1000, ho[3*q+1], h[q] & 63, ho[3*q+2]);
    return 0;
}
